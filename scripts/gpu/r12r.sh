#!/bin/bash
# r12r: conv5 (32->64 stride 2, direct) with one output row per wave -- bitwise A/B vs two rows,
# kernel-trace A/B.
cd "$GRAFT_REPO_ROOT" || exit 1
mkdir -p gpurun_out/r12r
timeout -k 10 120 python scripts/diag/out_bits.py gpurun_out/r12r/base.npz > gpurun_out/r12r/bits.log 2>&1 || exit $?
TMVS_LIB_PATH=$PWD/variants/nbw2/libtransmvs_hip.so timeout -k 10 120 python scripts/diag/out_bits.py gpurun_out/r12r/nbw2.npz >> gpurun_out/r12r/bits.log 2>&1 || exit $?
python scripts/diag/out_bits.py --compare gpurun_out/r12r/base.npz gpurun_out/r12r/nbw2.npz >> gpurun_out/r12r/bits.log 2>&1
rm -f gpurun_out/r12r/*.npz
bash scripts/ab_trace.sh r12r "conv3d_direct|total" base nbw2 base nbw2
