#!/bin/bash
# r12u: deconv3d_lds on 1x4 input tiles for every depth (2x2 when the depth is even in the product) --
# bitwise A/B and kernel-trace A/B.
cd "$GRAFT_REPO_ROOT" || exit 1
mkdir -p gpurun_out/r12u
timeout -k 10 120 python scripts/diag/out_bits.py gpurun_out/r12u/base.npz > gpurun_out/r12u/bits.log 2>&1 || exit $?
TMVS_LIB_PATH=$PWD/variants/td1/libtransmvs_hip.so timeout -k 10 120 python scripts/diag/out_bits.py gpurun_out/r12u/td1.npz >> gpurun_out/r12u/bits.log 2>&1 || exit $?
python scripts/diag/out_bits.py --compare gpurun_out/r12u/base.npz gpurun_out/r12u/td1.npz >> gpurun_out/r12u/bits.log 2>&1
rm -f gpurun_out/r12u/*.npz
bash scripts/ab_trace.sh r12u "deconv3d_lds|total" base td1 base td1 || exit $?
