#!/bin/bash
# r13a: warp_pair pixel-major rounds (base) vs plane-major rounds (oldmap): bitwise A/B of the
# hot path's outputs, then kernel-trace A/B (two alternating reps).
cd "$GRAFT_REPO_ROOT" || exit 1
mkdir -p gpurun_out/r13a
timeout -k 10 120 python scripts/diag/out_bits.py gpurun_out/r13a/base.npz > gpurun_out/r13a/bits.log 2>&1 || exit $?
TMVS_LIB_PATH=$PWD/variants/oldmap/libtransmvs_hip.so timeout -k 10 120 python scripts/diag/out_bits.py gpurun_out/r13a/oldmap.npz >> gpurun_out/r13a/bits.log 2>&1 || exit $?
python scripts/diag/out_bits.py --compare gpurun_out/r13a/base.npz gpurun_out/r13a/oldmap.npz >> gpurun_out/r13a/bits.log 2>&1
rm -f gpurun_out/r13a/*.npz
bash scripts/ab_trace.sh r13a "warp_|total" base oldmap || exit $?
bash scripts/ab_trace.sh r13a_2 "warp_|total" base oldmap || exit $?
