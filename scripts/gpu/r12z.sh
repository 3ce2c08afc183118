#!/bin/bash
# r12z (round-3 close): conv3 on the LDS kernel bitwise vs the direct kernel, then the whole GPU suite
# + smoke, then the round measurement (bench with CPU baseline, kernel trace, FETCH/WRITE passes).
cd "$GRAFT_REPO_ROOT" || exit 1
mkdir -p gpurun_out/r12z
timeout -k 10 120 python scripts/diag/out_bits.py gpurun_out/r12z/base.npz > gpurun_out/r12z/bits.log 2>&1 || exit $?
TMVS_LIB_PATH=$PWD/variants/direct/libtransmvs_hip.so timeout -k 10 120 python scripts/diag/out_bits.py gpurun_out/r12z/direct.npz >> gpurun_out/r12z/bits.log 2>&1 || exit $?
python scripts/diag/out_bits.py --compare gpurun_out/r12z/base.npz gpurun_out/r12z/direct.npz >> gpurun_out/r12z/bits.log 2>&1
rm -f gpurun_out/r12z/*.npz
bash scripts/gpu/full_check.sh r12z || exit $?
bash scripts/profile_round.sh r12z
