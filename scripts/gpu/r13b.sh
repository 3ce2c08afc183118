#!/bin/bash
# r13b: warp_dot_kernel (stages 2/3, dot first over unique taps): parity tests, output diff vs the
# row-pair build (nodot), kernel-trace A/B.
cd "$GRAFT_REPO_ROOT" || exit 1
mkdir -p gpurun_out/r13b
timeout -k 10 300 python -u -m pytest -x -v --timeout 200 --timeout-method thread tests/test_gpu_parity.py -m gpu -k "warp or e2e" > gpurun_out/r13b/pytest_parity.log 2>&1 || exit $?
timeout -k 10 120 python scripts/diag/out_bits.py gpurun_out/r13b/base.npz > gpurun_out/r13b/bits.log 2>&1 || exit $?
TMVS_LIB_PATH=$PWD/variants/nodot/libtransmvs_hip.so timeout -k 10 120 python scripts/diag/out_bits.py gpurun_out/r13b/nodot.npz >> gpurun_out/r13b/bits.log 2>&1 || exit $?
python scripts/diag/out_bits.py --compare gpurun_out/r13b/base.npz gpurun_out/r13b/nodot.npz >> gpurun_out/r13b/bits.log 2>&1
rm -f gpurun_out/r13b/*.npz
bash scripts/ab_trace.sh r13b "warp_|total" base nodot base nodot || exit $?
timeout -k 10 400 python -u -m pytest -x -v -s --timeout 350 --timeout-method thread tests/test_gpu_fullsize.py -m gpu -k c2 > gpurun_out/r13b/pytest_fullsize_c2.log 2>&1
