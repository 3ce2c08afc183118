#!/bin/bash
# r12t: conv5 2x2 tiling on the stage-2/3 grids -- bitwise A/B vs the 2x1 build, kernel-trace A/B,
# then the GPU parity/full-size tests.
cd "$GRAFT_REPO_ROOT" || exit 1
mkdir -p gpurun_out/r12t
timeout -k 10 120 python scripts/diag/out_bits.py gpurun_out/r12t/base.npz > gpurun_out/r12t/bits.log 2>&1 || exit $?
TMVS_LIB_PATH=$PWD/variants/c5prev/libtransmvs_hip.so timeout -k 10 120 python scripts/diag/out_bits.py gpurun_out/r12t/c5prev.npz >> gpurun_out/r12t/bits.log 2>&1 || exit $?
python scripts/diag/out_bits.py --compare gpurun_out/r12t/base.npz gpurun_out/r12t/c5prev.npz >> gpurun_out/r12t/bits.log 2>&1
rm -f gpurun_out/r12t/*.npz
bash scripts/ab_trace.sh r12t "conv3d_direct|total" base c5prev base c5prev || exit $?
timeout -k 10 400 python -u -m pytest -x -q --timeout 300 --timeout-method thread tests/test_gpu_parity.py tests/test_gpu_fullsize.py tests/test_gpu_train.py -m gpu > gpurun_out/r12t/pytest.log 2>&1
