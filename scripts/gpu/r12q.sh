#!/bin/bash
# r12q: stride-2 LDS tiles stored parity-split (even then odd columns per row) -- bitwise A/B vs the
# interleaved layout, parity/full-size/training tests, kernel-trace A/B.
cd "$GRAFT_REPO_ROOT" || exit 1
mkdir -p gpurun_out/r12q
timeout -k 10 120 python scripts/diag/out_bits.py gpurun_out/r12q/base.npz > gpurun_out/r12q/bits.log 2>&1 || exit $?
TMVS_LIB_PATH=$PWD/variants/nopar/libtransmvs_hip.so timeout -k 10 120 python scripts/diag/out_bits.py gpurun_out/r12q/nopar.npz >> gpurun_out/r12q/bits.log 2>&1 || exit $?
python scripts/diag/out_bits.py --compare gpurun_out/r12q/base.npz gpurun_out/r12q/nopar.npz >> gpurun_out/r12q/bits.log 2>&1
rm -f gpurun_out/r12q/*.npz
timeout -k 10 400 python -u -m pytest -x -q --timeout 300 --timeout-method thread tests/test_gpu_parity.py tests/test_gpu_fullsize.py tests/test_gpu_train.py -m gpu > gpurun_out/r12q/pytest.log 2>&1 || exit $?
bash scripts/ab_trace.sh r12q "conv3d_lds|total" base nopar base nopar
