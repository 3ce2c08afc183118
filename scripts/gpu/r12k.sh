#!/bin/bash
# r12k: stride-2 16/32-channel convs on the LDS-staged kernel -- bitwise A/B vs the direct kernel,
# parity + full-size + training tests, kernel-trace A/B (direct, 32->64 with 4 blocks per wave).
cd "$GRAFT_REPO_ROOT" || exit 1
mkdir -p gpurun_out/r12k
timeout -k 10 120 python scripts/diag/out_bits.py gpurun_out/r12k/base.npz > gpurun_out/r12k/bits.log 2>&1 || exit $?
TMVS_LIB_PATH=$PWD/variants/direct/libtransmvs_hip.so timeout -k 10 120 python scripts/diag/out_bits.py gpurun_out/r12k/direct.npz >> gpurun_out/r12k/bits.log 2>&1 || exit $?
python scripts/diag/out_bits.py --compare gpurun_out/r12k/base.npz gpurun_out/r12k/direct.npz >> gpurun_out/r12k/bits.log 2>&1
rm -f gpurun_out/r12k/*.npz
timeout -k 10 400 python -u -m pytest -x -q --timeout 300 --timeout-method thread tests/test_gpu_parity.py \
  tests/test_gpu_fullsize.py tests/test_gpu_train.py -m gpu > gpurun_out/r12k/pytest.log 2>&1 || exit $?
bash scripts/ab_trace.sh r12k "conv3d_direct|conv3d_lds|total" base direct mbb4 base direct mbb4

