#!/bin/bash
# r12f: parity/full-size/training GPU tests on the product build, bitwise A/B of the K/V butterfly
# (DPP vs ds_bpermute), kernel-trace A/B of the K/V butterfly and the stage-3 plane unroll.
cd "$GRAFT_REPO_ROOT" || exit 1
mkdir -p gpurun_out/r12f
timeout -k 10 120 python scripts/diag/out_bits.py gpurun_out/r12f/base.npz > gpurun_out/r12f/bits.log 2>&1 || exit $?
TMVS_LIB_PATH=$PWD/variants/kvshfl/libtransmvs_hip.so timeout -k 10 120 python scripts/diag/out_bits.py gpurun_out/r12f/kvshfl.npz >> gpurun_out/r12f/bits.log 2>&1 || exit $?
python scripts/diag/out_bits.py --compare gpurun_out/r12f/base.npz gpurun_out/r12f/kvshfl.npz >> gpurun_out/r12f/bits.log 2>&1
rm -f gpurun_out/r12f/*.npz
timeout -k 10 400 python -u -m pytest -x -q --timeout 300 --timeout-method thread tests/test_gpu_parity.py \
  tests/test_gpu_fullsize.py tests/test_gpu_train.py -m gpu > gpurun_out/r12f/pytest.log 2>&1 || exit $?
bash scripts/ab_trace.sh r12f "warp_pair|fmt_kv|s2c8|total" base kvshfl junroll2 base kvshfl junroll2
