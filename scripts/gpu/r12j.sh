#!/bin/bash
# r12j: direct stride-2 conv with one-step register prefetch -- bitwise A/B vs the nested-loop form,
# parity + full-size tests, kernel-trace A/B; then the inter-kernel gap traces (scripts/gpu/gaps.sh).
cd "$GRAFT_REPO_ROOT" || exit 1
mkdir -p gpurun_out/r12j
timeout -k 10 120 python scripts/diag/out_bits.py gpurun_out/r12j/base.npz > gpurun_out/r12j/bits.log 2>&1 || exit $?
TMVS_LIB_PATH=$PWD/variants/noprefetch/libtransmvs_hip.so timeout -k 10 120 python scripts/diag/out_bits.py gpurun_out/r12j/noprefetch.npz >> gpurun_out/r12j/bits.log 2>&1 || exit $?
python scripts/diag/out_bits.py --compare gpurun_out/r12j/base.npz gpurun_out/r12j/noprefetch.npz >> gpurun_out/r12j/bits.log 2>&1
rm -f gpurun_out/r12j/*.npz
timeout -k 10 400 python -u -m pytest -x -q --timeout 300 --timeout-method thread tests/test_gpu_parity.py \
  tests/test_gpu_fullsize.py -m gpu > gpurun_out/r12j/pytest.log 2>&1 || exit $?
bash scripts/ab_trace.sh r12j "conv3d_direct|total" base noprefetch base noprefetch || exit $?
bash scripts/gpu/gaps.sh r12i
