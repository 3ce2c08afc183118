#!/bin/bash
# r13h: warp_dot_kernel variants (6 waves/SIMD base; 4 waves; pipelined; 8 rounds in flight) vs the
# row-pair kernel, then parity, then the C4 stage-1 flip attribution
cd "$GRAFT_REPO_ROOT" || exit 1
mkdir -p gpurun_out/r13h
timeout -k 10 300 python -u -m pytest -x -q --timeout 200 --timeout-method thread tests/test_gpu_parity.py -m gpu -k "warp" > gpurun_out/r13h/pytest_parity.log 2>&1 || exit $?
bash scripts/ab_trace.sh r13h "warp_|total" base w4 pipe nbl8 nodot || exit $?
timeout -k 10 900 python -u scripts/diag/stage1_flip.py gpurun_out/r13h/c4_stage1_flip.json > gpurun_out/r13h/c4_stage1_flip.log 2>&1
