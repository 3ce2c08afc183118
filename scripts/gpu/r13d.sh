#!/bin/bash
# r13d: warp_dot_kernel, list reads / loads / reference reads batched per view, vs the row-pair build
cd "$GRAFT_REPO_ROOT" || exit 1
mkdir -p gpurun_out/r13d
timeout -k 10 300 python -u -m pytest -x -q --timeout 200 --timeout-method thread tests/test_gpu_parity.py -m gpu -k "warp" > gpurun_out/r13d/pytest_parity.log 2>&1 || exit $?
bash scripts/ab_trace.sh r13d "warp_|total" base nodot base || exit $?
