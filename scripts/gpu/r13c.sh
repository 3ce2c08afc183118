#!/bin/bash
# r13c: warp_dot_kernel with all load rounds of a view in flight (NB=8) / NB=4, vs the row-pair build
cd "$GRAFT_REPO_ROOT" || exit 1
mkdir -p gpurun_out/r13c
timeout -k 10 300 python -u -m pytest -x -q --timeout 200 --timeout-method thread tests/test_gpu_parity.py -m gpu -k "warp" > gpurun_out/r13c/pytest_parity.log 2>&1 || exit $?
bash scripts/ab_trace.sh r13c "warp_|total" base nb4 nodot base || exit $?
