#!/bin/bash
# r13e: warp_dot_kernel pipelined one view ahead, direct slots for pixels without a window
cd "$GRAFT_REPO_ROOT" || exit 1
mkdir -p gpurun_out/r13e
timeout -k 10 300 python -u -m pytest -x -q --timeout 200 --timeout-method thread tests/test_gpu_parity.py -m gpu -k "warp" > gpurun_out/r13e/pytest_parity.log 2>&1 || exit $?
bash scripts/ab_trace.sh r13e "warp_|total" base nodot base || exit $?
