#!/bin/bash
# GPU box: inference parity tests, then a rocprofv3 kernel trace of a short bench (no training, no
# e2e). Usage: bash scripts/gpu/parity_prof.sh TAG
TAG=$1
cd "$GRAFT_REPO_ROOT" || exit 1
export TMPDIR=/tmp
mkdir -p gpurun_out/$TAG
timeout -k 10 300 python -u -m pytest -x -q --timeout 200 --timeout-method thread tests/test_gpu_parity.py \
  > gpurun_out/$TAG/pytest.log 2>&1 || exit $?
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d gpurun_out/$TAG/prof -o run -- python3 bench.py --steps 10 \
  --warmup 3 --no-cpu-baseline --e2e-steps 0 --train-steps 0 > gpurun_out/$TAG/bench.json 2> gpurun_out/$TAG/bench.err
