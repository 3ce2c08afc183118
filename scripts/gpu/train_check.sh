#!/bin/bash
# GPU box: training parity tests, then the bench's training timing. Usage: bash scripts/gpu/train_check.sh TAG
TAG=$1
cd "$GRAFT_REPO_ROOT" || exit 1
mkdir -p gpurun_out/$TAG
timeout -k 10 500 python -u -m pytest -x -q --timeout 200 --timeout-method thread tests/test_gpu_train.py \
  tests/test_gpu_train_ref.py tests/test_gpu_featurenet.py > gpurun_out/$TAG/pytest.log 2>&1 || exit $?
timeout -k 10 300 python bench.py --steps 3 --warmup 1 --no-cpu-baseline --e2e-steps 0 --train-steps 3 \
  --profile-steps 1 > gpurun_out/$TAG/bench.json 2> gpurun_out/$TAG/bench.err
