#!/bin/bash
# r14o: training-path GPU tests on the XCD-grouped weight-gradient grids
cd "$GRAFT_REPO_ROOT" || exit 1
mkdir -p gpurun_out/r14o
timeout -k 10 900 python -u -m pytest -x -v --timeout 300 --timeout-method thread tests/test_gpu_train.py \
  tests/test_gpu_train_ref.py tests/test_gpu_train_c5.py tests/test_gpu_featurenet.py -m gpu > gpurun_out/r14o/pytest.log 2>&1
