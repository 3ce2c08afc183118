#!/bin/bash
# r14d: the C5 full-size training test alone, with its flip / log-probability report
cd "$GRAFT_REPO_ROOT" || exit 1
mkdir -p gpurun_out/r14d
timeout -k 10 600 python -u -m pytest -x -v -s --timeout 500 --timeout-method thread tests/test_gpu_train_c5.py -m gpu \
  -k full_size_vs_oracle > gpurun_out/r14d/pytest_c5.log 2>&1
