#!/bin/bash
# r21f: C5 FeatureNet backward vs the oracle (new test)
cd "$GRAFT_REPO_ROOT" || exit 1
export TMPDIR=/tmp
mkdir -p gpurun_out/r21f
timeout -k 10 900 python -u -m pytest tests/test_gpu_train_c5_featurenet.py -x -v -s --timeout 600 --timeout-method thread \
  2>&1 | tee gpurun_out/r21f/pytest.log | grep -E "PASS|FAIL|Error|worst|oracle done|passed|failed"
