#!/bin/bash
# GPU box: the whole -m gpu suite, then smoke(). Usage: bash scripts/gpu/full_check.sh TAG
TAG=$1
cd "$GRAFT_REPO_ROOT" || exit 1
mkdir -p gpurun_out/$TAG
timeout -k 10 900 python -u -m pytest -x -v --timeout 300 --timeout-method thread tests -m gpu \
  > gpurun_out/$TAG/pytest_gpu.log 2>&1 || exit $?
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/$TAG/smoke.log 2>&1
