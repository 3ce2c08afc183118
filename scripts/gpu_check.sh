#!/bin/bash
# GPU parity tests then (if no crash) the measurement session. Usage: scripts/gpu_check.sh TAG
TAG=${1:-dev}
cd "$GRAFT_REPO_ROOT" || exit 1
mkdir -p gpurun_out/$TAG
timeout -k 10 900 python -m pytest tests/ -m gpu -q -rA --timeout=300 > gpurun_out/$TAG/pytest_gpu.log 2>&1
rc=$?
echo "pytest rc=$rc"; grep -E "passed|failed|error" gpurun_out/$TAG/pytest_gpu.log | tail -3
if [ $rc -ne 0 ] && [ $rc -ne 1 ]; then exit $rc; fi
bash scripts/profile_round.sh $TAG
