#!/bin/bash
# r21t: the full GPU suite and smoke on the final hot-path build
cd "$GRAFT_REPO_ROOT" || exit 1
export TMPDIR=/tmp
mkdir -p gpurun_out/r21
timeout -k 10 1000 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > gpurun_out/r21/pytest_gpu.log 2>&1; rc=$?
tail -3 gpurun_out/r21/pytest_gpu.log
[ $rc -eq 0 ] || exit $rc
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke(); print('smoke ok')" > gpurun_out/r21/smoke.log 2>&1 || { tail -5 gpurun_out/r21/smoke.log; exit 1; }
tail -2 gpurun_out/r21/smoke.log
