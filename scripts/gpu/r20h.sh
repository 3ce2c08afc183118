#!/bin/bash
# r20h: C4 full-size + view-sharded world-4 tests with the top-2 cap at 2e-3; warp kernels on coherent hypotheses
cd "$GRAFT_REPO_ROOT" || exit 1
export TMPDIR=/tmp
O=gpurun_out/r20h; mkdir -p $O
timeout -k 10 200 python scripts/diag/warp_coherent.py 20 --json $O/warp_coherent.json > $O/warp_coherent.log 2>&1 || exit $?
cat $O/warp_coherent.log
TMVS_REPORT_DIR=$O/fullsize timeout -k 10 600 python -u -m pytest tests/test_gpu_fullsize.py -k "c4" -v --timeout 400 \
  --timeout-method thread > $O/pytest_c4.log 2>&1; rc=$?
tail -6 $O/pytest_c4.log
exit $rc
