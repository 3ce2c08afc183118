#!/bin/bash
# r20g: the whole GPU suite (full-size parity with three C2 seeds, multi-rank HIP view sharding, B=2 capture) + bench
cd "$GRAFT_REPO_ROOT" || exit 1
export TMPDIR=/tmp
O=gpurun_out/r20g; mkdir -p $O
TMVS_REPORT_DIR=$O/fullsize timeout -k 10 1000 python -u -m pytest tests -m gpu -v --timeout 400 --timeout-method thread \
  > $O/pytest_gpu.log 2>&1; rc=$?
tail -12 $O/pytest_gpu.log
[ $rc -eq 0 ] || [ $rc -eq 1 ] || exit $rc
timeout -k 10 300 python bench.py > $O/bench.log 2>&1 || exit $?
tail -c 1500 $O/bench.log
exit $rc
