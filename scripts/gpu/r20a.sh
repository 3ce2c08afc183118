#!/bin/bash
# r20a (round 6): conv5 K order A/B (tap-outer LDS = default, direct, chunk-outer), full-size parity incl.
# three C2 seeds and the multi-rank HIP view-sharded runs, chunk-order C2 seeds, bench, B=2 capture.
cd "$GRAFT_REPO_ROOT" || exit 1
export TMPDIR=/tmp
O=gpurun_out/r20a; mkdir -p $O
bash scripts/gpu/ab.sh r20a --layers conv5 c5direct c5chunk || exit $?
TMVS_REPORT_DIR=$O/fullsize timeout -k 10 900 python -u -m pytest tests/test_gpu_fullsize.py -v --timeout 400 \
  --timeout-method thread > $O/pytest_fullsize.log 2>&1; rc=$?
tail -15 $O/pytest_fullsize.log
[ $rc -eq 0 ] || [ $rc -eq 1 ] || exit $rc
TMVS_LIB_PATH=variants/c5chunk/libtransmvs_hip.so TMVS_REPORT_DIR=$O/fullsize_c5chunk timeout -k 10 400 \
  python -u -m pytest tests/test_gpu_fullsize.py -k c2_dtu -v --timeout 300 --timeout-method thread \
  > $O/pytest_c5chunk.log 2>&1; rc2=$?
tail -5 $O/pytest_c5chunk.log
[ $rc2 -eq 0 ] || [ $rc2 -eq 1 ] || exit $rc2
timeout -k 10 300 python bench.py > $O/bench.log 2>&1 || exit $?
tail -c 3000 $O/bench.log
timeout -k 10 300 python -u -m pytest tests/test_gpu_batch.py -v --timeout 250 --timeout-method thread \
  > $O/pytest_batch.log 2>&1; echo "batch rc=$?"
tail -5 $O/pytest_batch.log
exit $rc
