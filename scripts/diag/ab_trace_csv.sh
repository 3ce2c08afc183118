#!/bin/bash
# A/B of library variants by a rocprofv3 kernel trace (CSV) of the bench's hot-path step, one trace table
# per variant (scripts/trace_table.py). Usage: scripts/diag/ab_trace_csv.sh TAG NAME...  ("default" = in-tree lib)
TAG=$1; shift
cd "$GRAFT_REPO_ROOT" || exit 1
export TMPDIR=/tmp
OUT=gpurun_out/$TAG
mkdir -p $OUT
for v in "$@"; do
  if [ "$v" = default ]; then unset TMVS_LIB_PATH; else export TMVS_LIB_PATH=variants/$v/libtransmvs_hip.so; fi
  timeout -k 10 240 rocprofv3 --kernel-trace -d $OUT/$v -o run --output-format csv -- python3 bench.py --steps 10 \
      --warmup 3 --no-cpu-baseline --e2e-steps 0 --train-steps 0 --batch2-steps 0 > $OUT/$v.log 2>&1
  rc=$?
  if [ $rc -ne 0 ]; then echo "== $v rc=$rc"; tail -3 $OUT/$v.log; exit $rc; fi
  f=$(find $OUT/$v -name "*kernel_trace.csv" | head -1)
  python3 scripts/trace_table.py $f > $OUT/trace_$v.txt
  echo "== $v $(grep '"metric"' $OUT/$v.log | tail -1 | cut -c60-140)"
  head -25 $OUT/trace_$v.txt
done
