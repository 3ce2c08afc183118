#!/bin/bash
# rocprofv3 kernel trace + stats of the FeatureNet forward (5 DTU views, scripts/diag/featurenet_run.py)
# -> gpurun_out/TAG/fn_kernel_stats.csv
TAG=$1
cd "$GRAFT_REPO_ROOT" || exit 1
O=$GRAFT_REPO_ROOT/gpurun_out/$TAG; mkdir -p $O
cd /tmp && export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d /tmp/fnprof -o fn --output-format csv -- python $GRAFT_REPO_ROOT/scripts/diag/featurenet_run.py 5 \
  > $O/fn_trace.log 2>&1 || exit $?
f=$(find /tmp/fnprof -name "*kernel_stats.csv" | head -1)
cp "$f" $O/fn_kernel_stats.csv && head -12 $O/fn_kernel_stats.csv | cut -d, -f1-4
