#!/bin/bash
# rocprofv3 kernel trace + stats of the C5 training step (bench.py's train_depth_stages, graph replay):
# bash scripts/gpu/train_trace.sh TAG -> gpurun_out/TAG/train_kernel_stats.csv
TAG=$1
cd "$GRAFT_REPO_ROOT" || exit 1
O=$GRAFT_REPO_ROOT/gpurun_out/$TAG; mkdir -p $O
cd /tmp && export TMPDIR=/tmp
timeout -k 10 400 rocprofv3 --kernel-trace --stats -d /tmp/trprof -o tr --output-format csv -- python \
  $GRAFT_REPO_ROOT/bench.py --steps 1 --warmup 1 --no-cpu-baseline --e2e-steps 0 --train-steps 5 --profile-steps 0 \
  > $O/train_trace.log 2>&1 || exit $?
f=$(find /tmp/trprof -name "*kernel_stats.csv" | head -1)
cp "$f" $O/train_kernel_stats.csv && head -25 $O/train_kernel_stats.csv | cut -d, -f1-4
