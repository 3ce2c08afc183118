#!/bin/bash
# rocprofv3 kernel trace of a short bench run + per-(kernel, grid) mean durations.
# Usage: scripts/gpu_trace.sh TAG
TAG=${1:-trace}
cd "$GRAFT_REPO_ROOT" || exit 1
export TMPDIR=/tmp
OUT=gpurun_out/$TAG
mkdir -p $OUT
timeout -k 10 300 rocprofv3 --kernel-trace --stats -T -d $OUT/trace -o run --output-format csv -- \
    python3 bench.py --steps 5 --warmup 2 --no-cpu-baseline --profile-steps 0 > $OUT/trace.log 2>&1 || exit $?
python3 scripts/trace_table.py $OUT/trace/run_kernel_trace.csv | tee $OUT/trace_table.txt
