#!/bin/bash
# Measurement session on the GPU box: bench (with CPU baseline), rocprofv3 kernel-trace stats,
# and two PMC passes (FETCH_SIZE, WRITE_SIZE) for HBM traffic. Usage: scripts/profile_round.sh TAG
TAG=${1:-r01}
cd "$GRAFT_REPO_ROOT" || exit 1
export TMPDIR=/tmp
OUT=gpurun_out/$TAG
mkdir -p $OUT
timeout -k 10 400 python bench.py --steps 20 --warmup 5 > $OUT/bench.json 2> $OUT/bench.err || exit $?
tail -1 $OUT/bench.json
timeout -k 10 300 rocprofv3 --kernel-trace --stats -T -d $OUT/trace -o run --output-format csv -- \
    python3 bench.py --steps 5 --warmup 2 --no-cpu-baseline --e2e-steps 0 --train-steps 0 > $OUT/trace.log 2>&1 || exit $?
timeout -k 10 300 rocprofv3 --pmc FETCH_SIZE -T -d $OUT/pmc_fetch -o run --output-format csv -- \
    python3 bench.py --steps 2 --warmup 1 --no-cpu-baseline --profile-steps 0 --e2e-steps 0 --train-steps 0 --no-graph > $OUT/pmc_fetch.log 2>&1 || exit $?
timeout -k 10 300 rocprofv3 --pmc WRITE_SIZE -T -d $OUT/pmc_write -o run --output-format csv -- \
    python3 bench.py --steps 2 --warmup 1 --no-cpu-baseline --profile-steps 0 --e2e-steps 0 --train-steps 0 --no-graph > $OUT/pmc_write.log 2>&1 || exit $?
find $OUT -name "*.csv" | head -20
