#!/bin/bash
# Inter-kernel gaps of one step: kernel traces of the graph-replayed step with and without the
# pathway side stream, and of eager launches.
cd "$GRAFT_REPO_ROOT" || exit 1
export TMPDIR=/tmp
OUT=gpurun_out/$1
mkdir -p $OUT
for cfg in "graph:" "nooverlap:--no-overlap" "eager:--no-graph"; do
  name=${cfg%%:*}; flags=${cfg#*:}
  timeout -k 10 300 rocprofv3 --kernel-trace -T -d $OUT/$name -o run --output-format csv -- \
    python3 bench.py --steps 5 --warmup 2 --no-cpu-baseline --profile-steps 0 --e2e-steps 0 --train-steps 0 $flags \
    > $OUT/$name.log 2>&1 || exit $?
  tail -1 $OUT/$name.log | cut -c1-120
done
