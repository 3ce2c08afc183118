#!/bin/bash
# r16a: round-5 start: GPU suite + smoke + bench on the round-4 build (baseline for this round)
cd "$GRAFT_REPO_ROOT" || exit 1
bash scripts/gpu/full_check.sh r16a || exit $?
timeout -k 10 400 python bench.py --steps 20 --warmup 5 > gpurun_out/r16a/bench.json 2> gpurun_out/r16a/bench.err || exit $?
tail -1 gpurun_out/r16a/bench.json | cut -c1-400
