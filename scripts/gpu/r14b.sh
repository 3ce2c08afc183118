#!/bin/bash
# r14b: the whole -m gpu suite + smoke on the round-4 build (prob walk one plane ahead), full-size
# parity reports into gpurun_out/r14b/fullsize, then a bench line
cd "$GRAFT_REPO_ROOT" || exit 1
export TMVS_REPORT_DIR=$PWD/gpurun_out/r14b/fullsize
bash scripts/gpu/full_check.sh r14b || exit $?
timeout -k 10 400 python bench.py --steps 20 --warmup 5 > gpurun_out/r14b/bench.json 2> gpurun_out/r14b/bench.err
