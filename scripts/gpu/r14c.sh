#!/bin/bash
# r14c: the whole -m gpu suite + smoke (C4 cascade bound: moved pixels + 1 % of the footprint), full-size
# reports into gpurun_out/r14c/fullsize, then a bench line
cd "$GRAFT_REPO_ROOT" || exit 1
export TMVS_REPORT_DIR=$PWD/gpurun_out/r14c/fullsize
bash scripts/gpu/full_check.sh r14c || exit $?
timeout -k 10 400 python bench.py --steps 20 --warmup 5 > gpurun_out/r14c/bench.json 2> gpurun_out/r14c/bench.err
