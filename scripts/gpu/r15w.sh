#!/bin/bash
# r15w: the whole -m gpu suite + smoke on the round-4 final build (after the conv0 / prob tap-kernel DPP sums), full-size
# reports into gpurun_out/r15w/fullsize, then a bench line
cd "$GRAFT_REPO_ROOT" || exit 1
export TMVS_REPORT_DIR=$PWD/gpurun_out/r15w/fullsize
bash scripts/gpu/full_check.sh r15w || exit $?
timeout -k 10 400 python bench.py --steps 20 --warmup 5 > gpurun_out/r15w/bench.json 2> gpurun_out/r15w/bench.err
