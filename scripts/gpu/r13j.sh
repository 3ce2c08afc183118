#!/bin/bash
# r13j: the whole -m gpu suite (+ smoke) on the reverted warp / FMT build with the new tests, full-size
# parity reports into gpurun_out/r13j/fullsize, then a bench line
cd "$GRAFT_REPO_ROOT" || exit 1
export TMVS_REPORT_DIR=$PWD/gpurun_out/r13j/fullsize
bash scripts/gpu/full_check.sh r13j || exit $?
timeout -k 10 400 python bench.py --steps 20 --warmup 5 > gpurun_out/r13j/bench.json 2> gpurun_out/r13j/bench.err
