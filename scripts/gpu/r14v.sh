#!/bin/bash
# r14v: the whole -m gpu suite + smoke on the round-4 final build (training kernels changed since r14c), full-size
# reports into gpurun_out/r14v/fullsize, then a bench line
cd "$GRAFT_REPO_ROOT" || exit 1
export TMVS_REPORT_DIR=$PWD/gpurun_out/r14v/fullsize
bash scripts/gpu/full_check.sh r14v || exit $?
timeout -k 10 400 python bench.py --steps 20 --warmup 5 > gpurun_out/r14v/bench.json 2> gpurun_out/r14v/bench.err
