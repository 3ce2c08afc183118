#!/bin/bash
# r15x: the whole -m gpu suite + smoke on the round-4 final build (round-4 close: LayerNorm and small weight-gradient changes), full-size
# reports into gpurun_out/r15x/fullsize, then a bench line
cd "$GRAFT_REPO_ROOT" || exit 1
export TMVS_REPORT_DIR=$PWD/gpurun_out/r15x/fullsize
bash scripts/gpu/full_check.sh r15x || exit $?
timeout -k 10 400 python bench.py --steps 20 --warmup 5 > gpurun_out/r15x/bench.json 2> gpurun_out/r15x/bench.err
