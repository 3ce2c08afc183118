#!/bin/bash
# r15v: the whole -m gpu suite + smoke on the round-4 final build (round-4 training batch, BN fusion, PixelwiseNet DPP), full-size
# reports into gpurun_out/r15v/fullsize, then a bench line
cd "$GRAFT_REPO_ROOT" || exit 1
export TMVS_REPORT_DIR=$PWD/gpurun_out/r15v/fullsize
bash scripts/gpu/full_check.sh r15v || exit $?
timeout -k 10 400 python bench.py --steps 20 --warmup 5 > gpurun_out/r15v/bench.json 2> gpurun_out/r15v/bench.err
