#!/bin/bash
# r16h: the whole GPU suite + smoke on the current build, the bench, then the warp / CostRegNet PMC passes and the
# training-step glue call sites (r16f)
cd "$GRAFT_REPO_ROOT" || exit 1
export TMVS_REPORT_DIR=gpurun_out/r16h/fullsize
bash scripts/gpu/full_check.sh r16h || { tail -30 gpurun_out/r16h/pytest_gpu.log; exit 1; }
tail -3 gpurun_out/r16h/pytest_gpu.log; tail -2 gpurun_out/r16h/smoke.log
timeout -k 10 400 python bench.py --steps 20 --warmup 5 > gpurun_out/r16h/bench.json 2> gpurun_out/r16h/bench.err || exit $?
tail -1 gpurun_out/r16h/bench.json | cut -c1-300
bash scripts/gpu/r16f.sh
