#!/bin/bash
# r14q: kernel trace of the C5 training step (bench.train_timing, graph replay) on the current build
cd "$GRAFT_REPO_ROOT" || exit 1
O=gpurun_out/r14q
mkdir -p $O
export TMPDIR=/tmp
STEPS=3 timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $O/trace -o run --output-format csv -- python3 scripts/diag/train_step_prof.py > $O/train.log 2>&1
