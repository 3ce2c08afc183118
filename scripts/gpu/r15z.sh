#!/bin/bash
# r15z: round-4 close measurement on the final build: bench + kernel trace + FETCH/WRITE passes
# (profile_round.sh), then a kernel trace of the C5 training step (graph replay)
cd "$GRAFT_REPO_ROOT" || exit 1
export TMPDIR=/tmp
bash scripts/profile_round.sh r15z || exit $?
O=gpurun_out/r15z
STEPS=3 timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $O/train_trace -o run --output-format csv -- python3 scripts/diag/train_step_prof.py > $O/train.log 2>&1
