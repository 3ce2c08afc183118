#!/bin/bash
# r16f: warp_corr address-unit accounting (r16e) + the training step's torch glue call sites
cd "$GRAFT_REPO_ROOT" || exit 1
mkdir -p gpurun_out/r16f
timeout -k 10 300 python scripts/diag/train_glue.py 60 > gpurun_out/r16f/train_glue.txt 2>&1 || exit $?
head -70 gpurun_out/r16f/train_glue.txt
bash scripts/gpu/r16e.sh
