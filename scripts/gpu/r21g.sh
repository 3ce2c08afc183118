#!/bin/bash
# r21g: conditioning of C5 FeatureNet gradients (scripts/diag/c5_fnet_grad.py)
cd "$GRAFT_REPO_ROOT" || exit 1
export TMPDIR=/tmp
mkdir -p gpurun_out/r21g
timeout -k 10 900 python -u scripts/diag/c5_fnet_grad.py 0 2e-7 2e-6 2e-5 2>&1 | tee gpurun_out/r21g/c5_fnet_grad.txt
