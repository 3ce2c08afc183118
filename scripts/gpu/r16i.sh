#!/bin/bash
# r16i: tap-pair source layout A/B for the stage-2/3 warp (bitwise + time), training glue call sites
cd "$GRAFT_REPO_ROOT" || exit 1
O=gpurun_out/r16i; mkdir -p $O
timeout -k 10 200 python scripts/diag/warp_paired.py > $O/warp_paired.txt 2>&1 || exit $?
cat $O/warp_paired.txt
timeout -k 10 300 python scripts/diag/train_glue.py 60 > $O/train_glue.txt 2>&1 || exit $?
head -64 $O/train_glue.txt
