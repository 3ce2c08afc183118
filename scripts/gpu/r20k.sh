#!/bin/bash
# r20k: pathway16_mfma_kernel phase ablations (timing only; wrong outputs by construction)
# 1 no coarse 1x1 reduction, 2 no lateral loads, 4 no MFMA conv, 8 no halo build
cd "$GRAFT_REPO_ROOT" || exit 1
export TMPDIR=/tmp
bash scripts/diag/ab_trace_csv.sh r20k_trace default pwabl1 pwabl2 pwabl4 pwabl8
