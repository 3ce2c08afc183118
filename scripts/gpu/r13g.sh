#!/bin/bash
# r13g: warp_dot_kernel (slimmer geometry) PMC + timing vs the row-pair kernel, parity; then the C4
# stage-1 flip attribution (fp64 through FMT / cost volume / CostRegNet, reference thread spread)
cd "$GRAFT_REPO_ROOT" || exit 1
bash scripts/gpu/r13f.sh || exit $?
timeout -k 10 900 python -u scripts/diag/stage1_flip.py gpurun_out/r13g_c4_stage1_flip.json > gpurun_out/r13g_c4_stage1_flip.log 2>&1
