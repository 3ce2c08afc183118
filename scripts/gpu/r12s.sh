#!/bin/bash
# r12s: conv5 (32->64 stride 2, direct) rows x output blocks per wave: 2x1 (product), 4x1, 2x2.
cd "$GRAFT_REPO_ROOT" || exit 1
bash scripts/ab_trace.sh r12s "conv3d_direct|total" base n4m1 n2m2 base n4m1 n2m2
