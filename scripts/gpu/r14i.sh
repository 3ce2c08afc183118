#!/bin/bash
# r14i: conv2 (conv3d_c16_kernel) tile 4x4 (NBW 4) and scheduling-group A/Bs, kernel trace of the bench step
cd "$GRAFT_REPO_ROOT" || exit 1
O=gpurun_out/r14i
mkdir -p $O
export TMPDIR=/tmp
bash scripts/diag/ab_kernels.sh r14i/ab "conv3d_c16" c16_4x4 c16_sb3 c16_sb27 default > $O/c16_ab.txt 2>&1
rc=$?
rm -rf $O/ab/*/
exit $rc
