#!/bin/bash
# r14f: where the FMT K/V partial's time goes: 1 / 2 tiles per wave, no linears, one tile per step
cd "$GRAFT_REPO_ROOT" || exit 1
O=gpurun_out/r14f
mkdir -p $O
export TMPDIR=/tmp
bash scripts/diag/ab_kernels.sh r14f/ab "fmt_kv" tpw1 tpw2 nomfma nt1 > $O/kv_ab.txt 2>&1
rc=$?
rm -rf $O/ab/*/
exit $rc
