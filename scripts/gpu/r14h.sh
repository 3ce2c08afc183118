#!/bin/bash
# r14h: where tmvs_dcn_backward's data kernel spends its time: kernel trace of the product and of three
# ablation builds (no fixed-point conversion / no LDS atomics / no dcol FMAs; timing only)
cd "$GRAFT_REPO_ROOT" || exit 1
O=gpurun_out/r14h
mkdir -p $O
export TMPDIR=/tmp
for v in default ab_nocvt ab_noatom ab_nodcol; do
  if [ "$v" = default ]; then unset TMVS_LIB_PATH; else export TMVS_LIB_PATH=variants/$v/libtransmvs_hip.so; fi
  timeout -k 10 120 rocprofv3 --kernel-trace --stats -d $O/$v -o run -- python3 scripts/diag/dcn_bwd_kernels.py > $O/$v.log 2>&1 || exit $?
  echo "== $v" >> $O/summary.txt
  python3 scripts/diag/kernel_grid_times.py $O/$v/run_results.db dcn >> $O/summary.txt
done
rm -rf $O/*/
