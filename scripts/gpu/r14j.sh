#!/bin/bash
# r14j: DCN weight gradient with the offsets / mask logits loaded one chunk ahead of the gathers
# (BPRE) vs BROW only: bitwise dx / d offset-mask / dW, kernel trace of tmvs_dcn_backward
cd "$GRAFT_REPO_ROOT" || exit 1
O=gpurun_out/r14j
mkdir -p $O
export TMPDIR=/tmp
timeout -k 10 120 python scripts/diag/dcn_bwd_bits.py $O/new.npz > $O/bits.log 2>&1 &&
TMVS_LIB_PATH=variants/dcnw_nopre/libtransmvs_hip.so timeout -k 10 120 python scripts/diag/dcn_bwd_bits.py $O/old.npz >> $O/bits.log 2>&1 &&
python scripts/diag/dcn_bwd_bits.py --compare $O/old.npz $O/new.npz >> $O/bits.log 2>&1 &&
rm -f $O/old.npz $O/new.npz || exit 1
for v in default dcnw_nopre default dcnw_nopre; do
  if [ "$v" = default ]; then unset TMVS_LIB_PATH; else export TMVS_LIB_PATH=variants/$v/libtransmvs_hip.so; fi
  timeout -k 10 120 rocprofv3 --kernel-trace --stats -d $O/$v -o run -- python3 scripts/diag/dcn_bwd_kernels.py > $O/$v.log 2>&1 || exit $?
  echo "== $v" >> $O/summary.txt
  python3 scripts/diag/kernel_grid_times.py $O/$v/run_results.db dcn >> $O/summary.txt
  rm -rf $O/$v
done
