#!/bin/bash
# r20f: timing ablations of the fused conv11 + prob kernel (wrong results by construction): kernel stats per variant
cd "$GRAFT_REPO_ROOT" || exit 1
export TMPDIR=/tmp
O=gpurun_out/r20f; mkdir -p $O
for v in default abl1 abl2 abl4 nofuse; do
  if [ "$v" = default ]; then unset TMVS_LIB_PATH; else export TMVS_LIB_PATH=variants/$v/libtransmvs_hip.so; fi
  timeout -k 10 120 rocprofv3 --kernel-trace --stats -d $O/$v -o run --output-format csv -- python3 scripts/diag/dp_run.py 5 \
    > $O/$v.log 2>&1 || exit $?
  f=$(find $O/$v -name "*kernel_stats.csv" | head -1)
  echo "== $v"; grep -E "deconv_prob|deconv3d_c8|prob_wta|softmax_wta" $f | cut -d, -f1-4
done
