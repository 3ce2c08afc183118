#!/bin/bash
# FeatureNet kernel stats per library variant (rocprofv3 --stats over scripts/diag/featurenet_run.py):
# bash scripts/gpu/fn_kstats.sh TAG VARIANT... ("default" = the in-tree library)
TAG=$1; shift
cd "$GRAFT_REPO_ROOT" || exit 1
O=$GRAFT_REPO_ROOT/gpurun_out/$TAG; mkdir -p $O
cd /tmp && export TMPDIR=/tmp
for v in "$@"; do
  L=""; [ "$v" != default ] && L=$GRAFT_REPO_ROOT/variants/$v/libtransmvs_hip.so
  TMVS_LIB_PATH=$L timeout -k 10 300 rocprofv3 --kernel-trace --stats -d /tmp/fk_$v -o fk --output-format csv -- \
    python $GRAFT_REPO_ROOT/scripts/diag/featurenet_run.py 5 > $O/fk_$v.log 2>&1 || exit $?
  f=$(find /tmp/fk_$v -name "*kernel_stats.csv" | head -1); cp "$f" $O/fk_${v}_stats.csv
  echo "== $v"; cut -d, -f1-4 $O/fk_${v}_stats.csv | grep -v copyBuffer | cut -c1-120 | head -14
done
