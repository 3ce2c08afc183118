#!/bin/bash
# Kernel trace of the bench step for the window path: default library and variants/NAME (TMVS_WARP_WINDOW=1).
TAG=$1; shift
cd "$GRAFT_REPO_ROOT" || exit 1
export TMPDIR=/tmp
OUT=gpurun_out/$TAG
mkdir -p $OUT
for v in base "$@"; do
  if [ "$v" = base ]; then unset TMVS_LIB_PATH; else export TMVS_LIB_PATH=$PWD/variants/$v/libtransmvs_hip.so; fi
  timeout -k 10 300 rocprofv3 --kernel-trace -d $OUT/$v -o run --output-format csv -- \
    python3 bench.py --steps 5 --warmup 2 --no-cpu-baseline --profile-steps 0 --e2e-steps 0 --train-steps 0 \
    > $OUT/$v.log 2>&1 || { tail -20 $OUT/$v.log; exit 1; }
  python3 scripts/trace_table.py $OUT/$v/run_kernel_trace.csv > $OUT/$v.txt
  echo "== $v"; grep -E "warp_win|pw_agg|warp_corr_kernel" $OUT/$v.txt
done
