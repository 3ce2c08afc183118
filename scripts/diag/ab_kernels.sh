#!/bin/bash
# A/B of library variants by rocprofv3 kernel trace of the bench's hot-path step: per-(kernel, grid)
# average durations matching REGEX for the default library and each variants/NAME/.
# Usage: scripts/diag/ab_kernels.sh TAG "substr1 substr2" NAME...
TAG=$1; PATS=$2; shift 2
cd "$GRAFT_REPO_ROOT" || exit 1
export TMPDIR=/tmp
OUT=gpurun_out/$TAG
mkdir -p $OUT
for v in default "$@"; do
  if [ "$v" = default ]; then unset TMVS_LIB_PATH; else export TMVS_LIB_PATH=variants/$v/libtransmvs_hip.so; fi
  timeout -k 10 200 rocprofv3 --kernel-trace -d $OUT/$v -o run -- python3 bench.py --steps 10 --warmup 3 \
      --no-cpu-baseline --e2e-steps 0 --train-steps 0 > $OUT/$v.log 2>&1 || exit $?
  echo "== $v $(grep "\"metric\"" $OUT/$v.log | tail -1 | cut -c1-160)"
  python3 scripts/diag/kernel_grid_times.py $OUT/$v/run_results.db $PATS
done
