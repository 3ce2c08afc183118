#!/bin/bash
# A/B kernel timings: rocprofv3 kernel trace of a short bench run per library variant.
# Usage: scripts/ab_trace.sh TAG REGEX base VARIANT1 VARIANT2 ...   (variants/NAME/libtransmvs_hip.so)
TAG=$1; REGEX=$2; shift 2
cd "$GRAFT_REPO_ROOT" || exit 1
export TMPDIR=/tmp
for v in "$@"; do
  OUT=gpurun_out/$TAG/$v
  mkdir -p $OUT
  if [ "$v" = base ]; then unset TMVS_LIB_PATH; else export TMVS_LIB_PATH=$PWD/variants/$v/libtransmvs_hip.so; fi
  timeout -k 10 300 rocprofv3 --kernel-trace -T -d $OUT/trace -o run --output-format csv -- \
      python3 bench.py --steps 5 --warmup 2 --no-cpu-baseline --profile-steps 0 --e2e-steps 0 --train-steps 0 > $OUT/trace.log 2>&1 || exit $?
  python3 scripts/trace_table.py $OUT/trace/run_kernel_trace.csv > $OUT/trace_table.txt
  echo "== $v"
  grep -E "$REGEX" $OUT/trace_table.txt
done
