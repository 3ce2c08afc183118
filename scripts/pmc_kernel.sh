#!/bin/bash
# Per-kernel PMC passes (few counters each) over a short bench run.
# Usage: scripts/pmc_kernel.sh TAG KERNEL_REGEX "CTR1 CTR2" "CTR3 CTR4" ...
# PMC_PROG (optional) replaces the bench run, e.g. PMC_PROG="scripts/diag/featurenet_run.py 2".
TAG=$1; shift
REGEX=$1; shift
cd "$GRAFT_REPO_ROOT" || exit 1
export TMPDIR=/tmp
OUT=gpurun_out/$TAG
mkdir -p $OUT
i=0
for ctrs in "$@"; do
  i=$((i+1))
  timeout -k 10 240 rocprofv3 --pmc $ctrs --kernel-include-regex "$REGEX" -T -d $OUT/pmc_$i -o run \
      --output-format csv -- python3 ${PMC_PROG:-bench.py --steps 2 --warmup 1 --no-cpu-baseline --profile-steps 0 --e2e-steps 0 --train-steps 0 --no-graph} \
      > $OUT/pmc_$i.log 2>&1
  rc=$?
  echo "pass $i ($ctrs) rc=$rc"
  if [ $rc -ne 0 ]; then tail -5 $OUT/pmc_$i.log; fi
  if [ $rc -eq 124 ] || [ $rc -eq 137 ] || [ $rc -eq 134 ] || [ $rc -eq 139 ]; then exit $rc; fi
done
exit 0
