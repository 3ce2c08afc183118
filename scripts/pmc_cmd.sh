#!/bin/bash
# PMC passes (one rocprofv3 run each) over an arbitrary python command, filtered to one kernel.
# Usage: scripts/pmc_cmd.sh TAG KERNEL_REGEX "python args" "CTR1 CTR2" "CTR3" ...
TAG=$1; shift
REGEX=$1; shift
CMD=$1; shift
cd "$GRAFT_REPO_ROOT" || exit 1
export TMPDIR=/tmp
OUT=gpurun_out/$TAG
mkdir -p $OUT
i=0
for ctrs in "$@"; do
  i=$((i+1))
  timeout -k 10 240 rocprofv3 --pmc $ctrs --kernel-include-regex "$REGEX" -T -d $OUT/pmc_$i -o run \
      --output-format csv -- python3 $CMD > $OUT/pmc_$i.log 2>&1
  rc=$?
  echo "pass $i ($ctrs) rc=$rc"
  if [ $rc -ne 0 ]; then tail -5 $OUT/pmc_$i.log; exit $rc; fi
done
exit 0
