#!/bin/bash
# Diagnostic PMC passes over a short bench run. Usage: scripts/pmc_diag.sh TAG
TAG=${1:-diag}
cd "$GRAFT_REPO_ROOT" || exit 1
export TMPDIR=/tmp
OUT=gpurun_out/$TAG
mkdir -p $OUT
timeout -k 10 120 rocprofv3 -L > $OUT/counters_list.txt 2>&1
echo "list rc=$?"
run_pass() {
  local name=$1; shift
  timeout -k 10 300 rocprofv3 --pmc "$@" -T -d $OUT/pmc_$name -o run --output-format csv -- \
      python3 bench.py --steps 2 --warmup 1 --no-cpu-baseline --profile-steps 0 > $OUT/pmc_$name.log 2>&1
  local rc=$?
  echo "pass $name rc=$rc"
  return $rc
}
run_pass busy SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_VALU_MFMA_BUSY_CYCLES SQ_INSTS_VALU SQ_INSTS_LDS SQ_WAVES GRBM_GUI_ACTIVE || exit $?
run_pass lds SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE SQ_WAIT_INST_LDS SQ_WAIT_ANY SQ_ACTIVE_INST_ANY SQ_INSTS_VMEM_RD
exit 0
