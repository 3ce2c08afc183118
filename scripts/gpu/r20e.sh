#!/bin/bash
# r20e: PMC passes over the fused conv11 + prob kernel (scripts/diag/dp_run.py drives tmvs_costregnet_wta)
cd "$GRAFT_REPO_ROOT" || exit 1
export TMPDIR=/tmp
export PMC_PROG="scripts/diag/dp_run.py 2"
bash scripts/pmc_kernel.sh r20e deconv_prob \
  "SQ_WAVES SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_VALU_MFMA_BUSY_CYCLES GRBM_GUI_ACTIVE" \
  "SQ_INSTS_VALU SQ_INSTS_MFMA SQ_INSTS_LDS SQ_INSTS_SALU SQ_INSTS_SMEM SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_LDS SQ_INSTS_VMEM_RD" \
  "SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE SQ_WAIT_INST_LDS SQ_ACTIVE_INST_VMEM SQ_INSTS_VMEM_WR SQ_ACTIVE_INST_SCA SQ_INST_CYCLES_SMEM" || exit $?
python3 scripts/diag/pmc_dump.py r20e > gpurun_out/r20e/pmc_dump.txt; cat gpurun_out/r20e/pmc_dump.txt
timeout -k 10 120 python scripts/diag/dp_run.py 10
TMVS_LIB_PATH=variants/nofuse/libtransmvs_hip.so timeout -k 10 120 python scripts/diag/dp_run.py 10
