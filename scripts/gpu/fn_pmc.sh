#!/bin/bash
# PMC passes over the FeatureNet forward (DCN, 3x3 and trunk kernels): bash scripts/gpu/fn_pmc.sh TAG
TAG=$1
cd "$GRAFT_REPO_ROOT" || exit 1
PMC_PROG="scripts/diag/featurenet_run.py 1" bash scripts/pmc_kernel.sh $TAG "dcn_window|conv3x3_window|conv2d_bn_relu" \
  "SQ_WAVE_CYCLES SQ_INSTS_VALU SQ_VALU_MFMA_BUSY_CYCLES SQ_WAIT_INST_ANY SQ_WAIT_ANY SQ_ACTIVE_INST_ANY SQ_INSTS_MFMA GRBM_GUI_ACTIVE" \
  "SQ_INSTS_LDS SQ_WAIT_INST_LDS SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_LDS SQ_BUSY_CYCLES GRBM_GUI_ACTIVE" \
  || exit $?
python scripts/diag/pmc_dump.py $TAG > gpurun_out/$TAG/pmc_dump.txt && head -60 gpurun_out/$TAG/pmc_dump.txt
