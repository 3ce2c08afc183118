#!/bin/bash
# r12p: per-kernel PMC passes at the round-close build (same counter sets as round_measure.sh).
cd "$GRAFT_REPO_ROOT" || exit 1
bash scripts/pmc_kernel.sh r12p "warp_corr_kernel|warp_pair_kernel|conv0_kernel|conv3d_|deconv3d_|prob_|fmt_apply|fmt_kv_partial|pathway" \
  "SQ_WAVE_CYCLES SQ_INSTS_VALU SQ_VALU_MFMA_BUSY_CYCLES SQ_WAIT_INST_ANY SQ_WAIT_ANY SQ_ACTIVE_INST_ANY SQ_INSTS_VMEM_RD SQ_INSTS_VMEM_WR GRBM_GUI_ACTIVE" \
  "TA_TA_BUSY_sum TA_ADDR_STALLED_BY_TC_CYCLES_sum GRBM_GUI_ACTIVE" \
  "FETCH_SIZE GRBM_GUI_ACTIVE" "WRITE_SIZE GRBM_GUI_ACTIVE" \
  "SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE SQ_INSTS_LDS SQ_WAIT_INST_LDS GRBM_GUI_ACTIVE"
