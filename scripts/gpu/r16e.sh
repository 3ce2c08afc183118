#!/bin/bash
# r16e: warp_corr address-unit accounting: instruction, TA, TCP and TD counters per
# warp kernel (stage 1 warp_corr_kernel C=32, stage 2/3 warp_pair_kernel C=16/8)
cd "$GRAFT_REPO_ROOT" || exit 1
bash scripts/pmc_kernel.sh r16e "warp_" \
  "SQ_WAVE_CYCLES SQ_INSTS_VMEM_RD SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_LDS SQ_WAIT_INST_ANY SQ_ACTIVE_INST_VMEM GRBM_GUI_ACTIVE" \
  "TA_TA_BUSY_sum TA_BUFFER_READ_WAVEFRONTS_sum GRBM_GUI_ACTIVE" \
  "TA_ADDR_STALLED_BY_TC_CYCLES_sum TA_DATA_STALLED_BY_TC_CYCLES_sum GRBM_GUI_ACTIVE" \
  "TCP_TOTAL_CACHE_ACCESSES_sum TCP_TCC_READ_REQ_sum GRBM_GUI_ACTIVE" \
  "TCP_TCP_TA_DATA_STALL_CYCLES_sum TCP_READ_TAGCONFLICT_STALL_CYCLES_sum GRBM_GUI_ACTIVE" \
  "TD_TD_BUSY_sum TD_TC_STALL_sum GRBM_GUI_ACTIVE" || exit $?
python scripts/diag/pmc_dump.py r16e > gpurun_out/r16e/dump.txt
cat gpurun_out/r16e/dump.txt
# CostRegNet level-1 / full-resolution kernels: instruction mix and LDS waits
bash scripts/pmc_kernel.sh r16e_cr "conv3d_c16|conv3d_s2c8|deconv3d_c8|prob_wta|conv0_kernel" \
  "SQ_WAVE_CYCLES SQ_INSTS_MFMA SQ_INSTS_VALU SQ_INSTS_LDS SQ_WAIT_INST_LDS SQ_WAIT_INST_ANY SQ_ACTIVE_INST_LDS GRBM_GUI_ACTIVE" \
  "SQ_VALU_MFMA_BUSY_CYCLES SQ_INSTS_VMEM_RD SQ_INSTS_VMEM_WR SQ_ACTIVE_INST_VMEM SQ_INST_CYCLES_VMEM SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE GRBM_GUI_ACTIVE" || exit $?
python scripts/diag/pmc_dump.py r16e_cr > gpurun_out/r16e_cr/dump.txt
cat gpurun_out/r16e_cr/dump.txt
