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
