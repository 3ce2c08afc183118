#!/bin/bash
# r17d: PMC of the coarse CostRegNet kernels (conv3d_lds / conv3d_direct / deconv3d_lds): instruction mix,
# wait cycles, MFMA busy, address-unit load -- why conv6 / conv5 / deconv7 sit at 22-30 % of their MFMA floor
cd "$GRAFT_REPO_ROOT" || exit 1
bash scripts/pmc_kernel.sh r17d "conv3d_lds|conv3d_direct|deconv3d_lds" \
  "SQ_WAVE_CYCLES SQ_INSTS_MFMA SQ_INSTS_VALU SQ_INSTS_LDS SQ_WAIT_INST_LDS SQ_WAIT_INST_ANY SQ_ACTIVE_INST_LDS GRBM_GUI_ACTIVE" \
  "SQ_VALU_MFMA_BUSY_CYCLES SQ_INSTS_VMEM_RD SQ_INSTS_VMEM_WR SQ_ACTIVE_INST_VMEM SQ_INST_CYCLES_VMEM SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE GRBM_GUI_ACTIVE" \
  "SQ_WAIT_ANY SQ_BUSY_CYCLES SQ_WAVES SQ_ACTIVE_INST_ANY SQ_ACTIVE_INST_VALU SQ_INSTS_SALU GRBM_GUI_ACTIVE" \
  "TA_TA_BUSY_sum TA_BUFFER_READ_WAVEFRONTS_sum GRBM_GUI_ACTIVE" \
  "TA_ADDR_STALLED_BY_TC_CYCLES_sum TA_DATA_STALLED_BY_TC_CYCLES_sum GRBM_GUI_ACTIVE" || exit $?
python scripts/diag/pmc_dump.py r17d > gpurun_out/r17d/dump.txt
cat gpurun_out/r17d/dump.txt
