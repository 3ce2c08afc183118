#!/bin/bash
# Round-2 measurement session: bench + kernel trace + FETCH/WRITE passes (scripts/profile_round.sh) and a
# per-kernel PMC table of the hot-path kernels (TA, VALU, MFMA busy, LDS, L1, occupancy).
TAG=${1:-r05f}
cd "$GRAFT_REPO_ROOT" || exit 1
bash scripts/profile_round.sh $TAG || exit $?
python scripts/pmc_traffic.py $TAG > gpurun_out/$TAG/pmc_traffic.txt || exit $?
bash scripts/pmc_kernel.sh ${TAG}k "warp_corr_kernel|warp_pair_kernel|conv0_kernel|prob_kernel|conv3d_|deconv3d_|fmt_apply_kernel|fmt_kv_partial_kernel|pathway" \
  "FETCH_SIZE GRBM_GUI_ACTIVE" \
  "WRITE_SIZE GRBM_GUI_ACTIVE" \
  "TA_TA_BUSY_sum TA_ADDR_STALLED_BY_TC_CYCLES_sum GRBM_GUI_ACTIVE" \
  "SQ_WAVE_CYCLES SQ_INSTS_VALU SQ_VALU_MFMA_BUSY_CYCLES SQ_WAIT_INST_ANY SQ_WAIT_ANY SQ_INSTS_VMEM_RD GRBM_GUI_ACTIVE" \
  "SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE SQ_INSTS_LDS GRBM_GUI_ACTIVE" || exit $?
python scripts/pmc_report.py ${TAG}k > gpurun_out/${TAG}k/pmc_table.txt
cat gpurun_out/${TAG}k/pmc_table.txt
