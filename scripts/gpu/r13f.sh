#!/bin/bash
# r13f: PMC of warp_dot_kernel (SQ instruction mix, waits, LDS, TA) vs the row-pair kernel (nodot)
cd "$GRAFT_REPO_ROOT" || exit 1
CTRS1="SQ_WAVE_CYCLES SQ_INSTS_VALU SQ_INSTS_SALU SQ_WAIT_INST_ANY SQ_WAIT_ANY SQ_ACTIVE_INST_ANY SQ_INSTS_VMEM_RD SQ_INSTS_LDS GRBM_GUI_ACTIVE"
CTRS2="TA_TA_BUSY_sum TA_ADDR_STALLED_BY_TC_CYCLES_sum GRBM_GUI_ACTIVE"
CTRS3="SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE SQ_WAIT_INST_LDS SQ_INSTS_SMEM SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_LDS GRBM_GUI_ACTIVE"
bash scripts/pmc_kernel.sh r13f_dot "warp_dot_kernel|warp_pair_kernel" "$CTRS1" "$CTRS2" "$CTRS3" || exit $?
TMVS_LIB_PATH=$PWD/variants/nodot/libtransmvs_hip.so bash scripts/pmc_kernel.sh r13f_pair "warp_dot_kernel|warp_pair_kernel" "$CTRS1" "$CTRS2" "$CTRS3" || exit $?
python3 scripts/pmc_report.py r13f_dot > gpurun_out/r13f_report.txt
python3 scripts/pmc_report.py r13f_pair >> gpurun_out/r13f_report.txt
bash scripts/ab_trace.sh r13f "warp_|total" base nodot || exit $?
timeout -k 10 300 python -u -m pytest -x -q --timeout 200 --timeout-method thread tests/test_gpu_parity.py -m gpu -k "warp" > gpurun_out/r13f_pytest_parity.log 2>&1
