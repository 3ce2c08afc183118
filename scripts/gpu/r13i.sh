#!/bin/bash
# r13i: warp_dot variants A/B + parity; branch-free elu in the FMT (bitwise + timing vs elubr);
# new GPU tests (distributed, C5 full size); C4 stage-1 flip attribution
cd "$GRAFT_REPO_ROOT" || exit 1
mkdir -p gpurun_out/r13i
timeout -k 10 300 python -u -m pytest -x -q --timeout 200 --timeout-method thread tests/test_gpu_parity.py -m gpu -k "warp or fmt" > gpurun_out/r13i/pytest_parity.log 2>&1 || exit $?
timeout -k 10 120 python scripts/diag/out_bits.py gpurun_out/r13i/base.npz > gpurun_out/r13i/bits.log 2>&1 || exit $?
TMVS_LIB_PATH=$PWD/variants/elubr/libtransmvs_hip.so timeout -k 10 120 python scripts/diag/out_bits.py gpurun_out/r13i/elubr.npz >> gpurun_out/r13i/bits.log 2>&1 || exit $?
python scripts/diag/out_bits.py --compare gpurun_out/r13i/base.npz gpurun_out/r13i/elubr.npz >> gpurun_out/r13i/bits.log 2>&1
rm -f gpurun_out/r13i/*.npz
bash scripts/ab_trace.sh r13i "warp_|fmt_|total" base elubr w4 pipe nbl8 nodot || exit $?
timeout -k 10 600 python -u -m pytest -x -v -s --timeout 500 --timeout-method thread tests/test_gpu_distributed.py tests/test_gpu_train_c5.py -m gpu > gpurun_out/r13i/pytest_new.log 2>&1
timeout -k 10 900 python -u scripts/diag/stage1_flip.py gpurun_out/r13i/c4_stage1_flip.json > gpurun_out/r13i/c4_stage1_flip.log 2>&1
export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats -T -d gpurun_out/r13i/train_full -o run --output-format csv -- python3 scripts/diag/train_prof.py full 5 graph > gpurun_out/r13i/train_full.log 2>&1
python3 scripts/diag/stats_table.py gpurun_out/r13i/train_full/run_kernel_stats.csv > gpurun_out/r13i/train_full_kernels.txt 2>&1
