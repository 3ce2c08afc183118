#!/bin/bash
# Training-side check after a warp-backward change: the warp backward GPU tests, the C5 training step
# timings (bench.py train leg), and a kernel trace of the from-features step (graph replay).
# Usage: bash scripts/gpu/train_warp_check.sh TAG [pytest -k expression]
TAG=$1; K=${2:-"warp_corr or planes or depth_stages"}
cd "$GRAFT_REPO_ROOT" || exit 1
export TMPDIR=/tmp
OUT=gpurun_out/$TAG
mkdir -p $OUT
timeout -k 10 600 python -u -m pytest -x -v --timeout 300 --timeout-method thread ${FILES:-tests/test_gpu_train.py} -k "$K" \
  > $OUT/pytest.log 2>&1 || { tail -30 $OUT/pytest.log; exit 1; }
tail -3 $OUT/pytest.log
bash scripts/diag/ab_train.sh > $OUT/train_times.txt 2>&1 || exit $?
cat $OUT/train_times.txt
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $OUT/tp -o run --output-format csv -- \
  python3 scripts/diag/train_prof.py features 4 graph > $OUT/tp.log 2>&1 || exit $?
python3 scripts/diag/stats_table.py $OUT/tp/run_kernel_stats.csv 2>/dev/null | head -40 > $OUT/features_kernels.txt
head -25 $OUT/features_kernels.txt
