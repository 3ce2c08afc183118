#!/bin/bash
# Stage-1 LDS-window warp (tmvs_warp_corr_ws) vs warp_corr_kernel: the warp parity tests, then a kernel
# trace of the bench step with TMVS_WARP_WINDOW=0 / 1. Usage: bash scripts/gpu/warp_window_ab.sh TAG [pytest -k]
TAG=$1; K=${2:-"warp or e2e or golden or stage"}
cd "$GRAFT_REPO_ROOT" || exit 1
export TMPDIR=/tmp
OUT=gpurun_out/$TAG
mkdir -p $OUT
timeout -k 10 600 python -u -m pytest -x -v --timeout 300 --timeout-method thread tests/test_gpu_parity.py -k "$K" \
  > $OUT/parity.log 2>&1 || { tail -40 $OUT/parity.log; exit 1; }
tail -2 $OUT/parity.log
for e in 0 1; do
  TMVS_WARP_WINDOW=$e timeout -k 10 300 rocprofv3 --kernel-trace -d $OUT/w$e -o run --output-format csv -- \
    python3 bench.py --steps 5 --warmup 2 --no-cpu-baseline --profile-steps 0 --e2e-steps 0 --train-steps 0 \
    > $OUT/w$e.log 2>&1 || { tail -20 $OUT/w$e.log; exit 1; }
  python3 scripts/trace_table.py $OUT/w$e/run_kernel_trace.csv > $OUT/w$e.txt
  echo "== TMVS_WARP_WINDOW=$e $(grep '"metric"' $OUT/w$e.log | python3 -c "import json,sys; d=json.loads(sys.stdin.read()); print(d['value'], d['abs_depth_l1_vs_ref']['stage3_mean_abs_mm'], d['abs_depth_l1_vs_ref']['per_stage']['stage1'])")"
  grep -E "warp|pw_agg|total" $OUT/w$e.txt
done
