#!/bin/bash
# split FMT: bitwise tests, standalone timings, and the bench step with / without the split (kernel traces)
set -o pipefail
OUT=gpurun_out/${1:-fmt_split}; mkdir -p $OUT
export TMPDIR=/tmp
timeout -k 10 300 python -u -m pytest -x -v --timeout 120 --timeout-method thread tests/test_gpu_parity.py -k "fmt" > $OUT/pytest.log 2>&1 || { tail -30 $OUT/pytest.log; exit 1; }
tail -3 $OUT/pytest.log
timeout -k 10 120 python -u scripts/diag/fmt_time.py 40 > $OUT/fmt_time.txt 2>&1 || exit $?
grep "^fmt" $OUT/fmt_time.txt
for s in 0 1 0 1; do
  TMVS_SPLIT_FMT=$s timeout -k 10 300 python -u bench.py --steps 20 --warmup 5 --no-cpu-baseline --e2e-steps 0 --train-steps 0 --batch2-steps 0 > $OUT/bench_split$s.json 2> $OUT/bench_split$s.err || exit $?
  python3 -c "import json,sys; d=json.loads(open('$OUT/bench_split$s.json').read().strip().splitlines()[-1]); print('split', $s, d['value'], d['ms_per_step'], d.get('call_ms_overlapped',{}).get('tmvs_fmt_forward'), d['abs_depth_l1_vs_ref']['stage3_mean_abs_mm'])"
done
