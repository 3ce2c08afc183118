#!/bin/bash
# split FMT A/B: off / on / on with a high-priority FMT side stream, alternating; bench kernel trace of the split
set -o pipefail
OUT=gpurun_out/${1:-fmt_split2}; mkdir -p $OUT
export TMPDIR=/tmp
b() { timeout -k 10 300 python -u bench.py --steps 30 --warmup 5 --no-cpu-baseline --e2e-steps 0 --train-steps 0 --batch2-steps 0 > $OUT/bench_$1.json 2> $OUT/bench_$1.err || return $?
  python3 -c "import json; d=json.loads(open('$OUT/bench_$1.json').read().strip().splitlines()[-1]); print('$1', d['value'], d['ms_per_step'], d['call_ms_overlapped']['tmvs_fmt_forward'])"; }
for r in 1 2; do
  TMVS_SPLIT_FMT=0 b off$r || exit $?
  TMVS_SPLIT_FMT=1 b on$r || exit $?

done
timeout -k 10 300 rocprofv3 --kernel-trace -T -d $OUT/trace -o run --output-format csv -- python3 bench.py --steps 5 --warmup 2 --no-cpu-baseline --profile-steps 0 --e2e-steps 0 --train-steps 0 --batch2-steps 0 > $OUT/trace.log 2>&1 || exit $?
python3 scripts/trace_table.py $OUT/trace/run_kernel_trace.csv > $OUT/trace_table.txt
python3 scripts/trace_overlap.py $OUT/trace/run_kernel_trace.csv > $OUT/trace_overlap.txt 2>&1 || true
grep -E "fmt_|total" $OUT/trace_table.txt
