#!/bin/bash
# split FMT A/B on one box: off / on (chain-first order) / on (layer-by-layer order), 4 alternations
set -o pipefail
OUT=gpurun_out/${1:-fmt_split3}; mkdir -p $OUT
b() { timeout -k 10 300 python -u bench.py --steps 60 --warmup 10 --no-cpu-baseline --profile-steps 0 --e2e-steps 0 --train-steps 0 --batch2-steps 0 > $OUT/bench_$1.json 2> $OUT/bench_$1.err || return $?
  python3 -c "import json; d=json.loads(open('$OUT/bench_$1.json').read().strip().splitlines()[-1]); print('$1', d['value'], d['ms_per_step'], d['eager']['ms_per_step'])"; }
for r in 1 2 3 4; do
  TMVS_SPLIT_FMT=0 b off$r || exit $?
  TMVS_SPLIT_FMT=1 b on0_$r || exit $?
  TMVS_SPLIT_FMT=1 TMVS_LIB_PATH=variants/order1/libtransmvs_hip.so b on1_$r || exit $?
done
