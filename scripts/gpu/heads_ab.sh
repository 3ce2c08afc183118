#!/bin/bash
# forward() from images: FeatureNet's stage-2/3 heads serial vs on a side stream (bitwise test first), 3 alternations
set -o pipefail
OUT=gpurun_out/${1:-heads_ab}; mkdir -p $OUT
timeout -k 10 300 python -u -m pytest -x -v --timeout 200 --timeout-method thread tests/test_gpu_batch.py > $OUT/pytest.log 2>&1 || { tail -30 $OUT/pytest.log; exit 1; }
tail -2 $OUT/pytest.log
b() { timeout -k 10 300 python -u bench.py --steps 10 --warmup 3 --no-cpu-baseline --profile-steps 0 --e2e-steps 20 --train-steps 0 --batch2-steps 0 > $OUT/bench_$1.json 2> $OUT/bench_$1.err || return $?
  python3 -c "import json; d=json.loads(open('$OUT/bench_$1.json').read().strip().splitlines()[-1]); e=d['end_to_end']; print('$1', d['value'], 'e2e', e['depth_maps_per_s'], e['ms_per_depth_map'], e['featurenet_ms'])"; }
for r in 1 2 3; do
  TMVS_OVERLAP_HEADS=0 b serial$r || exit $?
  TMVS_OVERLAP_HEADS=1 b overlap$r || exit $?
done
