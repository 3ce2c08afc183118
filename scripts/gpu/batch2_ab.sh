#!/bin/bash
# B = 2 concurrent graphs and the B = 1 step: FMT split on / off, one or two side streams (3 alternations)
set -o pipefail
OUT=gpurun_out/${1:-batch2_ab}; mkdir -p $OUT
timeout -k 10 300 python -u -m pytest -x -v --timeout 200 --timeout-method thread tests/test_gpu_batch.py > $OUT/pytest.log 2>&1 || { tail -30 $OUT/pytest.log; exit 1; }
tail -2 $OUT/pytest.log
b() { timeout -k 10 300 python -u bench.py --steps 40 --warmup 10 --no-cpu-baseline --profile-steps 0 --e2e-steps 0 --train-steps 0 --batch2-steps 40 > $OUT/bench_$1.json 2> $OUT/bench_$1.err || return $?
  python3 -c "import json; d=json.loads(open('$OUT/bench_$1.json').read().strip().splitlines()[-1]); print('$1', d['value'], d['ms_per_step'], 'b2', d['batch2_concurrent']['depth_maps_per_s'])"; }
for r in 1 2 3; do
  TMVS_SPLIT_FMT=0 b nosplit$r || exit $?
  b split$r || exit $?
  TMVS_ONE_SIDE=1 b oneside$r || exit $?
  TMVS_PW_JOIN2=1 b join2_$r || exit $?
done
