#!/bin/bash
# stage-1 hypotheses on the FMT side stream vs in line (bitwise layouts test first), 3 alternations
set -o pipefail
OUT=gpurun_out/${1:-hyp1_ab}; mkdir -p $OUT
timeout -k 10 300 python -u -m pytest -x -v --timeout 200 --timeout-method thread tests/test_gpu_batch.py -k layouts > $OUT/pytest.log 2>&1 || { tail -30 $OUT/pytest.log; exit 1; }
tail -2 $OUT/pytest.log
b() { timeout -k 10 300 python -u bench.py --steps 60 --warmup 10 --no-cpu-baseline --profile-steps 0 --e2e-steps 0 --train-steps 0 --batch2-steps 0 > $OUT/bench_$1.json 2> $OUT/bench_$1.err || return $?
  python3 -c "import json; d=json.loads(open('$OUT/bench_$1.json').read().strip().splitlines()[-1]); print('$1', d['value'], d['ms_per_step'], d['eager']['ms_per_step'])"; }
for r in 1 2 3; do
  TMVS_HYP1_SIDE=0 b inline$r || exit $?
  TMVS_HYP1_SIDE=1 b side$r || exit $?
done
