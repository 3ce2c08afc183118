#!/bin/bash
# stream-layout A/B on one box: pathway on the main stream / forked after stage 1's cost volume / forked after
# the FMT, each without and with the reference view's pathway on the FMT side stream (bitwise test first)
set -o pipefail
OUT=gpurun_out/${1:-pathway_fork}; mkdir -p $OUT
timeout -k 10 300 python -u -m pytest -x -v --timeout 200 --timeout-method thread tests/test_gpu_batch.py -k layouts > $OUT/pytest.log 2>&1 || { tail -30 $OUT/pytest.log; exit 1; }
tail -2 $OUT/pytest.log
b() { timeout -k 10 300 python -u bench.py --steps 60 --warmup 10 --no-cpu-baseline --profile-steps 0 --e2e-steps 0 --train-steps 0 --batch2-steps 0 $2 > $OUT/bench_$1.json 2> $OUT/bench_$1.err || return $?
  python3 -c "import json; d=json.loads(open('$OUT/bench_$1.json').read().strip().splitlines()[-1]); print('$1', d['value'], d['ms_per_step'], d['eager']['ms_per_step'])"; }
for r in 1 2 3; do
  b main$r --no-overlap || exit $?
  TMVS_PATHWAY_FORK=warp b warp$r || exit $?
  TMVS_PATHWAY_FORK=fmt b fmt$r || exit $?
  TMVS_REF_PATHWAY=1 b refw$r || exit $?
  TMVS_REF_PATHWAY=1 TMVS_PATHWAY_FORK=fmt b reff$r || exit $?
done
