#!/bin/bash
# pathway fork point with the two-event join: after the FMT vs after the stage-1 cost volume (3 alternations)
set -o pipefail
OUT0=gpurun_out/${1:-fork_join2}; mkdir -p $OUT0
timeout -k 10 300 python -u -m pytest -x -v --timeout 200 --timeout-method thread tests/test_gpu_batch.py -k layouts > $OUT0/pytest.log 2>&1 || { tail -30 $OUT0/pytest.log; exit 1; }
tail -2 $OUT0/pytest.log
OUT=gpurun_out/${1:-fork_join2}; mkdir -p $OUT
b() { timeout -k 10 300 python -u bench.py --steps 60 --warmup 10 --no-cpu-baseline --profile-steps 0 --e2e-steps 0 --train-steps 0 --batch2-steps 0 > $OUT/bench_$1.json 2> $OUT/bench_$1.err || return $?
  python3 -c "import json; d=json.loads(open('$OUT/bench_$1.json').read().strip().splitlines()[-1]); print('$1', d['value'], d['ms_per_step'], d['eager']['ms_per_step'])"; }
for r in 1 2 3; do
  TMVS_PATHWAY_FORK=fmt b fmt$r || exit $?
  TMVS_PATHWAY_FORK=warp b warp$r || exit $?
  TMVS_PATHWAY_FORK=fmt_late b late$r || exit $?
done
