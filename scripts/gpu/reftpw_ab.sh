#!/bin/bash
# tiles per wave of the reference view's applies in the split FMT: occupancy-sized (base) vs 2 / 4 / 8
set -o pipefail
OUT=gpurun_out/${1:-reftpw}; mkdir -p $OUT
b() { timeout -k 10 300 python -u bench.py --steps 60 --warmup 10 --no-cpu-baseline --profile-steps 0 --e2e-steps 0 --train-steps 0 --batch2-steps 0 > $OUT/bench_$1.json 2> $OUT/bench_$1.err || return $?
  python3 -c "import json; d=json.loads(open('$OUT/bench_$1.json').read().strip().splitlines()[-1]); print('$1', d['value'], d['ms_per_step'])"; }
timeout -k 10 300 python -u -m pytest -x -v --timeout 200 --timeout-method thread tests/test_gpu_batch.py -k layouts > $OUT/pytest.log 2>&1 || { tail -30 $OUT/pytest.log; exit 1; }
tail -2 $OUT/pytest.log
for r in 1 2 3; do
  b base$r || exit $?
  for t in 2 4 8; do TMVS_LIB_PATH=variants/reftpw$t/libtransmvs_hip.so b tpw${t}_$r || exit $?; done
done
for t in 0 4; do
  TMVS_LIB_PATH=$([ $t = 0 ] || echo variants/reftpw$t/libtransmvs_hip.so) timeout -k 10 120 python -u scripts/diag/fmt_time.py 20 2>&1 | grep ^fmt
done
