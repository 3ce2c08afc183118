#!/bin/bash
# warp_corr parity tests + one bench line + rocprofv3 kernel stats. Usage: scripts/gpu_warp.sh TAG
TAG=${1:-dev}
cd "$GRAFT_REPO_ROOT" || exit 1
export TMPDIR=/tmp
OUT=gpurun_out/$TAG
mkdir -p $OUT
timeout -k 10 600 python -u -m pytest tests/test_gpu_parity.py -m gpu -x -q -rA --timeout 240 --timeout-method thread \
    -k "warp or e2e" > $OUT/pytest_warp.log 2>&1
rc=$?
echo "pytest rc=$rc"; grep -E "^(FAILED|ERROR)|passed|failed" $OUT/pytest_warp.log | tail -8
if [ $rc -ne 0 ] && [ $rc -ne 1 ]; then exit $rc; fi
timeout -k 10 300 python bench.py --steps 20 --warmup 5 --no-cpu-baseline > $OUT/bench.json 2> $OUT/bench.err || exit $?
python - "$OUT" <<'PY'
import json, sys
d = json.loads(open(f"{sys.argv[1]}/bench.json").read().strip().splitlines()[-1])
print("value", d["value"], "ms", d["ms_per_step"], d["kernel_ms_per_depth_map"])
for k in d["roofline_kernels"]:
    print(k["kernel"], k["achieved"], k["unit"], k["frac"], k["per_stage_ms"])
PY
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $OUT/trace -o run --output-format csv -- \
    python3 bench.py --steps 5 --warmup 2 --no-cpu-baseline --profile-steps 0 > $OUT/trace.log 2>&1 || exit $?
f=$(find $OUT/trace -name "*kernel_stats.csv" | head -1); head -25 "$f" | cut -c1-200
