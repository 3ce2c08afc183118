#!/bin/bash
# parity tests + one bench line (no profiling). Usage: scripts/gpu_quick.sh TAG
TAG=${1:-dev}
cd "$GRAFT_REPO_ROOT" || exit 1
mkdir -p gpurun_out/$TAG
timeout -k 10 900 python -m pytest tests/ -m gpu -q -rA --timeout=300 > gpurun_out/$TAG/pytest_gpu.log 2>&1
rc=$?
echo "pytest rc=$rc"; grep -E "^(FAILED|ERROR)|passed|failed" gpurun_out/$TAG/pytest_gpu.log | tail -8
if [ $rc -ne 0 ] && [ $rc -ne 1 ]; then exit $rc; fi
timeout -k 10 400 python bench.py --steps 20 --warmup 5 --no-cpu-baseline > gpurun_out/$TAG/bench.json 2> gpurun_out/$TAG/bench.err
rc=$?
python - "$TAG" <<'PY'
import json, sys
try:
    d = json.loads(open(f"gpurun_out/{sys.argv[1]}/bench.json").read().strip().splitlines()[-1])
    print("value", d["value"], "ms", d["ms_per_step"], {k: v for k, v in d["kernel_ms_per_depth_map"].items()})
    for k in d["roofline_kernels"]:
        print(k["kernel"], k["achieved"], k["unit"], k["frac"], k["per_stage_ms"])
except Exception as e:
    print("bench parse failed", e)
PY
exit $rc
