cd "$GRAFT_REPO_ROOT" || exit 1
export TMPDIR=/tmp
O=gpurun_out/crab; mkdir -p $O
timeout -k 10 300 python -u -m pytest tests/test_gpu_parity.py -q -x --timeout 120 --timeout-method thread > $O/pytest.log 2>&1; rc=$?
tail -1 $O/pytest.log; [ $rc -ne 0 ] && exit $rc
timeout -k 10 300 python bench.py --steps 30 --warmup 5 --no-cpu-baseline --e2e-steps 0 > $O/bench.json 2>/dev/null || exit $?
python -c "import json; d=json.loads(open('$O/bench.json').read().strip().splitlines()[-1]); print(d['value'], d['kernel_ms_per_depth_map'])"
timeout -k 10 300 rocprofv3 --kernel-trace --stats -T -d $O/trace -o run --output-format csv -- python3 bench.py --steps 5 --warmup 2 --no-cpu-baseline --e2e-steps 0 > $O/trace.log 2>&1 || exit $?
python scripts/trace_table.py $O/trace/run_kernel_trace.csv | grep -E "${AB_REGEX:-deconv|s2c8|total}"
