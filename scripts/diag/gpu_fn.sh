cd "$GRAFT_REPO_ROOT" || exit 1
export TMPDIR=/tmp
O=gpurun_out/fn2; mkdir -p $O
timeout -k 10 300 python -u -m pytest tests/test_gpu_featurenet.py tests/test_gpu_parity.py -q -x --timeout 120 --timeout-method thread > $O/pytest.log 2>&1; rc=$?
tail -3 $O/pytest.log; [ $rc -ne 0 ] && exit $rc
timeout -k 10 300 python scripts/diag/e2e_time.py > $O/e2e.txt 2>&1 || exit $?
grep featurenet $O/e2e.txt
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $O/fn -o fn --output-format csv -- python3 scripts/diag/featurenet_run.py 5 > $O/fn.log 2>&1 || exit $?
python scripts/diag/stats_table.py $(find $O/fn -name "*kernel_stats.csv" | head -1) 25
