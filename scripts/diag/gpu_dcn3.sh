cd "$GRAFT_REPO_ROOT" || exit 1
timeout -k 10 300 python -u -m pytest tests/test_gpu_featurenet.py -q -x --timeout 120 --timeout-method thread 2>&1 | tail -1
for sd in 0 1.5; do
DCN_FUSED=1 DCN_OFFSET_STD=$sd timeout -k 10 120 python scripts/diag/dcn_time.py 2>&1 | grep us || exit 1
done
