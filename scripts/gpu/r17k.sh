#!/bin/bash
# r17k: conv5 through the wave-split LDS kernel in the product (other K order): the full GPU suite
# (parity, full-size cascades, training, C5) and the bench trace
cd "$GRAFT_REPO_ROOT" || exit 1
O=gpurun_out/r17k; mkdir -p $O
timeout -k 10 1000 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > $O/pytest_gpu.log 2>&1; rc=$?
tail -5 $O/pytest_gpu.log; [ $rc -eq 0 ] || exit $rc
bash scripts/diag/ab_trace_csv.sh r17k_ab default old || exit $?
