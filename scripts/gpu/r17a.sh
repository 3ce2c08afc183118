#!/bin/bash
# r17a: branch-free MFMA loads (buffer OOB zeros) + late tile fetch in conv3d_lds, one-step prefetch in
# conv3d_direct. Per-layer A/B (bitwise vs the previous build "old"), parity tests, in-graph trace A/B.
cd "$GRAFT_REPO_ROOT" || exit 1
O=gpurun_out/r17a; mkdir -p $O
TMVS_LIB_PATH=variants/old/libtransmvs_hip.so timeout -k 10 200 python scripts/diag/costreg_layers.py --save /tmp/old.pt > $O/layers_old.txt 2>&1 || exit $?
timeout -k 10 200 python scripts/diag/costreg_layers.py --compare /tmp/old.pt > $O/layers_new.txt 2>&1 || exit $?
for v in early dir0; do
  TMVS_LIB_PATH=variants/$v/libtransmvs_hip.so timeout -k 10 200 python scripts/diag/costreg_layers.py --compare /tmp/old.pt > $O/layers_$v.txt 2>&1 || exit $?
done
tail -n 4 $O/layers_*.txt
timeout -k 10 400 python -u -m pytest tests/test_gpu_parity.py -x -q --timeout 200 --timeout-method thread > $O/pytest_parity.log 2>&1; rc=$?
tail -3 $O/pytest_parity.log; [ $rc -eq 0 ] || exit $rc
bash scripts/diag/ab_trace_csv.sh r17a_ab default old || exit $?
