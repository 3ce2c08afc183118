#!/bin/bash
# r17h: conv6 wave split in the product (1,2,4,4); conv4 / conv3 wave-split and conv5 (direct) tilings A/B,
# bitwise vs the product; parity tests; in-graph trace vs the round-start build
cd "$GRAFT_REPO_ROOT" || exit 1
O=gpurun_out/r17h; mkdir -p $O
L=conv3,conv4,conv5,conv6
timeout -k 10 200 python scripts/diag/costreg_layers.py --save /tmp/base.pt --layers $L > $O/layers_base.txt 2>&1 || exit $?
for v in c4a c4b c4c c3a c5a c5b c5c; do
  TMVS_LIB_PATH=variants/$v/libtransmvs_hip.so timeout -k 10 200 python scripts/diag/costreg_layers.py --compare /tmp/base.pt --layers $L > $O/layers_$v.txt 2>&1 || exit $?
done
tail -n 4 $O/layers_*.txt
timeout -k 10 400 python -u -m pytest tests/test_gpu_parity.py tests/test_gpu_fullsize.py -x -q --timeout 300 --timeout-method thread > $O/pytest.log 2>&1; rc=$?
tail -3 $O/pytest.log; [ $rc -eq 0 ] || exit $rc
bash scripts/diag/ab_trace_csv.sh r17h_ab default old || exit $?
