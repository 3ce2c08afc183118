#!/bin/bash
# r17e: conv3d_lds B fragments read one tap ahead (bpf) and one-MFMA schedule groups interleaving the
# accumulator chains (sgb): per-layer A/B vs the round-start build, parity tests, in-graph trace A/B
cd "$GRAFT_REPO_ROOT" || exit 1
O=gpurun_out/r17e; mkdir -p $O
L=conv3,conv4,conv6
TMVS_LIB_PATH=variants/old/libtransmvs_hip.so timeout -k 10 200 python scripts/diag/costreg_layers.py --save /tmp/old.pt --layers $L > $O/layers_old.txt 2>&1 || exit $?
timeout -k 10 200 python scripts/diag/costreg_layers.py --compare /tmp/old.pt --layers $L > $O/layers_new.txt 2>&1 || exit $?
for v in bpf0 sgb0 both0; do
  TMVS_LIB_PATH=variants/$v/libtransmvs_hip.so timeout -k 10 200 python scripts/diag/costreg_layers.py --compare /tmp/old.pt --layers $L > $O/layers_$v.txt 2>&1 || exit $?
done
tail -n 4 $O/layers_*.txt
timeout -k 10 400 python -u -m pytest tests/test_gpu_parity.py -x -q --timeout 200 --timeout-method thread > $O/pytest_parity.log 2>&1; rc=$?
tail -3 $O/pytest_parity.log; [ $rc -eq 0 ] || exit $rc
bash scripts/diag/ab_trace_csv.sh r17e_ab default both0 || exit $?
