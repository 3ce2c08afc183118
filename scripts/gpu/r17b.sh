#!/bin/bash
# r17b: deconv3d_lds LDS-fragment pipelining + batched skip reads; FMT token prefetch made effective
# (unconditional, two buffers in the apply, uniform loop, SGPR salt). Bits vs the round-start build
# ("old"), per-layer deconv A/B, in-graph trace A/B, parity tests.
cd "$GRAFT_REPO_ROOT" || exit 1
O=gpurun_out/r17b; mkdir -p $O
timeout -k 10 200 python scripts/diag/out_bits.py /tmp/new.npz > $O/bits_new.log 2>&1 || exit $?
TMVS_LIB_PATH=variants/old/libtransmvs_hip.so timeout -k 10 200 python scripts/diag/out_bits.py /tmp/old.npz > $O/bits_old.log 2>&1 || exit $?
python scripts/diag/out_bits.py --compare /tmp/old.npz /tmp/new.npz > $O/bits_compare.txt 2>&1; tail -2 $O/bits_compare.txt
TMVS_LIB_PATH=variants/old/libtransmvs_hip.so timeout -k 10 200 python scripts/diag/costreg_layers.py --save /tmp/old.pt --layers conv7,conv9 > $O/layers_old.txt 2>&1 || exit $?
timeout -k 10 200 python scripts/diag/costreg_layers.py --compare /tmp/old.pt --layers conv7,conv9 > $O/layers_new.txt 2>&1 || exit $?
TMVS_LIB_PATH=variants/dpipe0/libtransmvs_hip.so timeout -k 10 200 python scripts/diag/costreg_layers.py --compare /tmp/old.pt --layers conv7,conv9 > $O/layers_dpipe0.txt 2>&1 || exit $?
tail -n 4 $O/layers_*.txt
timeout -k 10 400 python -u -m pytest tests/test_gpu_parity.py -x -q --timeout 200 --timeout-method thread > $O/pytest_parity.log 2>&1; rc=$?
tail -3 $O/pytest_parity.log; [ $rc -eq 0 ] || exit $rc
bash scripts/diag/ab_trace_csv.sh r17b_ab default old fmtold dpipe0 || exit $?
