#!/bin/bash
# r17g: conv3d_lds wave split (WS: waves own distinct 16-channel output blocks, so they stop requesting
# identical weight fragments; r17f: without weight loads conv6 80.6 -> 50.3 us) -- per-layer A/B, bitwise
cd "$GRAFT_REPO_ROOT" || exit 1
O=gpurun_out/r17g; mkdir -p $O
L=conv3,conv4,conv6
timeout -k 10 200 python scripts/diag/costreg_layers.py --save /tmp/base.pt --layers $L > $O/layers_base.txt 2>&1 || exit $?
for v in c6ws2 c6ws4 c6ws4b c4ws2 c3ws2; do
  TMVS_LIB_PATH=variants/$v/libtransmvs_hip.so timeout -k 10 200 python scripts/diag/costreg_layers.py --compare /tmp/base.pt --layers $L > $O/layers_$v.txt 2>&1 || exit $?
done
tail -n 4 $O/layers_*.txt
