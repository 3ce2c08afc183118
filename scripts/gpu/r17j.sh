#!/bin/bash
# r17j: conv5 (32 -> 64, stride 2) through the LDS-tiled kernel with the wave split (other K order, so not
# bitwise: timing only here) vs the direct kernel
cd "$GRAFT_REPO_ROOT" || exit 1
O=gpurun_out/r17j; mkdir -p $O
L=conv5
timeout -k 10 200 python scripts/diag/costreg_layers.py --save /tmp/base.pt --layers $L > $O/layers_base.txt 2>&1 || exit $?
for v in c5l1 c5l2; do
  TMVS_LIB_PATH=variants/$v/libtransmvs_hip.so timeout -k 10 200 python scripts/diag/costreg_layers.py --compare /tmp/base.pt --layers $L > $O/layers_$v.txt 2>&1 || exit $?
done
tail -n 4 $O/layers_*.txt
