#!/bin/bash
# r17i: deconv3d_lds input tiles 2x4 / 4x2 / 2x8 (2 or 4 input rows per wave) vs 2x2; conv4 per-depth
# configuration in the product. Bitwise vs the product (base).
cd "$GRAFT_REPO_ROOT" || exit 1
O=gpurun_out/r17i; mkdir -p $O
L=conv4,conv7,conv9
timeout -k 10 200 python scripts/diag/costreg_layers.py --save /tmp/base.pt --layers $L > $O/layers_base.txt 2>&1 || exit $?
for v in dA dB dC; do
  TMVS_LIB_PATH=variants/$v/libtransmvs_hip.so timeout -k 10 200 python scripts/diag/costreg_layers.py --compare /tmp/base.pt --layers $L > $O/layers_$v.txt 2>&1 || exit $?
done
tail -n 4 $O/layers_*.txt
