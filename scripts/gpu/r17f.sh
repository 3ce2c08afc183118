#!/bin/bash
# r17f: timing ablations of conv3d_lds_kernel (conv3 / conv4 / conv6 at the bench's stage shapes): no weight
# loads (abl1), no next-chunk tile fetch (abl2), no chunk barriers/commit (abl4), both (abl6), no MFMAs (abl8).
# Wrong outputs by construction: timing only.
cd "$GRAFT_REPO_ROOT" || exit 1
O=gpurun_out/r17f; mkdir -p $O
L=conv3,conv4,conv6
timeout -k 10 200 python scripts/diag/costreg_layers.py --layers $L > $O/layers_new.txt 2>&1 || exit $?
for v in abl1 abl2 abl4 abl6 abl8; do
  TMVS_LIB_PATH=variants/$v/libtransmvs_hip.so timeout -k 10 200 python scripts/diag/costreg_layers.py --layers $L > $O/layers_$v.txt 2>&1 || exit $?
done
tail -n 4 $O/layers_*.txt
