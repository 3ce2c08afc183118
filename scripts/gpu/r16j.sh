#!/bin/bash
# r16j: LDS bank-conflict fixes A/B: deconv11 epilogue exchange slots (c8x), conv1 staging stride SW=18 (sw18)
cd "$GRAFT_REPO_ROOT" || exit 1
O=gpurun_out/r16j; mkdir -p $O
timeout -k 10 200 python scripts/diag/costreg_layers.py --save /tmp/base.pt --layers conv1,conv11 > $O/layers_base.txt 2>&1 || exit $?
for v in c8x sw18; do
  TMVS_LIB_PATH=variants/$v/libtransmvs_hip.so timeout -k 10 200 python scripts/diag/costreg_layers.py --compare /tmp/base.pt --layers conv1,conv11 > $O/layers_$v.txt 2>&1 || exit $?
done
cat $O/layers_base.txt $O/layers_c8x.txt $O/layers_sw18.txt
bash scripts/diag/ab_trace_csv.sh r16j_ab default c8x sw18 default c8x sw18 || exit $?
