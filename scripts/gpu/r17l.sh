#!/bin/bash
# r17l: fragment-major weight copies for the trunk's LDS-kernel layers (conv3..conv6), packed per call by
# frag_pack_kernel: bits vs the same build reading the standard packing (nofrag), in-graph trace A/B
cd "$GRAFT_REPO_ROOT" || exit 1
O=gpurun_out/r17l; mkdir -p $O
timeout -k 10 200 python scripts/diag/out_bits.py /tmp/new.npz > $O/bits_new.log 2>&1 || exit $?
TMVS_LIB_PATH=variants/nofrag/libtransmvs_hip.so timeout -k 10 200 python scripts/diag/out_bits.py /tmp/nofrag.npz > $O/bits_nofrag.log 2>&1 || exit $?
python scripts/diag/out_bits.py --compare /tmp/nofrag.npz /tmp/new.npz > $O/bits_compare.txt 2>&1; tail -2 $O/bits_compare.txt
bash scripts/diag/ab_trace_csv.sh r17l_ab default nofrag default nofrag || exit $?
