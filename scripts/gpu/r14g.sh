#!/bin/bash
# r14g: DCN weight gradient with one sample derivation per thread (two channel quads of one pixel)
# vs per quad: bitwise dx / d offset-mask / dW, and tmvs_dcn_backward timing
cd "$GRAFT_REPO_ROOT" || exit 1
O=gpurun_out/r14g
mkdir -p $O
timeout -k 10 120 python scripts/diag/dcn_bwd_bits.py $O/new.npz > $O/bits.log 2>&1 &&
TMVS_LIB_PATH=variants/dcnw0/libtransmvs_hip.so timeout -k 10 120 python scripts/diag/dcn_bwd_bits.py $O/old.npz >> $O/bits.log 2>&1 &&
python scripts/diag/dcn_bwd_bits.py --compare $O/old.npz $O/new.npz >> $O/bits.log 2>&1 &&
rm -f $O/old.npz $O/new.npz &&
timeout -k 10 120 python scripts/diag/dcn_bwd_time.py > $O/time.log 2>&1 &&
TMVS_LIB_PATH=variants/dcnw0/libtransmvs_hip.so timeout -k 10 120 python scripts/diag/dcn_bwd_time.py >> $O/time.log 2>&1 &&
timeout -k 10 120 python scripts/diag/dcn_bwd_time.py >> $O/time.log 2>&1 &&
TMVS_LIB_PATH=variants/dcnw0/libtransmvs_hip.so timeout -k 10 120 python scripts/diag/dcn_bwd_time.py >> $O/time.log 2>&1
