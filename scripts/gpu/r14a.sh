#!/bin/bash
# r14a: A/Bs on one box. (1) DCN backward data (LDS-staged offset/mask planes + pipelined taps vs the
# committed kernel): bitwise + timing. (2) CostRegNet: prob walk one plane ahead, conv0 fused into
# conv1 and conv11's skip, deconv chunk prefetch, conv weight lookahead -- bitwise hot-path outputs
# vs the committed costreg (probold) and per-kernel trace times for the variants.
cd "$GRAFT_REPO_ROOT" || exit 1
O=gpurun_out/r14a
mkdir -p $O
export TMPDIR=/tmp
timeout -k 10 120 python scripts/diag/dcn_bwd_bits.py $O/new.npz > $O/bits.log 2>&1 &&
TMVS_LIB_PATH=variants/dcnold/libtransmvs_hip.so timeout -k 10 120 python scripts/diag/dcn_bwd_bits.py $O/old.npz >> $O/bits.log 2>&1 &&
python scripts/diag/dcn_bwd_bits.py --compare $O/old.npz $O/new.npz >> $O/bits.log 2>&1 &&
rm -f $O/old.npz $O/new.npz &&
timeout -k 10 120 python scripts/diag/dcn_bwd_time.py > $O/time.log 2>&1 &&
TMVS_LIB_PATH=variants/dcnold/libtransmvs_hip.so timeout -k 10 120 python scripts/diag/dcn_bwd_time.py >> $O/time.log 2>&1 &&
timeout -k 10 120 python scripts/diag/dcn_bwd_time.py >> $O/time.log 2>&1 &&
timeout -k 10 120 python scripts/diag/out_bits.py $O/pnew.npz > $O/prob_bits.log 2>&1 &&
TMVS_LIB_PATH=variants/probold/libtransmvs_hip.so timeout -k 10 120 python scripts/diag/out_bits.py $O/pold.npz >> $O/prob_bits.log 2>&1 &&
python scripts/diag/out_bits.py --compare $O/pold.npz $O/pnew.npz >> $O/prob_bits.log 2>&1 &&
rm -f $O/pold.npz $O/pnew.npz &&
bash scripts/diag/ab_kernels.sh r14a/ab "prob conv0 deconv3d conv3d_lds s2c8" probold wla4 wla6 pfmin3 nopf > $O/cr_ab.txt 2>&1
rc=$?
rm -rf $O/ab/*/
exit $rc
