#!/bin/bash
# r14a: (1) DCN backward data A/B (LDS-staged offset/mask planes + pipelined taps vs the committed
# kernel): bitwise compare and timing; (2) prob walk with one plane of lookahead vs the committed
# prob kernels: bitwise hot-path outputs and kernel trace; (3) the whole -m gpu suite + smoke, bench
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
bash scripts/diag/ab_kernels.sh r14a/ab "prob conv0" probold > $O/prob_ab.txt 2>&1 || exit $?
rm -rf $O/ab/default $O/ab/probold
export TMVS_REPORT_DIR=$PWD/$O/fullsize
bash scripts/gpu/full_check.sh r14a || exit $?
timeout -k 10 400 python bench.py --steps 20 --warmup 5 > $O/bench.json 2> $O/bench.err
