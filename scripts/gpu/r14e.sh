#!/bin/bash
# r14e: FMT K/V partial: KNT tiles interleaved, PF tiles of tokens in flight (+ apply first tokens early);
# bitwise hot-path outputs vs the committed fmt.hip, kernel trace for PF = 4 (default), 2, 8 and old
cd "$GRAFT_REPO_ROOT" || exit 1
O=gpurun_out/r14e
mkdir -p $O
export TMPDIR=/tmp
timeout -k 10 120 python scripts/diag/out_bits.py $O/new.npz > $O/bits.log 2>&1 &&
TMVS_LIB_PATH=variants/fmtold/libtransmvs_hip.so timeout -k 10 120 python scripts/diag/out_bits.py $O/old.npz >> $O/bits.log 2>&1 &&
python scripts/diag/out_bits.py --compare $O/old.npz $O/new.npz >> $O/bits.log 2>&1 &&
rm -f $O/old.npz $O/new.npz &&
bash scripts/diag/ab_kernels.sh r14e/ab "fmt" fmtold nt2pf2 nt4pf4 nt1pf1 default > $O/fmt_ab.txt 2>&1
rc=$?
rm -rf $O/ab/*/
exit $rc
