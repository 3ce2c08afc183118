#!/bin/bash
# r17m: FMT linear layers with block-interleaved MFMA chains (32 % -> 5 % back-to-back dependent MFMAs in the
# apply): bits vs the previous build, in-graph trace A/B (twice)
cd "$GRAFT_REPO_ROOT" || exit 1
O=gpurun_out/r17m; mkdir -p $O
timeout -k 10 200 python scripts/diag/out_bits.py /tmp/new.npz > $O/bits_new.log 2>&1 || exit $?
TMVS_LIB_PATH=variants/fmthead/libtransmvs_hip.so timeout -k 10 200 python scripts/diag/out_bits.py /tmp/old.npz > $O/bits_old.log 2>&1 || exit $?
python scripts/diag/out_bits.py --compare /tmp/old.npz /tmp/new.npz > $O/bits_compare.txt 2>&1; tail -2 $O/bits_compare.txt
bash scripts/diag/ab_trace_csv.sh r17m_ab default fmthead || exit $?
grep fmt gpurun_out/r17m_ab/trace_*.txt
