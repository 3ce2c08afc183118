#!/bin/bash
# FMT A/B: product, apply tiles-per-wave sweep, branch-free elu, transposed K/V reduction (bit digests must agree)
set -o pipefail
OUT=gpurun_out/${1:-fmt_ab}; mkdir -p $OUT
run() { timeout -k 10 120 python -u scripts/diag/fmt_time.py 40 >> $OUT/fmt_ab.txt 2>&1; }
run || exit $?
for t in 2 3 4 5 6 8; do TMVS_LIB_PATH=variants/tpwenv/libtransmvs_hip.so TMVS_APPLY_TPW=$t run || exit $?; done
for v in elubf kvtr both; do TMVS_LIB_PATH=variants/$v/libtransmvs_hip.so run || exit $?; done
run || exit $?
cat $OUT/fmt_ab.txt
