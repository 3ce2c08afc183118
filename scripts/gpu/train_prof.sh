#!/bin/bash
set -o pipefail
OUT=gpurun_out/${1:-train_prof}; mkdir -p $OUT
export TMPDIR=/tmp
timeout -k 10 400 rocprofv3 --kernel-trace -d $OUT/trace -o run --output-format csv -- python3 scripts/diag/train_graph_prof.py 4 > $OUT/prof.log 2>&1 || { tail -20 $OUT/prof.log; exit 1; }
grep "replay ms" $OUT/prof.log
python3 scripts/diag/train_graph_table.py $OUT/trace/run_kernel_trace.csv 80 > $OUT/table.txt
head -70 $OUT/table.txt
