#!/bin/bash
# r17c: FMT K/V combine folded into the partial launch (last block per view); bits vs the round-start
# build, parity tests, in-graph trace A/B; FeatureNet kernel statistics (5 views, DTU size).
cd "$GRAFT_REPO_ROOT" || exit 1
export TMPDIR=/tmp
O=gpurun_out/r17c; mkdir -p $O
timeout -k 10 200 python scripts/diag/out_bits.py /tmp/new.npz > $O/bits_new.log 2>&1 || exit $?
TMVS_LIB_PATH=variants/old/libtransmvs_hip.so timeout -k 10 200 python scripts/diag/out_bits.py /tmp/old.npz > $O/bits_old.log 2>&1 || exit $?
python scripts/diag/out_bits.py --compare /tmp/old.npz /tmp/new.npz > $O/bits_compare.txt 2>&1; tail -2 $O/bits_compare.txt
timeout -k 10 400 python -u -m pytest tests/test_gpu_parity.py tests/test_gpu_train.py -x -q --timeout 200 --timeout-method thread > $O/pytest.log 2>&1; rc=$?
tail -3 $O/pytest.log; [ $rc -eq 0 ] || exit $rc
bash scripts/diag/ab_trace_csv.sh r17c_ab default old || exit $?
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $O/fn -o fn --output-format csv -- python3 scripts/diag/featurenet_run.py 5 > $O/fn.log 2>&1 || exit $?
f=$(find $O/fn -name "*kernel_stats.csv" | head -1); cp $f $O/featurenet_kernel_stats.csv; head -20 $f | cut -d, -f1-6
