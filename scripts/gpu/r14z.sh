#!/bin/bash
# r14z: MFMA DCN data kernel with the dy^T operands re-read per tap pair (rl: frees 32 VGPRs) and, in
# that room, the fp32 fixed-point conversion (rlf) vs the product: tmvs_dcn_backward bitwise, kernel
# times, C5 step times; prevg = the previous dcn_gather_windows_kernel indexing (flat, 64-bit divisions)
cd "$GRAFT_REPO_ROOT" || exit 1
O=$PWD/gpurun_out/r14z
mkdir -p $O
export TMPDIR=/tmp
timeout -k 10 200 python scripts/diag/dcn_bwd_bits.py $O/new.npz > $O/dcn_bits.log 2>&1 &&
TMVS_LIB_PATH=variants/rlf/libtransmvs_hip.so timeout -k 10 200 python scripts/diag/dcn_bwd_bits.py $O/rlf.npz >> $O/dcn_bits.log 2>&1 &&
python scripts/diag/dcn_bwd_bits.py --compare $O/new.npz $O/rlf.npz >> $O/dcn_bits.log 2>&1 &&
TMVS_LIB_PATH=variants/prevg/libtransmvs_hip.so timeout -k 10 200 python scripts/diag/dcn_bwd_bits.py $O/prevg.npz >> $O/dcn_bits.log 2>&1 &&
python scripts/diag/dcn_bwd_bits.py --compare $O/new.npz $O/prevg.npz >> $O/dcn_bits.log 2>&1 &&
rm -f $O/new.npz $O/rlf.npz $O/prevg.npz || exit 1
for v in default rl rlf prevg; do
  if [ "$v" = default ]; then unset TMVS_LIB_PATH; else export TMVS_LIB_PATH=variants/$v/libtransmvs_hip.so; fi
  STEPS=2 timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $O/$v -o run -- python3 scripts/diag/train_step_prof.py > $O/$v.log 2>&1 || exit $?
  echo "== $v" >> $O/summary.txt
  python3 scripts/diag/kernel_grid_times.py $O/$v/run_results.db dcn_bwd_data >> $O/summary.txt
  rm -rf $O/$v
done
for v in default rl rlf default rl rlf; do
  if [ "$v" = default ]; then unset TMVS_LIB_PATH; else export TMVS_LIB_PATH=variants/$v/libtransmvs_hip.so; fi
  timeout -k 10 300 python bench.py --steps 3 --warmup 1 --no-cpu-baseline --e2e-steps 0 > $O/bench_$v.json 2>> $O/bench.err || exit $?
  python3 -c "import json,sys; d=json.loads(open('$O/bench_$v.json').read().strip().splitlines()[-1]); t=d['train_depth_stages']; print('$v', t['ms_per_sample'], t['ms_per_sample_from_features'], d['value'])" >> $O/summary.txt
done
