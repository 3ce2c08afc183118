#!/bin/bash
# r14p: DCN backward data kernel with XCD-contiguous tile ranges vs blockIdx order:
# bitwise DCN gradients, DCN kernel trace, C5 training step
cd "$GRAFT_REPO_ROOT" || exit 1
O=gpurun_out/r14p
mkdir -p $O
export TMPDIR=/tmp
timeout -k 10 120 python scripts/diag/dcn_bwd_bits.py $O/new.npz > $O/bits.log 2>&1 &&
TMVS_LIB_PATH=variants/dxcd0/libtransmvs_hip.so timeout -k 10 120 python scripts/diag/dcn_bwd_bits.py $O/old.npz >> $O/bits.log 2>&1 &&
python scripts/diag/dcn_bwd_bits.py --compare $O/old.npz $O/new.npz >> $O/bits.log 2>&1 &&
rm -f $O/old.npz $O/new.npz || exit 1
for v in default dxcd0; do
  if [ "$v" = default ]; then unset TMVS_LIB_PATH; else export TMVS_LIB_PATH=variants/$v/libtransmvs_hip.so; fi
  timeout -k 10 120 rocprofv3 --kernel-trace --stats -d $O/$v -o run -- python3 scripts/diag/dcn_bwd_kernels.py > $O/$v.log 2>&1 || exit $?
  echo "== $v" >> $O/summary.txt
  python3 scripts/diag/kernel_grid_times.py $O/$v/run_results.db dcn >> $O/summary.txt
  rm -rf $O/$v
done
for v in default dxcd0 default dxcd0; do
  if [ "$v" = default ]; then unset TMVS_LIB_PATH; else export TMVS_LIB_PATH=variants/$v/libtransmvs_hip.so; fi
  timeout -k 10 300 python bench.py --steps 3 --warmup 1 --no-cpu-baseline --e2e-steps 0 > $O/bench_$v.json 2>> $O/bench.err || exit $?
  python3 -c "import json,sys; d=json.loads(open('$O/bench_$v.json').read().strip().splitlines()[-1]); t=d['train_depth_stages']; print('$v', t['ms_per_sample'], t['ms_per_sample_from_features'])" >> $O/summary.txt
done
