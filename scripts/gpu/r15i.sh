#!/bin/bash
# r15i: FMT LayerNorm forward with 16-byte row loads / stores (product) vs scalar (lnfold):
# training GPU tests, one C5 step bitwise, kernel times, C5 step times
cd "$GRAFT_REPO_ROOT" || exit 1
O=$PWD/gpurun_out/r15i
mkdir -p $O
export TMPDIR=/tmp
timeout -k 10 400 python -u -m pytest -x -v --timeout 300 --timeout-method thread tests/test_gpu_train.py > $O/pytest.log 2>&1 || exit $?
timeout -k 10 200 python scripts/diag/train_bits.py $O/new.npz > $O/bits.log 2>&1 &&
TMVS_LIB_PATH=variants/lnfold/libtransmvs_hip.so timeout -k 10 200 python scripts/diag/train_bits.py $O/old.npz >> $O/bits.log 2>&1 &&
python scripts/diag/train_bits.py --compare $O/old.npz $O/new.npz >> $O/bits.log 2>&1 &&
rm -f $O/old.npz $O/new.npz || exit 1
for v in default lnfold; do
  if [ "$v" = default ]; then unset TMVS_LIB_PATH; else export TMVS_LIB_PATH=variants/$v/libtransmvs_hip.so; fi
  STEPS=2 timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $O/$v -o run -- python3 scripts/diag/train_step_prof.py > $O/$v.log 2>&1 || exit $?
  echo "== $v" >> $O/summary.txt
  python3 scripts/diag/kernel_grid_times.py $O/$v/run_results.db layer_norm >> $O/summary.txt
  rm -rf $O/$v
done
for v in default lnfold default lnfold; do
  if [ "$v" = default ]; then unset TMVS_LIB_PATH; else export TMVS_LIB_PATH=variants/$v/libtransmvs_hip.so; fi
  timeout -k 10 300 python bench.py --steps 3 --warmup 1 --no-cpu-baseline --e2e-steps 0 > $O/bench_$v.json 2>> $O/bench.err || exit $?
  python3 -c "import json,sys; d=json.loads(open('$O/bench_$v.json').read().strip().splitlines()[-1]); t=d['train_depth_stages']; print('$v', t['ms_per_sample'], t['ms_per_sample_from_features'], d['value'])" >> $O/summary.txt
done
