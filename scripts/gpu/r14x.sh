#!/bin/bash
# r14x: round-4 training changes vs the committed tree (variants/headtree = git archive HEAD, built):
# DCN backward dcol on MFMA (32-output-channel instance), partial combines with 8 loads in flight
# (strided_sum), the offset/mask conv's data gradient accumulated in the conv epilogue
# (tmvs_conv3x3_nhwc_acc), warp backward flush rows from LDS (nosref = from global); fix32 = + fp32
# fixed-point conversion in the DCN scatter.
# GPU tests of the touched pieces, one C5 step bitwise vs HEAD, kernel trace, C5 step times.
cd "$GRAFT_REPO_ROOT" || exit 1
O=$PWD/gpurun_out/r14x
mkdir -p $O
export TMPDIR=/tmp
timeout -k 10 500 python -u -m pytest -x -v --timeout 300 --timeout-method thread tests/test_gpu_featurenet.py tests/test_gpu_train_ref.py tests/test_gpu_train.py > $O/pytest.log 2>&1 || exit $?
timeout -k 10 200 python scripts/diag/dcn_bwd_bits.py $O/new.npz > $O/dcn_bits.log 2>&1 &&
TMVS_LIB_PATH=variants/fix32/libtransmvs_hip.so timeout -k 10 200 python scripts/diag/dcn_bwd_bits.py $O/f32.npz >> $O/dcn_bits.log 2>&1 &&
python scripts/diag/dcn_bwd_bits.py --compare $O/f32.npz $O/new.npz >> $O/dcn_bits.log 2>&1 &&
rm -f $O/f32.npz $O/new.npz || exit 1
timeout -k 10 200 python scripts/diag/train_bits.py $O/new.npz > $O/bits.log 2>&1 &&
(cd variants/headtree && GRAFT_REPO_ROOT=$PWD timeout -k 10 200 python scripts/diag/train_bits.py $O/old.npz >> $O/bits.log 2>&1) &&
python scripts/diag/train_bits.py --compare $O/old.npz $O/new.npz >> $O/bits.log 2>&1 &&
rm -f $O/old.npz $O/new.npz || exit 1
for v in default fix32 nosref headtree; do
  unset TMVS_LIB_PATH; D=.
  if [ "$v" = fix32 ] || [ "$v" = nosref ]; then export TMVS_LIB_PATH=variants/$v/libtransmvs_hip.so; fi
  if [ "$v" = headtree ]; then D=variants/headtree; fi
  (cd $D && STEPS=2 GRAFT_REPO_ROOT=$PWD timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $O/$v -o run -- python3 scripts/diag/train_step_prof.py > $O/$v.log 2>&1) || exit $?
  echo "== $v" >> $O/summary.txt
  python3 scripts/diag/kernel_grid_times.py $O/$v/run_results.db dcn_bwd colsum sum_ conv3x3 elementwise warp_corr_bwd >> $O/summary.txt
  rm -rf $O/$v
done
for v in default headtree fix32 nosref default headtree fix32 nosref; do
  unset TMVS_LIB_PATH; D=.
  if [ "$v" = fix32 ] || [ "$v" = nosref ]; then export TMVS_LIB_PATH=variants/$v/libtransmvs_hip.so; fi
  if [ "$v" = headtree ]; then D=variants/headtree; fi
  (cd $D && timeout -k 10 300 python bench.py --steps 3 --warmup 1 --no-cpu-baseline --e2e-steps 0 > $O/bench_$v.json 2>> $O/bench.err) || exit $?
  python3 -c "import json,sys; d=json.loads(open('$O/bench_$v.json').read().strip().splitlines()[-1]); t=d['train_depth_stages']; print('$v', t['ms_per_sample'], t['ms_per_sample_from_features'], d['value'])" >> $O/summary.txt
done
