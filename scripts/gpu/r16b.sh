#!/bin/bash
# r16b: ADVICE-r4 tests (sticky flags, device lr, DCN non-finite dy), the gpu-seeded full-size cascades
# (C2-C4) and the all-gradient C5 comparison, then a short bench (eager line)
cd "$GRAFT_REPO_ROOT" || exit 1
O=gpurun_out/r16b; mkdir -p $O
export TMVS_REPORT_DIR=$O/fullsize
timeout -k 10 900 python -u -m pytest -x -v --timeout 400 --timeout-method thread \
  "tests/test_gpu_train.py::test_flat_adam_graph_replay_follows_lr_schedule" \
  "tests/test_gpu_train.py::test_graph_overflow_flags_are_sticky" \
  "tests/test_gpu_train.py::test_flat_adam_graph_replay_equals_eager_steps" \
  "tests/test_gpu_featurenet.py::test_dcn_backward_nonfinite_dy_poisons_dx" \
  tests/test_gpu_train_c5.py tests/test_gpu_fullsize.py -s > $O/pytest.log 2>&1 || exit $?
timeout -k 10 300 python bench.py --steps 20 --warmup 5 --no-cpu-baseline --e2e-steps 0 --train-steps 0 > $O/bench.json 2> $O/bench.err || exit $?
tail -1 $O/bench.json | cut -c1-300
timeout -k 10 200 python scripts/diag/costreg_layers.py --reps 20 > $O/layers.txt 2>&1 || exit $?
cat $O/layers.txt
