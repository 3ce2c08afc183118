#!/bin/bash
# A/B of library builds on the C5 training step (graph replay, from features and full). Usage:
#   bash scripts/diag/ab_train.sh VARIANT...   (variants/NAME/libtransmvs_hip.so)
cd "$GRAFT_REPO_ROOT" || exit 1
run() {
  timeout -k 10 300 python bench.py --steps 1 --warmup 1 --no-cpu-baseline --e2e-steps 0 --train-steps 5 \
    --profile-steps 1 2>/dev/null | python -c "import json,sys; d=json.loads(sys.stdin.read().strip().splitlines()[-1]); t=d['train_depth_stages']; print('$1', t['ms_per_sample'], t['ms_per_sample_from_features'], t['launch'][:60])"
}
run default || exit $?
for v in "$@"; do
  TMVS_LIB_PATH=variants/$v/libtransmvs_hip.so run $v || exit $?
done
