#!/bin/bash
# A/B of library builds on the bench's hot-path step: default library, then each variants/NAME/.
# Prints value and the per-entry-point HIP-event breakdown.
cd "$GRAFT_REPO_ROOT" || exit 1
run() {
  timeout -k 10 200 python bench.py --steps 20 --warmup 5 --no-cpu-baseline --e2e-steps 0 --train-steps 0 2>/dev/null | \
    python -c "import json,sys; d=json.loads(sys.stdin.read().strip().splitlines()[-1]); print('$1', d['value'], d['kernel_ms_per_depth_map'], d['roofline']['per_stage_ms'])"
}
run default || exit $?
for v in "$@"; do
  TMVS_LIB_PATH=variants/$v/libtransmvs_hip.so run $v || exit $?
done
