#!/bin/bash
# Bench A/B of the FMT-pathway side stream: default priority, high priority (-1), and no overlap.
# Alternates the three settings 3 times so drift hits them equally.
cd "$GRAFT_REPO_ROOT" || exit 1
run() {
  timeout -k 10 200 python bench.py --steps 40 --warmup 5 --no-cpu-baseline --e2e-steps 0 --train-steps 0 --profile-steps 0 "$@" 2>/dev/null | \
    python -c "import json,sys; d=json.loads(sys.stdin.read().strip().splitlines()[-1]); print('$*', d['value'], d['ms_per_step'])"
}
for rep in 1 2 3; do
  run --side-priority 0 || exit $?
  run --side-priority -1 || exit $?
  run --no-overlap || exit $?
done
