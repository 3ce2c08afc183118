#!/bin/bash
# r20j: prob + WTA walk rows per wave: 2 (default) vs 3 vs 4
cd "$GRAFT_REPO_ROOT" || exit 1
export TMPDIR=/tmp
bash scripts/gpu/ab.sh r20j --bits --trace pwr3 pwr4
