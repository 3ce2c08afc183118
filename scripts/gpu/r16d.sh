#!/bin/bash
# r16d = r16b (parity tests) then r16c (split-K A/B) in one box
cd "$GRAFT_REPO_ROOT" || exit 1
bash scripts/gpu/r16c.sh || exit $?
bash scripts/gpu/r16b.sh
