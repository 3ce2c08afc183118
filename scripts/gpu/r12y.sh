#!/bin/bash
# r12y (final state of round 3): the whole GPU suite + smoke, then the round measurement.
cd "$GRAFT_REPO_ROOT" || exit 1
bash scripts/gpu/full_check.sh r12y || exit $?
bash scripts/profile_round.sh r12y
