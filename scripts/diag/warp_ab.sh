#!/bin/bash
# A/B of warp_corr builds: the default library, then each variants/NAME/ library given
cd "$GRAFT_REPO_ROOT" || exit 1
timeout -k 10 120 python scripts/diag/warp_time.py || exit $?
for v in "$@"; do
  TMVS_LIB_PATH=variants/$v/libtransmvs_hip.so timeout -k 10 120 python scripts/diag/warp_time.py || exit $?
done
