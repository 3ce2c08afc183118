#!/bin/bash
# r20m: stage-2 pathway launches alone (scripts/diag/pathway_time.py): default vs pipelined forms and ablations
cd "$GRAFT_REPO_ROOT" || exit 1
export TMPDIR=/tmp
for v in default pwpipe pwpipe_nosb pwpipe_abl1 pwpipe_abl2 default pwpipe pwpipe_nosb; do
  if [ $v = default ]; then unset TMVS_LIB_PATH; else export TMVS_LIB_PATH=variants/$v/libtransmvs_hip.so; fi
  timeout -k 10 120 python scripts/diag/pathway_time.py 50 || exit 1
done
