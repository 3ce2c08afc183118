#!/bin/bash
# r20l: stage-2 pathway software-pipelined (pathway16_pipe_kernel), 512 / 256 / 1024 target workgroups
cd "$GRAFT_REPO_ROOT" || exit 1
export TMPDIR=/tmp
mkdir -p gpurun_out/r20l
for v in pwpipe pwpipe256 pwpipe1k; do
  TMVS_LIB_PATH=variants/$v/libtransmvs_hip.so timeout -k 10 300 python -u -m pytest tests/test_gpu_parity.py \
    -k "pathway" -x -q --timeout 120 --timeout-method thread > gpurun_out/r20l/pytest_$v.log 2>&1 || { tail -20 gpurun_out/r20l/pytest_$v.log; exit 1; }
  echo "pytest $v: $(tail -1 gpurun_out/r20l/pytest_$v.log)"
done
bash scripts/gpu/ab.sh r20l --bits --trace pwpipe pwpipe256 pwpipe1k
