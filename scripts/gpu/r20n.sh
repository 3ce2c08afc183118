#!/bin/bash
# r20n: fused-role pipelined stage-2 pathway (pathway16_pipe2_kernel): parity tests, standalone timing, bits
cd "$GRAFT_REPO_ROOT" || exit 1
export TMPDIR=/tmp
mkdir -p gpurun_out/r20n
for v in pwpipe2 pwpipe2sg; do
  TMVS_LIB_PATH=variants/$v/libtransmvs_hip.so timeout -k 10 300 python -u -m pytest tests/test_gpu_parity.py \
    -k "pathway" -x -q --timeout 120 --timeout-method thread > gpurun_out/r20n/pytest_$v.log 2>&1 || { tail -20 gpurun_out/r20n/pytest_$v.log; exit 1; }
  echo "pytest $v: $(tail -1 gpurun_out/r20n/pytest_$v.log)"
done
for v in default pwpipe2 pwpipe2sg pwpipe default pwpipe2 pwpipe2sg; do
  if [ $v = default ]; then unset TMVS_LIB_PATH; else export TMVS_LIB_PATH=variants/$v/libtransmvs_hip.so; fi
  timeout -k 10 120 python scripts/diag/pathway_time.py 50 || exit 1
done
unset TMVS_LIB_PATH
bash scripts/gpu/ab.sh r20n --bits --trace pwpipe2 pwpipe2sg
