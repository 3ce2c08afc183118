#!/bin/bash
# r20b: fused conv11 + prob kernel -- parity suites on the default (fused) library, the hot path's outputs bit
# for bit against the unfused build, kernel traces (default / nofuse / THI=4 / stage 1 fused too); then the
# B > 1 captures with one fork level (last: a segfault there ends the call).
cd "$GRAFT_REPO_ROOT" || exit 1
export TMPDIR=/tmp
O=gpurun_out/r20b; mkdir -p $O
bash scripts/gpu/ab.sh r20b --tests "tests/test_gpu_parity.py tests/test_gpu_featurenet.py tests/test_gpu_train_ref.py --deselect tests/test_gpu_parity.py::test_batch_samples_on_concurrent_streams_bitwise" \
  --bits --trace nofuse dp4 fuse2 || exit $?
timeout -k 10 300 python -u -m pytest -v --timeout 250 --timeout-method thread tests/test_gpu_batch.py \
  tests/test_gpu_parity.py::test_batch_samples_on_concurrent_streams_bitwise > $O/pytest_batch.log 2>&1
rc=$?
tail -5 $O/pytest_batch.log
exit $rc
