#!/bin/bash
# r20c: the wave-specialised fused conv11 + prob kernel (THI 8 default, THI 4 variant) vs the two-kernel form
cd "$GRAFT_REPO_ROOT" || exit 1
export TMPDIR=/tmp
bash scripts/gpu/ab.sh r20c --tests "tests/test_gpu_parity.py::test_costregnet_wta_equals_costregnet_then_softmax" \
  --bits --trace nofuse dp4
