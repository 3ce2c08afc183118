#!/bin/bash
# r20d: wave -> SIMD placement probe; the fused conv11 + prob kernel with its MFMA / walk roles placed three ways
cd "$GRAFT_REPO_ROOT" || exit 1
export TMPDIR=/tmp
timeout -k 10 60 scripts/micro/wave_simd > gpurun_out/r20d_wave_simd.txt 2>&1 || exit $?
cat gpurun_out/r20d_wave_simd.txt
bash scripts/gpu/ab.sh r20d --tests "tests/test_gpu_parity.py::test_costregnet_wta_equals_costregnet_then_softmax" \
  --bits --trace nofuse role1 role2
