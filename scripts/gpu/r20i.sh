#!/bin/bash
# r20i: Infinity-Cache row chunking of conv0 -> conv1 and conv11 -> prob/WTA (2 chunks default; 1 = off, 4)
cd "$GRAFT_REPO_ROOT" || exit 1
export TMPDIR=/tmp
bash scripts/gpu/ab.sh r20i --tests "tests/test_gpu_parity.py::test_costregnet_wta_equals_costregnet_then_softmax tests/test_gpu_parity.py::test_conv3d_layers tests/test_gpu_parity.py::test_deconv3d_layers" \
  --bits --trace mall1 mall4
