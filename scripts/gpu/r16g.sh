#!/bin/bash
# r16g: parity tests (r16b) + concurrent-batch test + bench; deconv11 direct-store and prob-WTA row A/B;
# then the warp PMC + training glue (r16f)
cd "$GRAFT_REPO_ROOT" || exit 1
O=gpurun_out/r16g; mkdir -p $O
timeout -k 10 300 python -u -m pytest -x -v --timeout 200 --timeout-method thread \
  "tests/test_gpu_parity.py::test_batch_samples_on_concurrent_streams_bitwise" \
  "tests/test_gpu_featurenet.py::test_dcn_backward_nonfinite_dy_poisons_dx" > $O/pytest_a.log 2>&1 || exit $?
tail -3 $O/pytest_a.log
timeout -k 10 200 python scripts/diag/costreg_layers.py --save /tmp/base.pt --layers conv1,conv11,prob > $O/layers_base.txt 2>&1 || exit $?
for v in c8d sw20; do
  TMVS_LIB_PATH=variants/$v/libtransmvs_hip.so timeout -k 10 200 python scripts/diag/costreg_layers.py --compare /tmp/base.pt --layers conv1,conv11,prob > $O/layers_$v.txt 2>&1 || exit $?
done
cat $O/layers_base.txt $O/layers_c8d.txt $O/layers_sw20.txt
bash scripts/diag/ab_trace_csv.sh r16g_ab default wta1 c8d sw20 || exit $?
bash scripts/gpu/r16b.sh || exit $?
bash scripts/gpu/r16f.sh
