#!/bin/bash
# r16c: split-K coarse-level convs (conv3d_splitk_kernel) A/B: per-layer times + output diff vs the product
# kernels, the raw-conv parity test on the variant, and the bench step's kernel trace per variant
cd "$GRAFT_REPO_ROOT" || exit 1
export TMPDIR=/tmp
O=gpurun_out/r16c; mkdir -p $O
# a failing test is reported, a timeout / abort / fault ends the script
soft() { rc=$1; if [ $rc -eq 124 ] || [ $rc -eq 137 ] || [ $rc -eq 134 ] || [ $rc -eq 139 ]; then exit $rc; fi; [ $rc -ne 0 ] && echo "FAILED rc=$rc"; return 0; }
timeout -k 10 200 python scripts/diag/costreg_layers.py --save /tmp/base.pt > $O/layers_base.txt 2>&1 || exit $?
cat $O/layers_base.txt
for v in sk15 skd skall pr2 c0x c28 c44; do
  TMVS_LIB_PATH=variants/$v/libtransmvs_hip.so timeout -k 10 200 python scripts/diag/costreg_layers.py --compare /tmp/base.pt > $O/layers_$v.txt 2>&1 || exit $?
  echo "== $v"; cat $O/layers_$v.txt
done
TMVS_LIB_PATH=variants/skall/libtransmvs_hip.so timeout -k 10 300 python -u -m pytest -x -q --timeout 120 --timeout-method thread \
  tests/test_gpu_train.py -k "conv3d_mfma_raw" > $O/pytest_raw_skall.log 2>&1; soft $?
tail -2 $O/pytest_raw_skall.log
TMVS_LIB_PATH=variants/pr2/libtransmvs_hip.so timeout -k 10 300 python -u -m pytest -x -q --timeout 120 --timeout-method thread \
  tests/test_gpu_parity.py -k "costregnet or e2e_c1 or cascade_48" > $O/pytest_pr2.log 2>&1; soft $?
tail -2 $O/pytest_pr2.log
bash scripts/diag/ab_kernels.sh r16c_ab "conv3d deconv3d prob conv0" skall pr2 c0x c44 > $O/ab.txt 2>&1 || exit $?
cat $O/ab.txt
