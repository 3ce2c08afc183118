#!/bin/bash
# One A/B driver for library variants on the GPU box (replaces the per-run r16*/r17* scripts; their outputs
# are under profiles/r16*, profiles/r17*). Variants are built here first with scripts/build_variant.py into
# variants/NAME/libtransmvs_hip.so; "default" is the in-tree library.
#
#   bash scripts/gpu/ab.sh TAG [--layers conv3,conv6 [--stages 1,2,3]] [--bits] [--tests "tests/a.py tests/b.py"]
#                              [--trace] VARIANT...
#
#   --layers  CostRegNet layers alone (scripts/diag/costreg_layers.py): default saved, each variant timed and
#             compared bit for bit (== / DIFF)
#   --bits    hot-path outputs of one C2 depth map (scripts/diag/out_bits.py), each variant vs default
#   --tests   pytest files run on the default library first (stops on failure)
#   --trace   rocprofv3 kernel trace of the bench step per library (scripts/diag/ab_trace_csv.sh)
#   --fnet    FeatureNet forward over the 5 DTU views per library (scripts/diag/featurenet_run.py)
#   --dcn STD the fused FeatureNet DCN alone at the head sizes (scripts/diag/dcn_time.py), offsets of STD px
#             (0 = the reference's zero-initialised offset conv), each variant compared bit for bit
# Every GPU step runs under its own time limit and the script stops at the first failure.
TAG=$1; shift
cd "$GRAFT_REPO_ROOT" || exit 1
LAYERS=""; STAGES="1,2,3"; BITS=0; TESTS=""; TRACE=0; DCN=""; FNET=0; VARIANTS=()
while [ $# -gt 0 ]; do
  case "$1" in
    --layers) LAYERS=$2; shift 2 ;;
    --stages) STAGES=$2; shift 2 ;;
    --bits) BITS=1; shift ;;
    --tests) TESTS=$2; shift 2 ;;
    --trace) TRACE=1; shift ;;
    --dcn) DCN=$2; shift 2 ;;
    --fnet) FNET=1; shift ;;
    *) VARIANTS+=("$1"); shift ;;
  esac
done
O=gpurun_out/$TAG; mkdir -p $O
lib() { [ "$1" = default ] && echo "" || echo "variants/$1/libtransmvs_hip.so"; }
if [ -n "$TESTS" ]; then
  timeout -k 10 1000 python -u -m pytest $TESTS -x -q --timeout 300 --timeout-method thread > $O/pytest.log 2>&1; rc=$?
  tail -3 $O/pytest.log; [ $rc -eq 0 ] || exit $rc
fi
if [ -n "$LAYERS" ]; then
  timeout -k 10 200 python scripts/diag/costreg_layers.py --save /tmp/ab_base.pt --layers $LAYERS --stages $STAGES \
    > $O/layers_default.txt 2>&1 || exit $?
  for v in "${VARIANTS[@]}"; do
    TMVS_LIB_PATH=$(lib $v) timeout -k 10 200 python scripts/diag/costreg_layers.py --compare /tmp/ab_base.pt \
      --layers $LAYERS --stages $STAGES > $O/layers_$v.txt 2>&1 || exit $?
  done
  tail -n 4 $O/layers_*.txt
fi
if [ -n "$DCN" ]; then
  DCN_FUSED=1 DCN_OFFSET_STD=$DCN DCN_SAVE=/tmp/ab_dcn.pt timeout -k 10 200 python scripts/diag/dcn_time.py \
    > $O/dcn_default.txt 2>&1 || exit $?
  for v in "${VARIANTS[@]}"; do
    DCN_FUSED=1 DCN_OFFSET_STD=$DCN DCN_COMPARE=/tmp/ab_dcn.pt TMVS_DCN_TAG=$v TMVS_LIB_PATH=$(lib $v) \
      timeout -k 10 200 python scripts/diag/dcn_time.py > $O/dcn_$v.txt 2>&1 || exit $?
  done
  grep -h " us" $O/dcn_*.txt
fi
if [ $FNET -eq 1 ]; then
  for v in default "${VARIANTS[@]}" default "${VARIANTS[@]}"; do  # two alternating rounds
    TMVS_LIB_PATH=$(lib $v) timeout -k 10 200 python scripts/diag/featurenet_run.py 20 2>&1 | grep FeatureNet \
      >> $O/fnet.txt || exit $?
  done
  cat $O/fnet.txt
fi
if [ $BITS -eq 1 ]; then
  timeout -k 10 200 python scripts/diag/out_bits.py /tmp/ab_default.npz > $O/bits_default.log 2>&1 || exit $?
  for v in "${VARIANTS[@]}"; do
    TMVS_LIB_PATH=$(lib $v) timeout -k 10 200 python scripts/diag/out_bits.py /tmp/ab_$v.npz > $O/bits_$v.log 2>&1 || exit $?
    python scripts/diag/out_bits.py --compare /tmp/ab_default.npz /tmp/ab_$v.npz > $O/bits_compare_$v.txt 2>&1
    echo "bits $v: $(tail -1 $O/bits_compare_$v.txt)"
  done
fi
if [ $TRACE -eq 1 ]; then
  bash scripts/diag/ab_trace_csv.sh ${TAG}_trace default "${VARIANTS[@]}" || exit $?
fi
exit 0
