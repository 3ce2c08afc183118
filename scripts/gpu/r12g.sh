#!/bin/bash
# r12g: bitwise A/B of the apply kernel's token sums (permlane swaps vs ds_bpermute), parity tests,
# kernel-trace A/B.
cd "$GRAFT_REPO_ROOT" || exit 1
mkdir -p gpurun_out/r12g
timeout -k 10 120 python scripts/diag/out_bits.py gpurun_out/r12g/base.npz > gpurun_out/r12g/bits.log 2>&1 || exit $?
TMVS_LIB_PATH=$PWD/variants/tokshfl/libtransmvs_hip.so timeout -k 10 120 python scripts/diag/out_bits.py gpurun_out/r12g/tokshfl.npz >> gpurun_out/r12g/bits.log 2>&1 || exit $?
python scripts/diag/out_bits.py --compare gpurun_out/r12g/base.npz gpurun_out/r12g/tokshfl.npz >> gpurun_out/r12g/bits.log 2>&1
rm -f gpurun_out/r12g/*.npz
timeout -k 10 300 python -u -m pytest -x -q --timeout 300 --timeout-method thread tests/test_gpu_parity.py -m gpu > gpurun_out/r12g/pytest.log 2>&1 || exit $?
bash scripts/ab_trace.sh r12g "fmt_apply|total" base tokshfl base tokshfl
