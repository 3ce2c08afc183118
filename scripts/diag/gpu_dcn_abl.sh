cd "$GRAFT_REPO_ROOT" || exit 1
for v in abl1 abl2; do
DCN_FUSED=1 DCN_OFFSET_STD=0 TMVS_DCN_TAG=$v TMVS_LIB_PATH=variants/$v/libtransmvs_hip.so timeout -k 10 120 python scripts/diag/dcn_time.py 2>&1 | grep us || exit 1
done
DCN_FUSED=1 DCN_OFFSET_STD=0 TMVS_DCN_TAG=prod timeout -k 10 120 python scripts/diag/dcn_time.py 2>&1 | grep us
