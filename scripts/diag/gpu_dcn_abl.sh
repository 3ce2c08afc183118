cd "$GRAFT_REPO_ROOT" || exit 1
O=gpurun_out/dcnabl; mkdir -p $O
for v in abl1 abl2; do
DCN_OFFSET_STD=0 TMVS_DCN_TAG=$v TMVS_LIB_PATH=variants/$v/libtransmvs_hip.so timeout -k 10 120 python scripts/diag/dcn_time.py > $O/t_$v.txt 2>&1 || exit $?
done
DCN_OFFSET_STD=0 TMVS_DCN_TAG=prod timeout -k 10 120 python scripts/diag/dcn_time.py > $O/t_prod.txt 2>&1 || exit $?
cat $O/t_*.txt | grep us
