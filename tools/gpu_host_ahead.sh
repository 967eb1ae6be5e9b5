cd $GRAFT_REPO_ROOT
for v in "" "ROC_SIGNAL_POOL_SIZE=16384" "DEBUG_CLR_MAX_BATCH_SIZE=1024" "AMD_DIRECT_DISPATCH=0"; do
echo "== $v"; eval "$v timeout -k 10 120 python tools/host_ahead.py" 2>&1 | grep step | tail -4
done
