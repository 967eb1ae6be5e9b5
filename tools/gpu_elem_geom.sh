# BN reduce / apply kernels under other block counts of the reduction geometry (UNETSEG_RED_TARGET)
cd $GRAFT_REPO_ROOT
for t in 2048 1024 4096 8192; do
  echo "== RED_TARGET $t"
  UNETSEG_RED_TARGET=$t timeout -k 10 200 python3 tools/elem_bench.py 2>&1 | grep -E "plain|mbits +reduce|summed" || exit 1
done
