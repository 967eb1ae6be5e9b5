# isolated upsample timings (tools/up_bench.py): tools/ab/A/ (library + fast-call binding) vs the tree's library, interleaved
cd $GRAFT_REPO_ROOT
for i in 1 2; do
echo "== A"; UNETSEG_LIB_PATH=tools/ab/A/libunetseg_hip.so timeout -k 10 120 python tools/up_bench.py 2>&1 | grep H= || exit 1
echo "== B"; timeout -k 10 120 python tools/up_bench.py 2>&1 | grep H= || exit 1
done
