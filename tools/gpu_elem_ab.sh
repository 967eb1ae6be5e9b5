# BN kernel microbench (tools/elem_bench.py) for the library builds A (tools/ab/A) and B (in-tree)
cd $GRAFT_REPO_ROOT
for v in A B; do
  if [ $v = B ]; then L=unet-embroidery-seg_amd/unetseg_hip/libunetseg_hip.so; else L=tools/ab/$v/libunetseg_hip.so; fi
  echo "== $v"
  UNETSEG_LIB_PATH=$L timeout -k 10 200 python3 tools/elem_bench.py 2>&1 | grep -i "finalize (" || exit 1
done
