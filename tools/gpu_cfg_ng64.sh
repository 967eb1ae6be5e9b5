# the 192 -> 64 3x3 concat conv at 256x256 (up_concat1.conv1) under the Ng <= 64 TN configurations
cd $GRAFT_REPO_ROOT
for c in auto 11 12 14 6 20; do
  echo "== cfg=$c"
  if [ "$c" = auto ]; then cc=""; else cc=$c; fi
  UNETSEG_TN_CFG=$cc timeout -k 10 120 python tools/conv_bench.py 16,256,256,64,128,64,3,1,1 2>&1 | grep -v amdgpu | cut -c1-110 || exit 1
done
