# 3x3 decoder / encoder layers under forced TN configurations (isolated conv_bench, BN stats on)
cd $GRAFT_REPO_ROOT
SH="16,128,128,128,0,128,3,1,1 16,64,64,256,0,256,3,1,1 16,32,32,512,0,512,3,1,1 16,128,128,256,256,128,3,1,1 16,64,64,128,0,128,3,1,1"
for c in auto 3 8 10 19; do
  echo "== cfg=$c"
  if [ "$c" = auto ]; then cc=""; else cc=$c; fi
  UNETSEG_TN_CFG=$cc STATS=1 timeout -k 10 120 python tools/conv_bench.py $SH 2>&1 | grep -v amdgpu | cut -c1-110 || exit 1
done
