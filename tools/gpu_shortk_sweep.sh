# short-K 1x1 conv shapes of the ResNet-50 encoder under several TN configurations
cd $GRAFT_REPO_ROOT
SH="16,128,128,64,0,256,1,1,0 16,128,128,256,0,64,1,1,0 16,128,128,256,0,128,1,1,0 16,64,64,128,0,512,1,1,0 16,64,64,512,0,128,1,1,0 16,32,32,256,0,1024,1,1,0 16,32,32,1024,0,256,1,1,0 16,16,16,512,0,2048,1,1,0 16,16,16,2048,0,512,1,1,0"
for c in auto 3 5 6 8 10 12 13; do
  echo "== cfg=$c"
  if [ "$c" = auto ]; then cc=""; else cc=$c; fi
  UNETSEG_TN_CFG=$cc STATS=1 timeout -k 10 120 python tools/conv_bench.py $SH 2>&1 | grep -v amdgpu | cut -c1-100 || exit 1
done
