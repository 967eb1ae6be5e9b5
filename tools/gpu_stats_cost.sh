# cost of the BN-statistics epilogue on short-K 1x1 convs: conv_bench with and without STATS
cd $GRAFT_REPO_ROOT
SH="16,128,128,64,0,256,1,1,0 16,128,128,256,0,64,1,1,0 16,64,64,128,0,512,1,1,0 16,32,32,256,0,1024,1,1,0 16,128,128,64,0,64,3,1,1 16,64,64,512,512,256,3,1,1"
for st in 0 1; do
  echo "== STATS=$st"
  STATS=$st timeout -k 10 120 python tools/conv_bench.py $SH 2>&1 | grep -v amdgpu | cut -c1-64 || exit 1
done
