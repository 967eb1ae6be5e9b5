cd $GRAFT_REPO_ROOT
SH="8,256,256,128,0,128,3,1,1 8,128,128,256,0,256,3,1,1 16,128,128,128,0,128,3,1,1 16,64,64,256,0,256,3,1,1 8,64,64,512,0,512,3,1,1"
for c in none 10 7 13; do
  if [ $c = none ]; then E="X=1"; else E="UNETSEG_TN_CFG=$c"; fi
  echo "== $c"
  env $E timeout -k 10 200 python3 tools/conv_bench.py $SH 2>&1 | grep -v amdgpu.ids | cut -c1-80 || exit 1
done
