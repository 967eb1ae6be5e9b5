cd $GRAFT_REPO_ROOT
for cfg in ${CFGS:-none 19 3 2 7 1 6}; do
  if [ $cfg = none ]; then E="X=1"; else E="UNETSEG_TN_CFG=$cfg"; fi
  echo "== $cfg"
  env $E timeout -k 10 120 python3 tools/conv_bench.py 8,512,512,128,0,32,1,1,0 8,512,512,64,0,32,1,1,0 16,128,128,256,0,64,1,1,0 2>&1 | grep -v amdgpu.ids || exit 1
done
