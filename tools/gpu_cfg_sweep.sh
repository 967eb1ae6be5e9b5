# TN configuration sweep over 1x1 shapes (fwd/dgrad timings; wgrad unaffected)
SH="16,128,128,64,0,256,1,1,0 16,128,128,256,0,64,1,1,0 16,64,64,128,0,512,1,1,0 16,64,64,512,0,128,1,1,0 16,32,32,256,0,1024,1,1,0 16,32,32,1024,0,256,1,1,0 16,16,16,512,0,2048,1,1,0 16,16,16,2048,0,512,1,1,0 16,16,16,512,0,512,3,1,1"
for c in "" 1 2 3 4 5; do
  echo "== cfg=${c:-auto}"
  UNETSEG_TN_CFG=$c STATS=1 timeout -k 10 120 python tools/conv_bench.py $SH 2>&1 | grep -v amdgpu | cut -c1-100
done
