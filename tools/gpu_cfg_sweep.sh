# TN configuration sweep (fwd/dgrad timings) over $SH shapes for configs $CFGS
for c in $CFGS; do
  echo "== cfg=$c"
  if [ "$c" = auto ]; then cc=""; else cc=$c; fi
  UNETSEG_TN_CFG=$cc STATS=1 timeout -k 10 120 python tools/conv_bench.py $SH 2>&1 | grep -v amdgpu | cut -c1-82
done
