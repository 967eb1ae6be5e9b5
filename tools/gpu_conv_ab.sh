# isolated conv timings (tools/conv_bench.py, STATS/ACC as the bench calls use them) under two library
# environments, then an interleaved bench A/B: ENV_A / ENV_B, SHAPES (conv_bench shape list)
cd $GRAFT_REPO_ROOT
for v in A B; do
  if [ $v = A ]; then E="$ENV_A"; else E="$ENV_B"; fi
  echo "== $v ($E)"
  env $E STATS=1 timeout -k 10 120 python tools/conv_bench.py $SHAPES 2>&1 | grep -v amdgpu | cut -c1-130 || exit 1
done
NOTEST=1 NB=${NB:-3} bash tools/gpu_ab_env.sh
