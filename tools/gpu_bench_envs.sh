# bench under several env settings (ENVS separated by ';', an empty entry = defaults), one line each
#   ENVS=";UNETSEG_HALO_WG_MAXG=128;UNETSEG_WG_BLOCKS=256" bash tools/gpu_bench_envs.sh
IFS=';' read -ra ARR <<< "$ENVS"
for e in "${ARR[@]}"; do
  r=$(eval "env $e timeout -k 10 300 python bench.py --cpu-baseline 0 --probe 0" 2>/dev/null | tail -1 | python -c "import json,sys; d=json.load(sys.stdin); print(d['value'], d['ms_per_step'])")
  echo "[$e] $r"
done
