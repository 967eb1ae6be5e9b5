# interleaved C2 bench sweep of environment knobs (VARIANTS = ';'-separated "label|ENV=1 ENV2=2"), $NB rounds
set -o pipefail
cd $GRAFT_REPO_ROOT
IFS=';' read -ra VS <<< "$VARIANTS"
for i in $(seq 1 ${NB:-2}); do
  for v in "${VS[@]}"; do
    IFS='|' read -r label envs <<< "$v"
    r=$(env $envs timeout -k 10 300 python bench.py --cpu-baseline 0 --card-probe 0 --probe 0 --extra-configs 0 --steps 30 $BENCH_ARGS 2>/dev/null | tail -1 | python -c "import json,sys; d=json.load(sys.stdin); print(d['value'], d['median_gpu_ms_per_step'])") || exit 1
    echo "$label $r"
  done
done
