# interleaved bench A/B/C.. of one library build under several environments, $NB rounds:
#   ARMS="base=;serial512=UNETSEG_WG_SERIAL_HW=262144" BENCH_ARGS="--model attention_unet --batch 8"
# (arm = name=ENV [ENV ...]; an empty ENV runs the defaults)
set -o pipefail
cd $GRAFT_REPO_ROOT
IFS=';' read -ra AR <<< "$ARMS"
for i in $(seq 1 ${NB:-2}); do
  for arm in "${AR[@]}"; do
    name=${arm%%=*}; E=${arm#*=}
    env $E timeout -k 10 400 python bench.py --cpu-baseline 0 --probe 0 --card-probe 0 $BENCH_ARGS 2>/dev/null | tail -1 | python -c "
import json,sys; d=json.load(sys.stdin); c=d.get('configs') or {}
print('$name', d['value'], d['ms_per_step'], ' '.join(f'{k} {v[\"value\"]}' for k, v in c.items()), flush=True)" || exit 1
  done
done
