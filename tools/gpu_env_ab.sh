# interleaved bench A/B of one library build under two environments: A as is, B with $ENV_B
# (e.g. ENV_B="UNETSEG_RED_TARGET=512"), C2 + C4 + C5 in one bench process per arm, $NB rounds
set -o pipefail
cd $GRAFT_REPO_ROOT
for i in $(seq 1 ${NB:-2}); do
  for v in A B; do
    if [ $v = A ]; then E=""; else E="$ENV_B"; fi
    env $E timeout -k 10 400 python bench.py --cpu-baseline 0 --probe 0 --card-probe 0 $BENCH_ARGS 2>/dev/null | tail -1 | python -c "
import json,sys; d=json.load(sys.stdin); c=d.get('configs') or {}
print('$v', d['value'], d['ms_per_step'], ' '.join(f'{k} {v[\"value\"]}' for k, v in c.items()), flush=True)" || exit 1
  done
done
