# interleaved bench A/B of two library builds over C2 and the extra configurations (C4, C5) of one
# bench run per arm: A = ${LIB_A:-tools/ab/A/libunetseg_hip.so}, B = the in-tree build ($NB rounds)
set -o pipefail
cd $GRAFT_REPO_ROOT
for i in $(seq 1 ${NB:-2}); do
  for v in A B; do
    if [ $v = A ]; then L=${LIB_A:-tools/ab/A/libunetseg_hip.so}; else L=unet-embroidery-seg_amd/unetseg_hip/libunetseg_hip.so; fi
    UNETSEG_LIB_PATH=$L timeout -k 10 400 python bench.py --cpu-baseline 0 --probe 0 --card-probe 0 $BENCH_ARGS 2>/dev/null | tail -1 | python -c "
import json,sys; d=json.load(sys.stdin); c=d.get('configs') or {}
print('$v', d['value'], d['ms_per_step'], ' '.join(f'{k} {v[\"value\"]}' for k, v in c.items()), flush=True)" || exit 1
  done
done
