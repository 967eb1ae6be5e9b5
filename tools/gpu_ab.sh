#!/bin/bash
# Interleaved bench A/B/C... of environment variants on one box (no test suite):
#   tools/gpu_ab.sh ENV_A ENV_B [...]      (each variant: VAR=value pairs joined by "+", or "-" for none)
# NB rounds (default 3); BENCH_ARGS passed to bench.py; EXTRA=1 also times C4 / C5.
set -o pipefail
export TMPDIR=/tmp
ex=0
[ -n "$EXTRA" ] && ex=1
for i in $(seq 1 ${NB:-3}); do
  k=0
  for v in "$@"; do
    E="${v//+/ }"
    [ "$E" = "-" ] && E=""
    env $E timeout -k 10 300 python bench.py --cpu-baseline 0 --probe 0 --card-probe 0 --extra-configs $ex $BENCH_ARGS 2>/dev/null | tail -1 | \
      python -c "import json,sys; d=json.load(sys.stdin); c=d.get('configs',{}); print('$k', d['value'], d['median_gpu_ms_per_step'], d.get('peak_alloc_gib'), ' '.join(f'{t}={v[\"value\"]}/{v.get(\"peak_alloc_gib\")}' for t,v in c.items()), '[$v]')" || exit 1
    k=$((k+1))
  done
done
