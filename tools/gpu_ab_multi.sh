# interleaved bench of several (library, environment) variants: VARIANTS = ';'-separated entries
# "label|lib|ENV=1 ENV2=1" (lib: A = tools/ab/A/libunetseg_hip.so, B = the in-tree build), $NB rounds
set -o pipefail
cd $GRAFT_REPO_ROOT
IFS=';' read -ra VS <<< "$VARIANTS"
for i in $(seq 1 ${NB:-2}); do
  for v in "${VS[@]}"; do
    IFS='|' read -r label lib envs <<< "$v"
    if [ "$lib" = A ]; then L=tools/ab/A/libunetseg_hip.so; else L=unet-embroidery-seg_amd/unetseg_hip/libunetseg_hip.so; fi
    env UNETSEG_LIB_PATH=$L $envs timeout -k 10 300 python bench.py --cpu-baseline 0 --probe 0 $BENCH_ARGS 2>/dev/null | tail -1 | python -c "import json,sys; d=json.load(sys.stdin); print('$label', d['value'], d['ms_per_step'])" || exit 1
  done
done
