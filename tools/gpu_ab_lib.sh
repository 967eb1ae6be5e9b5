# pack test + interleaved bench A/B: A = tools/ab_old.so, B = the in-tree build; $NB rounds
set -o pipefail
[ -n "$NOTEST" ] || timeout -k 10 300 python -u -m pytest tests/test_gpu_ops.py -x -q --timeout 120 --timeout-method thread -k "${TESTK:-pack}" > gpurun_out/ab_t.log 2>&1 || { echo TESTS FAILED; tail -30 gpurun_out/ab_t.log; exit 1; }
[ -n "$NOTEST" ] || echo "tests: $(tail -1 gpurun_out/ab_t.log)"
for i in $(seq 1 ${NB:-2}); do
  for v in A B; do
    if [ $v = A ]; then L=tools/ab_old.so; else L=unet-embroidery-seg_amd/unetseg_hip/libunetseg_hip.so; fi
    UNETSEG_LIB_PATH=$L timeout -k 10 300 python bench.py --cpu-baseline 0 --probe 0 $BENCH_ARGS 2>/dev/null | tail -1 | python -c "import json,sys; d=json.load(sys.stdin); print('$v', d['value'], d['ms_per_step'])" || exit 1
  done
done
