# full GPU suite, then interleaved bench A/B on the in-tree build: A runs with $ENV_A, B with $ENV_B
set -o pipefail
if [ -z "$NOTEST" ]; then
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > gpurun_out/gpu_tests.log 2>&1 || { echo TESTS FAILED; tail -30 gpurun_out/gpu_tests.log; exit 1; }
tail -1 gpurun_out/gpu_tests.log
fi
for i in $(seq 1 ${NB:-2}); do
  for v in A B; do
    if [ $v = A ]; then E="$ENV_A"; else E="$ENV_B"; fi
    env $E timeout -k 10 300 python bench.py --cpu-baseline 0 --probe 0 $BENCH_ARGS 2>/dev/null | tail -1 | python -c "import json,sys; d=json.load(sys.stdin); print('$v', d['value'], d['ms_per_step'])" || exit 1
  done
done
