# full GPU test suite (one process), then $NB bench runs
set -o pipefail
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > gpurun_out/full_t.log 2>&1 || { echo "TESTS FAILED"; tail -40 gpurun_out/full_t.log; exit 1; }
echo "tests: $(tail -1 gpurun_out/full_t.log)"
for i in $(seq 1 ${NB:-2}); do
  timeout -k 10 300 python bench.py --cpu-baseline 0 --probe 0 2>/dev/null | tail -1 | python -c "import json,sys; d=json.load(sys.stdin); print('bench', d['value'], d['ms_per_step'])" || exit 1
done
