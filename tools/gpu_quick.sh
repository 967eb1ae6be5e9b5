# conv parity tests, per-layer timings of $SH, then $NB bench runs
set -o pipefail
timeout -k 10 300 python -u -m pytest tests/test_gpu_ops.py -x -q --timeout 120 --timeout-method thread -k "conv" > gpurun_out/quick_t.log 2>&1 || { echo "TESTS FAILED"; tail -30 gpurun_out/quick_t.log; exit 1; }
echo "tests: $(tail -1 gpurun_out/quick_t.log)"
if [ -n "$SH" ]; then timeout -k 10 200 python tools/conv_bench.py $SH 2>&1 | grep -v "^W\|^E\|amdgpu.ids" || exit 1; fi
for i in $(seq 1 ${NB:-2}); do
  timeout -k 10 300 python bench.py --cpu-baseline 0 --probe 0 2>/dev/null | tail -1 | python -c "import json,sys; d=json.load(sys.stdin); print('bench', d['value'], d['ms_per_step'])" || exit 1
done
