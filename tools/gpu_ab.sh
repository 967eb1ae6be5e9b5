# bench A/B: BENCH_A / BENCH_B are extra bench.py args (or env prefixes); tests first unless NOTEST=1
set -o pipefail
if [ -z "$NOTEST" ]; then
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > gpurun_out/gpu_tests.log 2>&1 || { echo TESTS FAILED; tail -30 gpurun_out/gpu_tests.log; exit 1; }
tail -2 gpurun_out/gpu_tests.log
fi
eval "$ENV_A timeout -k 10 300 python bench.py --cpu-baseline 0 $BENCH_A" > gpurun_out/bench_a.json 2> gpurun_out/bench_a.err && \
eval "$ENV_B timeout -k 10 300 python bench.py --cpu-baseline 0 $BENCH_B" > gpurun_out/bench_b.json 2> gpurun_out/bench_b.err
rc=$?
python - <<'PY'
import json
for f in ("a", "b"):
    try:
        d = json.loads(open(f"gpurun_out/bench_{f}.json").read().strip().splitlines()[-1])
        print(f, d["value"], "img/s", d["ms_per_step"], "ms", {k: v["ms_per_step"] for k, v in d["roofline"]["kernels"].items()})
    except Exception as e:
        print(f, "failed", e)
PY
exit $rc
