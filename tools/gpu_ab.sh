# A/B of the bench (overlap on / off) after the GPU test suite; run from the repo root on the box
set -o pipefail
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > gpurun_out/gpu_tests.log 2>&1 || { echo TESTS FAILED; tail -30 gpurun_out/gpu_tests.log; exit 1; }
tail -2 gpurun_out/gpu_tests.log
timeout -k 10 300 python bench.py --cpu-baseline 0 > gpurun_out/bench_on.json 2> gpurun_out/bench_on.err && \
UNETSEG_NO_OVERLAP=1 timeout -k 10 300 python bench.py --cpu-baseline 0 > gpurun_out/bench_off.json 2> gpurun_out/bench_off.err
rc=$?
python - <<'PY'
import json
for f in ("on", "off"):
    try:
        d = json.loads(open(f"gpurun_out/bench_{f}.json").read().strip().splitlines()[-1])
        print(f, d["value"], "img/s", d["ms_per_step"], "ms", {k: v["ms_per_step"] for k, v in d["roofline"]["kernels"].items()})
    except Exception as e:
        print(f, "failed", e)
PY
exit $rc
