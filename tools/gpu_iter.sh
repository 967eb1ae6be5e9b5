# one iteration of kernel work: selected GPU tests ($TESTS, pytest -k $TESTK), bench line, kernel
# durations of $KPAT under rocprofv3 kernel-trace
set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
if [ -n "$TESTS" ]; then
  timeout -k 10 400 python -u -m pytest $TESTS -x -q --timeout 150 --timeout-method thread ${TESTK:+-k "$TESTK"} > gpurun_out/iter_t.log 2>&1 || { echo TESTS FAILED; tail -40 gpurun_out/iter_t.log; exit 1; }
  echo "tests: $(tail -1 gpurun_out/iter_t.log)"
fi
for i in $(seq 1 ${NB:-1}); do
timeout -k 10 300 python bench.py --cpu-baseline 0 --probe 0 $BENCH_ARGS 2>gpurun_out/iter_b.err | tail -1 | python -c "import json,sys; d=json.load(sys.stdin); print('bench', d['value'], d['ms_per_step'])" || { tail gpurun_out/iter_b.err; exit 1; }
done
[ -n "$KPAT" ] && KPAT="$KPAT" bash tools/gpu_kstat.sh
exit 0
