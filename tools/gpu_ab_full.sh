# full GPU suite, kernel stats of $KPAT, then interleaved bench A/B (A = tools/ab_old.so, B = in-tree)
set -o pipefail
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > gpurun_out/gpu_tests.log 2>&1 || { echo TESTS FAILED; tail -30 gpurun_out/gpu_tests.log; exit 1; }
tail -1 gpurun_out/gpu_tests.log
bash tools/gpu_kstat.sh || exit 1
NOTEST=1 NB=${NB:-2} TESTK=none bash tools/gpu_ab_lib.sh
