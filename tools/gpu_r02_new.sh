set -o pipefail
timeout -k 10 900 python -u -m pytest tests/test_gpu_round2.py -v --timeout 300 --timeout-method thread ${1:+-k "$1"} > gpurun_out/r02_new.log 2>&1
rc=$?
grep -E "PASSED|FAILED|ERROR|passed|failed|^E " gpurun_out/r02_new.log | tail -70
exit $rc
