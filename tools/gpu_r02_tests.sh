# round 2: the new full-size / configuration parity tests (args: pytest -k filter, optional)
set -o pipefail
K=${1:-}
timeout -k 10 900 python -u -m pytest tests/test_gpu_configs.py tests/test_gpu_losses_full.py tests/test_gpu_fullsize.py -v -s --timeout 300 --timeout-method thread ${K:+-k "$K"} > gpurun_out/r02_tests.log 2>&1
rc=$?
grep -E "PASSED|FAILED|ERROR|passed|failed|eval 512|train 512|loss hip|grad rel|^  [a-z]|^E " gpurun_out/r02_tests.log | tail -80
exit $rc
