set -o pipefail
timeout -k 10 400 python -u -m pytest tests/test_gpu_ddp.py tests/test_gpu_fullsize.py -v -s --timeout 300 --timeout-method thread > gpurun_out/r02_ddp.log 2>&1
rc=$?
grep -E "PASSED|FAILED|ERROR|passed|failed|eval 512|train 512|loss hip|grad rel|well-cond|^E " gpurun_out/r02_ddp.log | tail -40
exit $rc
