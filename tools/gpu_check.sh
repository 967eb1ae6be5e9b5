set -o pipefail
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > gpurun_out/gpu_tests.log 2>&1 || { echo TESTS FAILED; tail -30 gpurun_out/gpu_tests.log; exit 1; }
tail -1 gpurun_out/gpu_tests.log
timeout -k 10 300 python tools/conv_bench.py > gpurun_out/convbench.txt 2>&1
timeout -k 10 300 python bench.py --cpu-baseline 0 > gpurun_out/bench_a.json 2> gpurun_out/bench_a.err
tail -1 gpurun_out/bench_a.json | cut -c1-400
