set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > gpurun_out/gpu_tests.log 2>&1 && \
timeout -k 10 300 python bench.py > gpurun_out/bench1.json 2> gpurun_out/bench1.err && \
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/prof1 -o run -- python bench.py --steps 5 --warmup 2 --cpu-baseline 0 > gpurun_out/prof1.log 2>&1
echo EXIT $?
tail -3 gpurun_out/gpu_tests.log; cat gpurun_out/bench1.json
