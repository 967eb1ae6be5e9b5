set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
timeout -k 10 300 rocprofv3 --kernel-trace --output-format csv -d gpurun_out/gp -o run -- python bench.py --steps 5 --warmup 2 --cpu-baseline 0 --probe 0 > gpurun_out/gp.log 2>&1 || { echo PROF FAILED; tail -20 gpurun_out/gp.log; exit 1; }
D=$(dirname $(find gpurun_out/gp -name run_kernel_trace.csv | head -1))
python tools/gaps.py $D 40 > gpurun_out/gaps.txt
python tools/tail_gap.py $D 30 >> gpurun_out/gaps.txt
python tools/trace_streams.py $D 4 > gpurun_out/streams.txt
cat gpurun_out/gaps.txt | head -80
