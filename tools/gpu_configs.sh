# C4 / C5 bench lines (BASELINE.json configs[3], configs[4] at one GPU) + a kernel-stats profile of C4
set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
timeout -k 10 400 python bench.py --model attention_unet --batch 8 --cpu-batch 2 > gpurun_out/bench_c4.json 2> gpurun_out/bench_c4.err || { echo C4 FAILED; tail -20 gpurun_out/bench_c4.err; exit 1; }
tail -1 gpurun_out/bench_c4.json | cut -c1-300
timeout -k 10 400 python bench.py --model multitask_unet --batch 8 --loss bce --cpu-batch 4 > gpurun_out/bench_c5.json 2> gpurun_out/bench_c5.err || { echo C5 FAILED; tail -20 gpurun_out/bench_c5.err; exit 1; }
tail -1 gpurun_out/bench_c5.json | cut -c1-300
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/c4prof -o run -- python bench.py --model attention_unet --batch 8 --steps 5 --warmup 2 --cpu-baseline 0 > gpurun_out/c4prof.log 2>&1 || { echo PROF FAILED; tail -20 gpurun_out/c4prof.log; exit 1; }
D=$(dirname $(find gpurun_out/c4prof -name run_kernel_trace.csv | head -1))
python tools/prof_summary.py $D 8 40 > gpurun_out/c4_kernel_stats_summary.txt && python tools/trace_streams.py $D 4 > gpurun_out/c4_streams.txt
head -5 gpurun_out/c4_kernel_stats_summary.txt
UNETSEG_PROBE_DUMP=gpurun_out/c4_probe.txt timeout -k 10 300 python bench.py --model attention_unet --batch 8 --steps 2 --warmup 1 --cpu-baseline 0 > /dev/null 2>&1 || exit 1
rm -f $D/run_kernel_trace.csv
