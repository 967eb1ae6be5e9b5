set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
timeout -k 10 300 rocprofv3 --kernel-trace --hip-trace --output-format csv -d gpurun_out/sl -o run -- python bench.py --steps 5 --warmup 2 --cpu-baseline 0 --probe 0 > gpurun_out/sl.log 2>&1 || { echo PROF FAILED; tail -20 gpurun_out/sl.log; exit 1; }
python tools/slack.py gpurun_out/sl 30 > gpurun_out/slack.txt; cat gpurun_out/slack.txt
rm -f gpurun_out/sl/*/*hip_api_trace.csv.gz
