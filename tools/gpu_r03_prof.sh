# Round 3: bench line + kernel trace of the current build.
set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
TAG=${TAG:-r03c}
timeout -k 10 300 python bench.py --cpu-baseline 0 > gpurun_out/${TAG}_bench.json 2> gpurun_out/${TAG}_bench.err || { tail gpurun_out/${TAG}_bench.err; exit 1; }
cut -c1-300 gpurun_out/${TAG}_bench.json
timeout -k 10 200 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/${TAG}_prof -o run -- python bench.py --steps 5 --warmup 2 --cpu-baseline 0 --probe 0 > gpurun_out/${TAG}_prof.log 2>&1 || { echo prof failed; tail gpurun_out/${TAG}_prof.log; exit 1; }
UNETSEG_PROBE_DUMP=gpurun_out/${TAG}_probe_ov.txt timeout -k 10 200 python bench.py --cpu-baseline 0 --steps 3 > /dev/null 2>&1 || { echo probe failed; exit 1; }
echo done
