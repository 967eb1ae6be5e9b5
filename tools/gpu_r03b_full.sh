# Round 3 (second session): the whole GPU suite, smoke, one bench line and a kernel-trace profile.
set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
timeout -k 10 700 python -u -m pytest -x -v -s -rA --durations=25 --timeout 300 --timeout-method thread -m gpu tests > gpurun_out/r03b_gputest.log 2>&1 || { echo gpu tests failed; grep -v "^E  *+" gpurun_out/r03b_gputest.log | grep -B5 -A40 "FAILED\|Error" | tail -60 | cut -c1-400; exit 1; }
grep -h " passed\|failed" gpurun_out/r03b_gputest.log | tail -3
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/r03b_smoke.log 2>&1 || { echo smoke failed; tail -20 gpurun_out/r03b_smoke.log; exit 1; }
tail -3 gpurun_out/r03b_smoke.log
timeout -k 10 300 python bench.py > gpurun_out/r03b_bench.json 2> gpurun_out/r03b_bench.err || { echo bench failed; tail gpurun_out/r03b_bench.err; exit 1; }
cut -c1-700 gpurun_out/r03b_bench.json
timeout -k 10 200 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/r03b_prof -o run -- python bench.py --steps 5 --warmup 2 --cpu-baseline 0 --probe 0 > gpurun_out/r03b_prof.log 2>&1 || { echo prof failed; exit 1; }
python tools/trace_streams.py gpurun_out/r03b_prof 2 > gpurun_out/r03b_streams.txt 2>&1 || echo "streams failed"
echo done
