# Round 3: the whole GPU suite (prints kept for the full-size / model tests), smoke, bench, kernel trace.
set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
timeout -k 10 1000 python -u -m pytest -x -v -rA --timeout 600 --timeout-method thread -m gpu tests > gpurun_out/r03_gputest.log 2>&1 || { echo gpu tests failed; grep -v "^E  *+" gpurun_out/r03_gputest.log | grep -B5 -A40 "FAILED\|Error\|error" | tail -60 | cut -c1-400; exit 1; }
grep -h "attention_unet 512\|unet_plain 128\|train 512\|fp32 512\|grad rel\|hip-emu\|loss hip\|worst 4\|well-cond\| passed\|failed" gpurun_out/r03_gputest.log | cut -c1-300
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/r03a_smoke.log 2>&1 || { echo smoke failed; tail -20 gpurun_out/r03a_smoke.log; exit 1; }
tail -3 gpurun_out/r03a_smoke.log
timeout -k 10 400 python bench.py > gpurun_out/r03a_bench.json 2> gpurun_out/r03a_bench.err || { echo bench failed; tail gpurun_out/r03a_bench.err; exit 1; }
cut -c1-600 gpurun_out/r03a_bench.json
timeout -k 10 300 rocprofv3 --kernel-trace --output-format csv -d gpurun_out/r03a_prof -o run -- python bench.py --steps 3 --warmup 1 --cpu-baseline 0 --probe 0 > gpurun_out/r03a_prof.log 2>&1 || { echo prof failed; exit 1; }
echo done
timeout -k 10 300 python tools/layer_table.py --top 80 > gpurun_out/r03a_layers.txt 2>&1 || echo "layer table failed"
python tools/trace_gaps.py gpurun_out/r03a_prof 2 > gpurun_out/r03a_gaps.txt 2>&1 || echo "gaps failed"
python tools/trace_streams.py gpurun_out/r03a_prof 2 > gpurun_out/r03a_streams.txt 2>&1 || echo "streams failed"
