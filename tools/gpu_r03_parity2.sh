# Round 3: full-size / DP tests (prints kept: -s), smoke, one bench line, a kernel trace.
set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
T="python -u -m pytest -x -v -s --timeout 600 --timeout-method thread -m gpu"
timeout -k 10 900 $T tests/test_gpu_fullsize.py tests/test_gpu_ddp.py tests/test_gpu_c4c5.py -k "fullsize or ddp or train_step or golden" > gpurun_out/r03a_tests2.log 2>&1 || { echo tests2 failed; grep -v "^E  *+" gpurun_out/r03a_tests2.log | tail -40 | cut -c1-400; exit 1; }
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/r03a_smoke.log 2>&1 || { echo smoke failed; tail -20 gpurun_out/r03a_smoke.log; exit 1; }
timeout -k 10 400 python bench.py > gpurun_out/r03a_bench.json 2> gpurun_out/r03a_bench.err || { echo bench failed; tail gpurun_out/r03a_bench.err; exit 1; }
timeout -k 10 300 rocprofv3 --kernel-trace --output-format csv -d gpurun_out/r03a_prof -o run -- python bench.py --steps 3 --warmup 1 --cpu-baseline 0 --probe 0 > gpurun_out/r03a_prof.log 2>&1 || { echo prof failed; exit 1; }
grep -h "PASS\|FAIL\|attention_unet 512\|unet_plain 128\|train 512\|fp32 512\|grad rel\|hip-emu\|loss hip\|worst 4\|well-cond" gpurun_out/r03a_tests2.log | cut -c1-300
tail -3 gpurun_out/r03a_smoke.log
cut -c1-600 gpurun_out/r03a_bench.json
