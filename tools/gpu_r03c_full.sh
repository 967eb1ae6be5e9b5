# Round 3 (end): the whole GPU suite (prints kept for the full-size / model tests) and smoke.
set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
timeout -k 10 1000 python -u -m pytest -x -v -rA --timeout 600 --timeout-method thread -m gpu tests > gpurun_out/r03_gputest.log 2>&1 || { echo gpu tests failed; grep -v "^E  *+" gpurun_out/r03_gputest.log | grep -B5 -A40 "FAILED\|Error\|error" | tail -60 | cut -c1-400; exit 1; }
grep -h "attention_unet 512\|unet_plain 128\|train 512\|fp32 512\|grad rel\|hip-emu\|loss hip\|worst 4\|well-cond\| passed\|failed" gpurun_out/r03_gputest.log | cut -c1-300
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/r03_smoke.log 2>&1 || { echo smoke failed; tail -20 gpurun_out/r03_smoke.log; exit 1; }
tail -3 gpurun_out/r03_smoke.log
echo done
