# Round 3 (end): the whole GPU suite and smoke, then the C2 profile set (bench line, kernel stats,
# PMC traffic / MFMA busy, streams, configs, gaps), the C4 / C5 bench lines, stem A/B.
set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest -x -v -rA --timeout 300 --timeout-method thread -m gpu tests > gpurun_out/r03_gputest.log 2>&1 || { echo gpu tests failed; grep -v "^E  *+" gpurun_out/r03_gputest.log | grep -B5 -A40 "FAILED\|Error\|error" | tail -60 | cut -c1-400; exit 1; }
tail -1 gpurun_out/r03_gputest.log
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/r03_smoke.log 2>&1 || { echo smoke failed; tail -20 gpurun_out/r03_smoke.log; exit 1; }
tail -2 gpurun_out/r03_smoke.log
bash tools/gpu_profile_round.sh r03 unet_resnet50 16 lovasz_hinge || exit 1
python tools/trace_gaps.py gpurun_out/r03_prof 4 > gpurun_out/r03_gaps.txt 2>&1 || echo "gaps failed"
timeout -k 10 200 python bench.py --model attention_unet --batch 8 > gpurun_out/r03_attention_bench.json 2> gpurun_out/r03_attention_bench.err || { echo C4 bench failed; exit 1; }
timeout -k 10 200 python bench.py --model multitask_unet --batch 8 > gpurun_out/r03_multitask_bench.json 2> gpurun_out/r03_multitask_bench.err || { echo C5 bench failed; exit 1; }
cut -c1-160 gpurun_out/r03_attention_bench.json gpurun_out/r03_multitask_bench.json
grep -h "stem_halo\|maxpool" gpurun_out/r03_prof/run_kernel_stats.csv | cut -d, -f1-4 || true
for i in 1 2; do for v in on tn; do
  case $v in on) E="UNETSEG_X=0";; tn) E="UNETSEG_STEM_TN=1";; esac
  env $E timeout -k 10 200 python bench.py --cpu-baseline 0 --probe 0 --steps 20 2>/dev/null | python -c "import json,sys; d=json.loads(sys.stdin.read()); print('$v', d['value'], d['ms_per_step'])" || exit 1
done; done
echo done
