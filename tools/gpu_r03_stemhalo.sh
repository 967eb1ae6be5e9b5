# Round 3: the ResNet stem forward on a persistent-halo kernel: parity (float64 reference, BN partials),
# coverage, per-kernel time, A/B against the TN stem (UNETSEG_STEM_TN=1).
set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
timeout -k 10 400 python -u -m pytest -x -v --timeout 200 --timeout-method thread tests/test_gpu_configs.py tests/test_gpu_models.py -k "stem or covered or unet_resnet50" > gpurun_out/stemh_t.log 2>&1 || { grep -v "^E  *+" gpurun_out/stemh_t.log | grep -B3 -A30 "FAILED\|Error" | tail -50 | cut -c1-300; exit 1; }
grep -c PASSED gpurun_out/stemh_t.log
timeout -k 10 200 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/stemh_prof -o run -- python bench.py --cpu-baseline 0 --probe 0 --steps 5 --warmup 2 > gpurun_out/stemh_prof.log 2>&1 || { tail -20 gpurun_out/stemh_prof.log; exit 1; }
grep -h "stem\|maxpool" gpurun_out/stemh_prof/run_kernel_stats.csv | cut -d, -f1-4 || true
for i in 1 2 3; do for v in on tn; do
  case $v in on) E="UNETSEG_X=0";; tn) E="UNETSEG_STEM_TN=1";; esac
  env $E timeout -k 10 200 python bench.py --cpu-baseline 0 --probe 0 --steps 20 2>/dev/null | python -c "import json,sys; d=json.loads(sys.stdin.read()); print('$v', d['value'], d['ms_per_step'])" || exit 1
done; done
echo done
