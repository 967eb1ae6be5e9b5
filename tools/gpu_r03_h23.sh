# Round 3: 128x128 halo-A ring (config 23) parity + A/B; multitask_unet at B=8 vs B=16 (C5 efficiency).
set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
timeout -k 10 500 python -u -m pytest -x -q --timeout 200 --timeout-method thread tests/test_gpu_configs.py tests/test_gpu_models.py > gpurun_out/h23_t.log 2>&1 || { grep -v "^E  *+" gpurun_out/h23_t.log | grep -B3 -A30 "FAILED\|Error" | tail -50 | cut -c1-300; exit 1; }
tail -1 gpurun_out/h23_t.log
for i in 1 2 3; do for v in h23 no23; do
  case $v in h23) E="UNETSEG_X=0";; no23) E="UNETSEG_TN_CFG_NO23=1";; esac
  env $E timeout -k 10 200 python bench.py --cpu-baseline 0 --probe 0 --steps 20 2>/dev/null | python -c "import json,sys; d=json.loads(sys.stdin.read()); print('$v', d['value'], d['ms_per_step'])" || exit 1
done; done
for b in 8 16; do
  timeout -k 10 200 python bench.py --model multitask_unet --batch $b --loss bce --cpu-baseline 0 --probe 0 --steps 20 2>/dev/null | python -c "import json,sys; d=json.loads(sys.stdin.read()); print('multitask B=$b', d['value'], d['ms_per_step'])" || exit 1
  timeout -k 10 200 python bench.py --model unet_resnet50 --batch $b --cpu-baseline 0 --probe 0 --steps 20 2>/dev/null | python -c "import json,sys; d=json.loads(sys.stdin.read()); print('unet_resnet50 B=$b', d['value'], d['ms_per_step'])" || exit 1
  timeout -k 10 200 python bench.py --model unet_resnet50 --batch $b --loss bce --cpu-baseline 0 --probe 0 --steps 20 2>/dev/null | python -c "import json,sys; d=json.loads(sys.stdin.read()); print('unet_resnet50 bce B=$b', d['value'], d['ms_per_step'])" || exit 1
done
echo done
