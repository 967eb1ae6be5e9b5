# Round 3: the 256x64 halo-A ring (<= 64 output channels): config cases, layer table, step A/B.
set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
timeout -k 10 400 python -u -m pytest -x -q --timeout 200 --timeout-method thread tests/test_gpu_configs.py tests/test_gpu_models.py > gpurun_out/hring3_t.log 2>&1 || { grep -v "^E  *+" gpurun_out/hring3_t.log | grep -B3 -A30 "FAILED\|Error" | tail -50 | cut -c1-300; exit 1; }
tail -1 gpurun_out/hring3_t.log
timeout -k 10 300 python tools/layer_table.py --top 300 > gpurun_out/hring3_layers.txt 2>&1 || { tail gpurun_out/hring3_layers.txt; exit 1; }
grep "16,256,256,64,128,64,3,3" gpurun_out/hring3_layers.txt
for i in 1 2 3; do for v in h64 no64; do
  case $v in h64) E="UNETSEG_X=0";; no64) E="UNETSEG_TN_CFG_NO22=1";; esac
  env $E timeout -k 10 200 python bench.py --cpu-baseline 0 --probe 0 --steps 20 2>/dev/null | python -c "import json,sys; d=json.loads(sys.stdin.read()); print('$v', d['value'], d['ms_per_step'])" || exit 1
done; done
echo done
