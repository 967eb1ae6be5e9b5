# Round 3: halo-A ring (UNETSEG_TN_HALO=1) parity cases, per-layer table and step A/B against the gather ring.
set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest -x -v --timeout 120 --timeout-method thread tests/test_gpu_configs.py -k "halo_ring or ring256x128" > gpurun_out/hring_t.log 2>&1 || { grep -v "^E  *+" gpurun_out/hring_t.log | grep -B3 -A30 "FAILED\|Error" | tail -50 | cut -c1-300; exit 1; }
grep -c PASSED gpurun_out/hring_t.log
UNETSEG_TN_HALO=1 timeout -k 10 300 python tools/layer_table.py --top 300 > gpurun_out/hring_layers.txt 2>&1 || { tail gpurun_out/hring_layers.txt; exit 1; }
for i in 1 2 3; do for v in base hring; do
  case $v in base) E="UNETSEG_X=0";; hring) E="UNETSEG_TN_HALO=1";; esac
  env $E timeout -k 10 200 python bench.py --cpu-baseline 0 --probe 0 --steps 20 2>/dev/null | python -c "import json,sys; d=json.loads(sys.stdin.read()); print('$v', d['value'], d['ms_per_step'])" || exit 1
done; done
echo done
