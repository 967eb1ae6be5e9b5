# LDS-DMA ring issue stagger (UNETSEG_TN_SCHED) A/B: parity of the ring cases, layer table, step
set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
UNETSEG_TN_SCHED=1 timeout -k 10 300 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_gpu_configs.py -k "ring" > gpurun_out/ts_t.log 2>&1 || { tail -30 gpurun_out/ts_t.log; exit 1; }
tail -1 gpurun_out/ts_t.log
for v in 0 1; do
  UNETSEG_TN_SCHED=$v timeout -k 10 300 python tools/layer_table.py --top 200 > gpurun_out/layers_s$v.txt 2>&1 || exit 1
  echo "== sched $v"; head -14 gpurun_out/layers_s$v.txt | tail -11; grep TOTAL gpurun_out/layers_s$v.txt
done
for i in 1 2; do for v in 0 1; do
  UNETSEG_TN_SCHED=$v timeout -k 10 200 python bench.py --cpu-baseline 0 --probe 0 --steps 20 2>/dev/null | python -c "import json,sys; d=json.loads(sys.stdin.read()); print('sched $v', d['value'], d['ms_per_step'])"
done; done
