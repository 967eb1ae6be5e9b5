# Round 3: halo-A ring with the next chunk's halo DMA split over taps 0/3/6 (UNETSEG_TN_HALO_SPLIT=3): parity + A/B.
set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
UNETSEG_TN_HALO_SPLIT=3 timeout -k 10 300 python -u -m pytest -x -q --timeout 200 --timeout-method thread tests/test_gpu_configs.py -k "halo_ring or covered" > gpurun_out/split_t.log 2>&1 || { grep -v "^E  *+" gpurun_out/split_t.log | grep -B3 -A30 "FAILED\|Error" | tail -50 | cut -c1-300; exit 1; }
tail -1 gpurun_out/split_t.log
for i in 1 2 3; do for v in one three; do
  case $v in one) E="UNETSEG_X=0";; three) E="UNETSEG_TN_HALO_SPLIT=3";; esac
  env $E timeout -k 10 200 python bench.py --cpu-baseline 0 --probe 0 --steps 20 2>/dev/null | python -c "import json,sys; d=json.loads(sys.stdin.read()); print('$v', d['value'], d['ms_per_step'])" || exit 1
done; done
echo done
