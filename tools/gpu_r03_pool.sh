# Round 3: specialised 3x3 stride-2 maxpool kernels (stem pool): parity vs the generic kernels, A/B.
set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest -x -v --timeout 200 --timeout-method thread tests/test_gpu_maxpool.py tests/test_gpu_ops.py -k "maxpool" > gpurun_out/pool_t.log 2>&1 || { grep -v "^E  *+" gpurun_out/pool_t.log | grep -B3 -A30 "FAILED\|Error" | tail -50 | cut -c1-300; exit 1; }
grep -c PASSED gpurun_out/pool_t.log
timeout -k 10 200 rocprofv3 --kernel-trace --stats -d gpurun_out/pool_prof -o run -- python bench.py --cpu-baseline 0 --probe 0 --steps 5 --warmup 2 > gpurun_out/pool_prof.log 2>&1 || { tail -20 gpurun_out/pool_prof.log; exit 1; }
grep -h "maxpool" gpurun_out/pool_prof/*kernel_stats.csv | cut -d, -f1-4 || true
for i in 1 2 3; do for v in on generic; do
  case $v in on) E="UNETSEG_X=0";; generic) E="UNETSEG_MAXPOOL_GENERIC=1";; esac
  env $E timeout -k 10 200 python bench.py --cpu-baseline 0 --probe 0 --steps 20 2>/dev/null | python -c "import json,sys; d=json.loads(sys.stdin.read()); print('$v', d['value'], d['ms_per_step'])" || exit 1
done; done
echo done
