# Round 3: halo-A ring as the default -- config cases (both rings), model / full-size / fusion /
# overlap / determinism tests, then a step A/B of the weight-ring depth (3 vs 4 stages).
set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest -x -q --timeout 200 --timeout-method thread tests/test_gpu_configs.py tests/test_gpu_models.py tests/test_gpu_fusions.py tests/test_gpu_overlap.py tests/test_gpu_determinism.py tests/test_gpu_fullsize.py tests/test_gpu_c4c5.py > gpurun_out/hring2_t.log 2>&1 || { grep -v "^E  *+" gpurun_out/hring2_t.log | grep -B3 -A30 "FAILED\|Error" | tail -50 | cut -c1-300; exit 1; }
tail -1 gpurun_out/hring2_t.log
UNETSEG_TN_HALO_NS4=1 timeout -k 10 300 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_gpu_configs.py -k "halo_ring" > gpurun_out/hring2_ns4.log 2>&1 || { tail -30 gpurun_out/hring2_ns4.log; exit 1; }
tail -1 gpurun_out/hring2_ns4.log
for i in 1 2 3; do for v in ns3 ns4 gather; do
  case $v in ns3) E="UNETSEG_X=0";; ns4) E="UNETSEG_TN_HALO_NS4=1";; gather) E="UNETSEG_TN_NO_HALO_RING=1";; esac
  env $E timeout -k 10 200 python bench.py --cpu-baseline 0 --probe 0 --steps 20 2>/dev/null | python -c "import json,sys; d=json.loads(sys.stdin.read()); print('$v', d['value'], d['ms_per_step'])" || exit 1
done; done
echo done
