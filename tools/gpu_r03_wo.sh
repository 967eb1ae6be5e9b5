# Round 3: batched write-out loads (accumulate / post 3) -- parity, then lib A/B (A = previous build).
set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
timeout -k 10 500 python -u -m pytest -x -q --timeout 200 --timeout-method thread tests/test_gpu_configs.py tests/test_gpu_post_res.py tests/test_gpu_fusions.py tests/test_gpu_determinism.py > gpurun_out/wo_t.log 2>&1 || { grep -v "^E  *+" gpurun_out/wo_t.log | grep -B3 -A30 "FAILED\|Error" | tail -50 | cut -c1-300; exit 1; }
tail -1 gpurun_out/wo_t.log
for i in 1 2 3; do for v in A B; do
  if [ $v = A ]; then L=abl/lib_A.so; else L=unet-embroidery-seg_amd/unetseg_hip/libunetseg_hip.so; fi
  UNETSEG_TN_HALO_SPLIT=3 UNETSEG_LIB_PATH=$L timeout -k 10 200 python bench.py --cpu-baseline 0 --probe 0 --steps 20 2>/dev/null | python -c "import json,sys; d=json.loads(sys.stdin.read()); print('$v', d['value'], d['ms_per_step'])" || exit 1
done; done
echo done
