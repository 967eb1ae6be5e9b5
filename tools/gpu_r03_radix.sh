# Round 3: radix scatter through LDS (coalesced runs) -- Lovasz parity, then lib A/B (A = previous build).
set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
timeout -k 10 500 python -u -m pytest -x -q --timeout 200 --timeout-method thread tests/test_gpu_losses_full.py tests/test_gpu_ops.py tests/test_gpu_round2.py tests/test_gpu_targets.py tests/test_gpu_determinism.py -k "lovasz or Lovasz or loss or golden or determinism or ignore" > gpurun_out/radix_t.log 2>&1 || { grep -v "^E  *+" gpurun_out/radix_t.log | grep -B3 -A30 "FAILED\|Error" | tail -50 | cut -c1-300; exit 1; }
tail -1 gpurun_out/radix_t.log
for i in 1 2 3; do for v in A B; do
  if [ $v = A ]; then L=abl/lib_A.so; else L=unet-embroidery-seg_amd/unetseg_hip/libunetseg_hip.so; fi
  UNETSEG_TN_HALO_SPLIT=3 UNETSEG_LIB_PATH=$L timeout -k 10 200 python bench.py --cpu-baseline 0 --probe 0 --steps 20 2>/dev/null | python -c "import json,sys; d=json.loads(sys.stdin.read()); print('$v', d['value'], d['ms_per_step'])" || exit 1
done; done
timeout -k 10 200 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/radix_prof -o run -- python bench.py --steps 3 --warmup 1 --cpu-baseline 0 --probe 0 > gpurun_out/radix_prof.log 2>&1 || { echo prof failed; exit 1; }
grep -i "radix" gpurun_out/radix_prof/run_kernel_stats.csv | cut -c1-200
echo done
