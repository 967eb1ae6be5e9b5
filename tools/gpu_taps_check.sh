# TN precomputed-tap ring: conv parity with the DMA configs forced, then per-layer A/B and the bench
set -o pipefail
for c in 7 9; do
  UNETSEG_TN_CFG=$c timeout -k 10 300 python -u -m pytest tests/test_gpu_ops.py -x -q --timeout 120 --timeout-method thread -k "conv" > gpurun_out/taps_t$c.log 2>&1 || { echo "cfg $c FAILED"; tail -30 gpurun_out/taps_t$c.log; exit 1; }
  echo "cfg $c: $(tail -1 gpurun_out/taps_t$c.log)"
done
SH="16,32,32,1024,2048,512,3,1,1 16,128,128,256,256,128,3,1,1 16,64,64,512,512,256,3,1,1 16,64,64,512,0,128,1,1,0 16,16,16,512,0,512,3,1,1"
timeout -k 10 200 python tools/conv_bench.py $SH > gpurun_out/taps_on.txt 2>&1 || exit 1
UNETSEG_TN_NO_TAPS=1 timeout -k 10 200 python tools/conv_bench.py $SH > gpurun_out/taps_off.txt 2>&1 || exit 1
echo "--- taps on"; grep -v "^W\|^E\|amdgpu.ids" gpurun_out/taps_on.txt
echo "--- taps off"; grep -v "^W\|^E\|amdgpu.ids" gpurun_out/taps_off.txt
if [ -z "$NOBENCH" ]; then
  ENVS=";UNETSEG_TN_NO_TAPS=1;" bash tools/gpu_bench_envs.sh
fi
