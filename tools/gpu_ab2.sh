# parity (conv + stem tests), per-layer timings of $SH with and without $ENVB, then interleaved bench A/B
set -o pipefail
timeout -k 10 300 python -u -m pytest tests/test_gpu_ops.py -x -q --timeout 120 --timeout-method thread -k "conv or stem" > gpurun_out/ab2_t.log 2>&1 || { echo "TESTS FAILED"; tail -30 gpurun_out/ab2_t.log; exit 1; }
echo "tests: $(tail -1 gpurun_out/ab2_t.log)"
if [ -n "$SH" ]; then
  echo "--- default"; timeout -k 10 200 python tools/conv_bench.py $SH 2>&1 | grep -v "^W\|^E\|amdgpu.ids" || exit 1
  echo "--- $ENVB"; env $ENVB timeout -k 10 200 python tools/conv_bench.py $SH 2>&1 | grep -v "^W\|^E\|amdgpu.ids" || exit 1
fi
ENVS=";$ENVB;;$ENVB" bash tools/gpu_bench_envs.sh
