for c in 7 8 9 10; do
  UNETSEG_TN_CFG=$c timeout -k 10 300 python -u -m pytest tests/test_gpu_ops.py -x -q --timeout 120 --timeout-method thread -k "conv" > gpurun_out/dma_t$c.log 2>&1
  echo "cfg $c: $(tail -1 gpurun_out/dma_t$c.log)"
done
