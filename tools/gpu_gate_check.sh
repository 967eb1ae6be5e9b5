# attention-gate bf16 op test under padded / unpadded narrow gradients and with / without the side stream
for e in X=1 X=2 UNETSEG_NO_PADK=1 UNETSEG_NO_OVERLAP=1 "UNETSEG_NO_OVERLAP=1 UNETSEG_NO_PADK=1"; do
  echo "== $e"
  env $e timeout -k 10 200 python -u -m pytest tests/test_gpu_ops.py -q --timeout 120 --timeout-method thread -k "attention_gate and bf16" 2>&1 | grep -E "^E +AssertionError|passed|failed" || exit 1
done
