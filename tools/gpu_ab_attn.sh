# attention-gate backward pixels per block (UNETSEG_ATTN_TILE) A/B on C4, parity first
cd $GRAFT_REPO_ROOT
UNETSEG_ATTN_TILE=1024 timeout -k 10 300 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests -m gpu -k "attn or attention" > gpurun_out/attn_tests.log 2>&1 || { tail -30 gpurun_out/attn_tests.log; exit 1; }
tail -1 gpurun_out/attn_tests.log
for i in 1 2 3; do
for v in 128 512 1024; do
  r=$(UNETSEG_ATTN_TILE=$v timeout -k 10 300 python bench.py --model attention_unet --batch 8 --cpu-baseline 0 --probe 0 2>/dev/null | tail -1 | python -c "import json,sys; d=json.load(sys.stdin); print(d['value'], d['ms_per_step'])") || exit 1
  echo "tile=$v: $r"
done
done
