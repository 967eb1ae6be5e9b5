# upsample rows-per-block (UNETSEG_UP_ROWS) A/B, interleaved; parity first at a ragged block size
cd $GRAFT_REPO_ROOT
UNETSEG_UP_ROWS=3 timeout -k 10 300 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests -m gpu -k "upsample" > gpurun_out/uprows_tests.log 2>&1 || { tail -20 gpurun_out/uprows_tests.log; exit 1; }
tail -2 gpurun_out/uprows_tests.log
for i in 1 2 3; do
for v in 4 2 8; do
  r=$(UNETSEG_UP_ROWS=$v timeout -k 10 300 python bench.py --cpu-baseline 0 --probe 0 2>/dev/null | tail -1 | python -c "import json,sys; d=json.load(sys.stdin); print(d['value'], d['ms_per_step'])") || exit 1
  echo "up_rows=$v: $r"
done
done
