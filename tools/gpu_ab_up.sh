# upsample backward A/B: tools/ab/A/ (previous build: library + its fast-call binding, see gpu_ab_lib.sh) vs the tree's library, parity first
cd $GRAFT_REPO_ROOT
timeout -k 10 300 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests -m gpu -k "upsample or fusion or golden or model" > gpurun_out/up_tests.log 2>&1 || { tail -30 gpurun_out/up_tests.log; exit 1; }
tail -2 gpurun_out/up_tests.log
UNETSEG_UP_ROWS=8 timeout -k 10 300 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests -m gpu -k "upsample" > gpurun_out/up_tests8.log 2>&1 || { tail -30 gpurun_out/up_tests8.log; exit 1; }
tail -1 gpurun_out/up_tests8.log
for i in 1 2 3; do
for v in A B B8; do
  case $v in A) E="UNETSEG_LIB_PATH=tools/ab/A/libunetseg_hip.so";; B) E="X=1";; B8) E="UNETSEG_UP_ROWS=8";; esac
  r=$(env $E timeout -k 10 300 python bench.py --cpu-baseline 0 --probe 0 2>/dev/null | tail -1 | python -c "import json,sys; d=json.load(sys.stdin); print(d['value'], d['ms_per_step'])") || exit 1
  echo "$v: $r"
done
done
