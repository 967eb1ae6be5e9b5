# Round 3: hold the decoder's 3x3 weight gradients back to the encoder backward (ctx.flushed guard).
set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
UNETSEG_WG_DEFER_HW=1024 UNETSEG_WG_FLUSH=layer3 timeout -k 10 400 python -u -m pytest -x -q --timeout 200 --timeout-method thread tests/test_gpu_overlap.py tests/test_gpu_determinism.py tests/test_gpu_ddp.py > gpurun_out/defer2_t.log 2>&1 || { tail -30 gpurun_out/defer2_t.log; exit 1; }
tail -1 gpurun_out/defer2_t.log
for i in 1 2 3; do for v in base a_l4 a_l3 a_dec c_l4 c_l3; do
  case $v in base) E="UNETSEG_X=0";; a_l4) E="UNETSEG_WG_DEFER_HW=1024 UNETSEG_WG_FLUSH=layer4";;
    a_l3) E="UNETSEG_WG_DEFER_HW=1024 UNETSEG_WG_FLUSH=layer3";; a_dec) E="UNETSEG_WG_DEFER_HW=1024 UNETSEG_WG_FLUSH=decoder";;
    c_l4) E="UNETSEG_WG_DEFER_HW=1024 UNETSEG_WG_DEFER_CAT=1 UNETSEG_WG_FLUSH=layer4";;
    c_l3) E="UNETSEG_WG_DEFER_HW=1024 UNETSEG_WG_DEFER_CAT=1 UNETSEG_WG_FLUSH=layer3";; esac
  env $E timeout -k 10 200 python bench.py --cpu-baseline 0 --probe 0 --steps 20 2>/dev/null | python -c "import json,sys; d=json.loads(sys.stdin.read()); print('$v', d['value'], d['ms_per_step'])" || exit 1
done; done
echo done
