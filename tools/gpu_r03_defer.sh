# Round 3: held-back decoder weight gradients (UNETSEG_WG_DEFER_HW / UNETSEG_WG_FLUSH): parity of a
# bf16 train step + the overlapped-Adam and 2-rank paths with the knob on, then an interleaved step A/B.
set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
UNETSEG_WG_DEFER_HW=65536 timeout -k 10 400 python -u -m pytest -x -q --timeout 200 --timeout-method thread tests/test_gpu_overlap.py tests/test_gpu_determinism.py tests/test_gpu_fullsize.py -k "overlap or determinism or bf16" > gpurun_out/defer_t.log 2>&1 || { tail -30 gpurun_out/defer_t.log; exit 1; }
tail -1 gpurun_out/defer_t.log
for i in 1 2 3; do for v in base d256dec d256l4 d256l3 d128l3; do
  case $v in base) E="UNETSEG_X=0";; d256dec) E="UNETSEG_WG_DEFER_HW=65536 UNETSEG_WG_FLUSH=decoder";;
    d256l4) E="UNETSEG_WG_DEFER_HW=65536 UNETSEG_WG_FLUSH=layer4";; d256l3) E="UNETSEG_WG_DEFER_HW=65536 UNETSEG_WG_FLUSH=layer3";;
    d128l3) E="UNETSEG_WG_DEFER_HW=16384 UNETSEG_WG_FLUSH=layer3";; esac
  env $E timeout -k 10 200 python bench.py --cpu-baseline 0 --probe 0 --steps 20 2>/dev/null | python -c "import json,sys; d=json.loads(sys.stdin.read()); print('$v', d['value'], d['ms_per_step'])" || exit 1
done; done
echo done
