# Round 3: residual BN backward pass 1 for a layer's last block (post 3 onto the skip-concat slice) and
# ReLU mask bits between the 512^2 decoder convs (fwd_mask + post 4): parity, coverage, A/B of each.
set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
timeout -k 10 500 python -u -m pytest -x -v -s --timeout 200 --timeout-method thread tests/test_gpu_relu_bits.py tests/test_gpu_post_res.py tests/test_gpu_configs.py -k "relu_bits or mask or post4 or post_res or covered" > gpurun_out/bits_t.log 2>&1 || { grep -v "^E  *+" gpurun_out/bits_t.log | grep -B3 -A30 "FAILED\|Error" | tail -50 | cut -c1-300; exit 1; }
grep -h "PASSED\|SKIPPED\|relative L2" gpurun_out/bits_t.log | cut -c1-200
timeout -k 10 600 python -u -m pytest -x -q --timeout 200 --timeout-method thread tests/test_gpu_models.py tests/test_gpu_determinism.py tests/test_gpu_fullsize.py tests/test_gpu_ddp.py tests/test_gpu_bnfold.py tests/test_gpu_overlap.py tests/test_gpu_fusions.py > gpurun_out/bits_t2.log 2>&1 || { grep -v "^E  *+" gpurun_out/bits_t2.log | grep -B3 -A30 "FAILED\|Error" | tail -50 | cut -c1-300; exit 1; }
tail -1 gpurun_out/bits_t2.log
for i in 1 2 3; do for v in on nomulti nobits; do
  case $v in on) E="UNETSEG_X=0";; nomulti) E="UNETSEG_NO_POST_RES_MULTI=1";; nobits) E="UNETSEG_NO_RELU_BITS=1";; esac
  env $E timeout -k 10 200 python bench.py --cpu-baseline 0 --probe 0 --steps 20 2>/dev/null | python -c "import json,sys; d=json.loads(sys.stdin.read()); print('$v', d['value'], d['ms_per_step'])" || exit 1
done; done
echo done
