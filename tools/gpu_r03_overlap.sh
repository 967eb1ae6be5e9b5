set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
timeout -k 10 400 python -u -m pytest -x -q --timeout 300 --timeout-method thread tests/test_gpu_overlap.py tests/test_gpu_ddp.py -k "overlap or True" -rA > gpurun_out/ov_tests.log 2>&1 || { tail -40 gpurun_out/ov_tests.log; exit 1; }
tail -12 gpurun_out/ov_tests.log
for i in 1 2 3; do
  for o in 0 1; do
    timeout -k 10 200 python bench.py --cpu-baseline 0 --probe 0 --steps 20 --overlap-adam $o 2>/dev/null | python -c "import json,sys; d=json.loads(sys.stdin.read()); print('overlap', d['overlap_adam'], d['value'], d['ms_per_step'])"
  done
done
