set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
timeout -k 10 600 python -u -m pytest -x -v --timeout 600 --timeout-method thread -m gpu tests/test_gpu_ddp.py -k "bf16-16" > gpurun_out/dbg_ddp.log 2>&1; grep -n "parameters differ\|passed\|failed" gpurun_out/dbg_ddp.log | cut -c1-2500
