set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
timeout -k 10 200 python tools/dbg/attn_c4.py 8 512 64 128 32 > gpurun_out/dbg_attn1.log 2>&1; tail -12 gpurun_out/dbg_attn1.log
timeout -k 10 200 python tools/dbg/attn_c4.py 8 64 512 1024 256 > gpurun_out/dbg_attn2.log 2>&1; tail -12 gpurun_out/dbg_attn2.log
