# Round 3: host enqueue time per step vs the GPU (overlapped Adam, created stream), allocator activity.
set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
timeout -k 10 200 python tools/host_ahead.py 2>&1 | grep -v amdgpu.ids
HA_OVERLAP=0 timeout -k 10 200 python tools/host_ahead.py 2>&1 | grep -v amdgpu.ids | tail -3
echo done
