set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
timeout -k 10 200 python tools/tail_probe.py --steps 8 2>&1 | grep -v amdgpu.ids
timeout -k 10 200 python tools/tail_probe.py --steps 8 2>&1 | grep -v amdgpu.ids
timeout -k 10 200 python bench.py --cpu-baseline 0 2>/dev/null | cut -c1-200
