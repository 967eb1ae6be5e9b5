set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
timeout -k 10 300 python tools/elem_bench.py > gpurun_out/r03_elem.txt 2>&1 || { tail gpurun_out/r03_elem.txt; exit 1; }
grep -v amdgpu.ids gpurun_out/r03_elem.txt
