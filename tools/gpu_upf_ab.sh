# isolated upsample timings for tools/ab/A and the in-tree build, then the interleaved step A/B
set -o pipefail
cd $GRAFT_REPO_ROOT
for v in A B; do
  if [ $v = B ]; then L=unet-embroidery-seg_amd/unetseg_hip/libunetseg_hip.so; else L=tools/ab/A/libunetseg_hip.so; fi
  echo "== $v"
  UNETSEG_LIB_PATH=$L timeout -k 10 120 python3 tools/up_bench.py 2>&1 | grep -v amdgpu.ids || exit 1
done
timeout -k 10 300 python -u -m pytest -x -q --timeout 120 --timeout-method thread -m gpu tests/test_gpu_ops.py -k "upsample or up_" 2>&1 | tail -2 || exit 1
NB=${NB:-3} bash tools/gpu_ab_all.sh
