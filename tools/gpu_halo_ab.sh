# isolated halo3 shapes (fwd / dgrad / wgrad per call; then the forward with BN statistics) for library
# builds in tools/ab/<v> and the in-tree build B, then the parity cases named by TESTS on B
set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
SH="16,512,512,64,0,64,3,1,1 16,256,256,64,0,64,3,1,1 16,128,128,64,0,64,3,1,1"
for v in ${VARIANTS:-A C B}; do
  if [ $v = B ]; then L=unet-embroidery-seg_amd/unetseg_hip/libunetseg_hip.so; else L=tools/ab/$v/libunetseg_hip.so; fi
  echo "== $v"
  UNETSEG_LIB_PATH=$L timeout -k 10 120 python3 tools/conv_bench.py $SH 2>&1 | grep -v amdgpu.ids || exit 1
  echo "-- stats"
  STATS=1 UNETSEG_LIB_PATH=$L timeout -k 10 120 python3 tools/conv_bench.py $SH 2>&1 | grep -v amdgpu.ids | cut -c1-60 || exit 1
done
if [ -n "$TESTS" ]; then
  timeout -k 10 600 python -u -m pytest -x -q --timeout 120 --timeout-method thread -m gpu $TESTS 2>&1 | tail -5
fi
