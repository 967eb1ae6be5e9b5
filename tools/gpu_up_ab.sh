# isolated upsample timings (tools/up_bench.py) for the library builds tools/ab/$V and the in-tree B,
# then the interleaved step A/B with tools/ab/$V as the A arm
set -o pipefail
cd $GRAFT_REPO_ROOT
for v in ${V:-P} B; do
  if [ $v = B ]; then L=unet-embroidery-seg_amd/unetseg_hip/libunetseg_hip.so; else L=tools/ab/$v/libunetseg_hip.so; fi
  echo "== $v"
  UNETSEG_LIB_PATH=$L timeout -k 10 120 python3 tools/up_bench.py 2>&1 | grep -v amdgpu.ids || exit 1
done
LIB_A=tools/ab/${V:-P}/libunetseg_hip.so NB=${NB:-3} bash tools/gpu_ab_all.sh
