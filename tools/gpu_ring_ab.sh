# halo-A ring variants (env knobs) on the U-Net's 3x3 ring shapes, isolated per call (conv_bench)
cd $GRAFT_REPO_ROOT
SH="16,128,128,256,256,128,3,1,1 16,64,64,512,512,256,3,1,1 8,256,256,128,256,128,3,1,1 8,128,128,256,0,256,3,1,1 8,512,512,64,128,64,3,1,1 16,256,256,64,128,64,3,1,1"
for v in ${VARIANTS:-base|X=1}; do
  IFS='|' read -r label envs <<< "$v"
  echo "== $label"
  env $envs timeout -k 10 200 python3 tools/conv_bench.py $SH 2>&1 | grep -v amdgpu.ids | cut -c1-110 || exit 1
done
