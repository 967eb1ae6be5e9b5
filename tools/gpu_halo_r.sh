# halo3r (register-resident weights, 3 halo stages) vs halo3 (LDS weights): parity + timing
set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
T="tests/test_gpu_configs.py tests/test_gpu_fusions.py"
timeout -k 10 300 python -u -m pytest -x -q --timeout 120 --timeout-method thread $T -k "halo or head" > gpurun_out/hr_t8.log 2>&1 || { tail -30 gpurun_out/hr_t8.log; exit 1; }
tail -2 gpurun_out/hr_t8.log
UNETSEG_HALO_R_NW=4 timeout -k 10 300 python -u -m pytest -x -q --timeout 120 --timeout-method thread $T -k "halo or head" > gpurun_out/hr_t4.log 2>&1 || { tail -30 gpurun_out/hr_t4.log; exit 1; }
tail -2 gpurun_out/hr_t4.log
SH="16,512,512,64,0,64,3,1,1 16,256,256,64,0,64,3,1,1 16,128,128,64,0,64,3,1,1"
for v in V1 R8 R4; do
  case $v in V1) E="UNETSEG_HALO_V1=1";; R8) E="UNETSEG_HALO_R_NW=8";; R4) E="UNETSEG_HALO_R_NW=4";; esac
  echo "== $v"
  env $E timeout -k 10 120 python3 tools/conv_bench.py $SH 2>&1 | grep -v amdgpu.ids
  env $E STATS=1 timeout -k 10 120 python3 tools/conv_bench.py 16,512,512,64,0,64,3,1,1 2>&1 | grep -v amdgpu.ids
done
for i in 1 2; do for v in V1 R8; do
  case $v in V1) E="UNETSEG_HALO_V1=1";; R8) E="UNETSEG_HALO_R_NW=8";; esac
  env $E timeout -k 10 200 python bench.py --cpu-baseline 0 --probe 0 --steps 20 2>/dev/null | python -c "import json,sys; d=json.loads(sys.stdin.read()); print('$v', d['value'], d['ms_per_step'])"
done; done
timeout -k 10 400 python tools/loader_bench.py --out gpurun_out/r03_loader.json 2>gpurun_out/loader.err | cut -c1-300
