cd $GRAFT_REPO_ROOT
timeout -k 10 400 python -u -m pytest tests/test_gpu_configs.py -x -q --timeout 150 --timeout-method thread > gpurun_out/gc.log 2>&1; echo "cfg tests rc=$?"; tail -3 gpurun_out/gc.log
for c in auto 20 6; do echo "== cfg $c (Ng<=64, 1 step)"; UNETSEG_TN_CFG=$( [ $c = auto ] && echo "" || echo $c ) STATS=1 timeout -k 10 60 python tools/conv_bench.py 16,128,128,64,0,64,1,1,0 2>&1 | grep -v amdgpu | cut -c1-75; done
for c in auto 19 4; do echo "== cfg $c (1 step, Ng 256)"; UNETSEG_TN_CFG=$( [ $c = auto ] && echo "" || echo $c ) STATS=1 timeout -k 10 60 python tools/conv_bench.py 16,128,128,64,0,256,1,1,0 2>&1 | grep -v amdgpu | cut -c1-75; done
for c in auto 19; do echo "== cfg $c (8-16 steps)"; UNETSEG_TN_CFG=$( [ $c = auto ] && echo "" || echo $c ) STATS=1 timeout -k 10 60 python tools/conv_bench.py 16,64,64,512,0,128,1,1,0 16,32,32,1024,0,256,1,1,0 16,64,64,128,0,512,1,1,0 2>&1 | grep -v amdgpu | cut -c1-130; done
