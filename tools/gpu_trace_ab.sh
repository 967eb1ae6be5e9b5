# kernel traces of the bench for two env settings (A: as is, B: $ENV_B)
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
timeout -k 10 300 rocprofv3 --kernel-trace --output-format csv -d gpurun_out/tra -o run -- python bench.py --steps 4 --warmup 2 --cpu-baseline 0 --probe 0 > gpurun_out/tra.log 2>&1 && \
eval "$ENV_B timeout -k 10 300 rocprofv3 --kernel-trace --output-format csv -d gpurun_out/trb -o run -- python bench.py --steps 4 --warmup 2 --cpu-baseline 0 --probe 0" > gpurun_out/trb.log 2>&1
