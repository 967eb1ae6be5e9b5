set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
STATS=1 REPS=5 timeout -k 10 300 rocprofv3 --kernel-trace --stats -d gpurun_out/hstat -o hs -- python3 tools/conv_bench.py 16,512,512,64,0,64,3,1,1 > gpurun_out/hstat.log 2>&1
f=$(ls gpurun_out/hstat/*/hs_kernel_stats.csv 2>/dev/null || find gpurun_out/hstat -name '*kernel_stats.csv' | head -1)
cut -c1-200 $f | head -20
