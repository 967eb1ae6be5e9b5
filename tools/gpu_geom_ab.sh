set -o pipefail
cd $GRAFT_REPO_ROOT
for t in 1024 512; do echo "== B RED_TARGET $t"; UNETSEG_RED_TARGET=$t timeout -k 10 200 python3 tools/elem_bench.py 2>&1 | grep -E "plain|mbits +reduce|summed" || exit 1; done
NB=3 bash tools/gpu_ab_all.sh
