# Round artifacts on one MI355X: bench line, rocprofv3 kernel stats, PMC HBM traffic (two passes).
#   bash tools/gpu_profile_round.sh <round tag, e.g. r01>
# Outputs under gpurun_out/<tag>_*; copy the summaries into profiles/ afterwards.
set -o pipefail
TAG=${1:-r01}
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
WL="unet_resnet50 binary seg 512x512, per-GPU batch 16, lovasz_hinge + Adam"
timeout -k 10 400 python bench.py > gpurun_out/${TAG}_bench.json 2> gpurun_out/${TAG}_bench.err || { echo bench failed; tail gpurun_out/${TAG}_bench.err; exit 1; }
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/${TAG}_prof -o run -- python bench.py --steps 5 --warmup 2 --cpu-baseline 0 > gpurun_out/${TAG}_prof.log 2>&1 || { echo prof failed; exit 1; }
timeout -s KILL 300 rocprofv3 --pmc FETCH_SIZE --kernel-trace --output-format csv -d gpurun_out/${TAG}_pmcF -o run -- python bench.py --steps 2 --warmup 1 --cpu-baseline 0 --probe 0 > gpurun_out/${TAG}_pmcF.log 2>&1 || { echo pmc fetch failed; exit 1; }
timeout -s KILL 300 rocprofv3 --pmc WRITE_SIZE --kernel-trace --output-format csv -d gpurun_out/${TAG}_pmcW -o run -- python bench.py --steps 2 --warmup 1 --cpu-baseline 0 --probe 0 > gpurun_out/${TAG}_pmcW.log 2>&1 || { echo pmc write failed; exit 1; }
python tools/pmc_traffic.py gpurun_out/${TAG}_pmcF gpurun_out/${TAG}_pmcW gpurun_out/${TAG}_traffic.json "$WL" > /dev/null
python tools/prof_summary.py gpurun_out/${TAG}_prof 8 40 > gpurun_out/${TAG}_kernel_stats_summary.txt
python tools/trace_streams.py gpurun_out/${TAG}_prof 4 > gpurun_out/${TAG}_streams.txt
tail -1 gpurun_out/${TAG}_bench.json | cut -c1-200
