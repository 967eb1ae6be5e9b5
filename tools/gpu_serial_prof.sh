# Serialized (no wgrad-stream overlap) step: bench wall time + per-kernel totals per step, and the
# overlapped bench for comparison.   bash tools/gpu_serial_prof.sh <tag> [model] [batch]
set -o pipefail
TAG=${1:-ser}
MODEL=${2:-unet_resnet50}
BATCH=${3:-16}
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
B="--model $MODEL --batch $BATCH --cpu-baseline 0 --probe 0"
timeout -k 10 300 python bench.py $B --steps 20 --warmup 5 > gpurun_out/${TAG}_ovl.json 2> gpurun_out/${TAG}_ovl.err || { echo bench failed; tail gpurun_out/${TAG}_ovl.err; exit 1; }
UNETSEG_NO_OVERLAP=1 timeout -k 10 300 python bench.py $B --steps 20 --warmup 5 > gpurun_out/${TAG}_ser.json 2> gpurun_out/${TAG}_ser.err || { echo bench failed; exit 1; }
UNETSEG_NO_OVERLAP=1 timeout -k 10 300 rocprofv3 --kernel-trace --output-format csv -d gpurun_out/${TAG}_prof -o run -- python bench.py $B --steps 5 --warmup 2 > gpurun_out/${TAG}_prof.log 2>&1 || { echo prof failed; exit 1; }
python tools/trace_streams.py gpurun_out/${TAG}_prof 4 80 > gpurun_out/${TAG}_streams.txt
rm -rf gpurun_out/${TAG}_prof
grep -o '"ms_per_step": [0-9.]*' gpurun_out/${TAG}_ovl.json gpurun_out/${TAG}_ser.json
