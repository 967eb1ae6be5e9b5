# Round artifacts on one MI355X: bench line, rocprofv3 kernel stats, PMC HBM traffic (two passes),
# PMC MFMA utilisation (one pass), conv kernel-configuration table.
#   COMMIT=<sha> bash tools/gpu_profile_round.sh <round tag, e.g. r02> [model] [batch] [loss]
# Outputs under gpurun_out/<tag>_*; copy the summaries into profiles/ afterwards.  COMMIT (the tree's
# git sha, substituted on the host before the call: the GPU box gets no .git) is written into every
# summary.
set -o pipefail
TAG=${1:-r02}
MODEL=${2:-unet_resnet50}
BATCH=${3:-16}
LOSS=${4:-lovasz_hinge}
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
if [ "$MODEL" = multitask_unet ]; then TASK="seg+cls multitask"; else TASK="binary seg"; fi
WL="$MODEL $TASK 512x512, per-GPU batch $BATCH, $LOSS + Adam"
B="--model $MODEL --batch $BATCH --loss $LOSS"
# the C2 line carries the extra configurations (C4, C5); a C4 / C5 run times its own model only
if [ "$MODEL" = unet_resnet50 ]; then XB=""; else XB="--extra-configs 0 --cpu-baseline 0"; fi
timeout -k 10 400 python bench.py $B $XB > gpurun_out/${TAG}_bench.json 2> gpurun_out/${TAG}_bench.err || { echo bench failed; tail gpurun_out/${TAG}_bench.err; exit 1; }
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/${TAG}_prof -o run -- python bench.py $B --steps 5 --warmup 2 --cpu-baseline 0 --extra-configs 0 --card-probe 0 --host-probe 0 --probe 0 > gpurun_out/${TAG}_prof.log 2>&1 || { echo prof failed; exit 1; }
timeout -s KILL 300 rocprofv3 --pmc FETCH_SIZE --kernel-trace --output-format csv -d gpurun_out/${TAG}_pmcF -o run -- python bench.py $B --steps 2 --warmup 1 --cpu-baseline 0 --probe 0 --extra-configs 0 --card-probe 0 --host-probe 0 > gpurun_out/${TAG}_pmcF.log 2>&1 || { echo pmc fetch failed; exit 1; }
timeout -s KILL 300 rocprofv3 --pmc WRITE_SIZE --kernel-trace --output-format csv -d gpurun_out/${TAG}_pmcW -o run -- python bench.py $B --steps 2 --warmup 1 --cpu-baseline 0 --probe 0 --extra-configs 0 --card-probe 0 --host-probe 0 > gpurun_out/${TAG}_pmcW.log 2>&1 || { echo pmc write failed; exit 1; }
timeout -s KILL 300 rocprofv3 --pmc SQ_VALU_MFMA_BUSY_CYCLES SQ_INSTS_MFMA GRBM_GUI_ACTIVE SQ_WAVES --kernel-trace --output-format csv -d gpurun_out/${TAG}_pmcM -o run -- python bench.py $B --steps 2 --warmup 1 --cpu-baseline 0 --probe 0 --extra-configs 0 --card-probe 0 --host-probe 0 > gpurun_out/${TAG}_pmcM.log 2>&1 || { echo pmc mfma failed; exit 1; }
python tools/pmc_traffic.py gpurun_out/${TAG}_pmcF gpurun_out/${TAG}_pmcW gpurun_out/${TAG}_traffic.json "$WL" > /dev/null
python tools/pmc_mfma.py gpurun_out/${TAG}_pmcM gpurun_out/${TAG}_mfma.json "$WL" > /dev/null
python tools/prof_summary.py gpurun_out/${TAG}_prof auto 40 > gpurun_out/${TAG}_kernel_stats_summary.txt
python tools/trace_streams.py gpurun_out/${TAG}_prof 4 > gpurun_out/${TAG}_streams.txt
python tools/trace_gaps.py gpurun_out/${TAG}_prof 2 > gpurun_out/${TAG}_gaps.txt
python tools/critical_path.py gpurun_out/${TAG}_prof gpurun_out/${TAG}_traffic.json gpurun_out/${TAG}_bench.json 4 > gpurun_out/${TAG}_critical_path.md || echo "critical path failed"
timeout -k 10 240 python tools/bench_conv_configs.py --model $MODEL --batch $BATCH --out gpurun_out/${TAG}_conv_configs.txt > /dev/null 2>&1 || echo "config table failed"
python - "$TAG" "${COMMIT:-unknown}" <<'PYEOF'
import json, sys
tag, commit = sys.argv[1:3]
for f in ("kernel_stats_summary.txt", "streams.txt", "gaps.txt", "conv_configs.txt", "critical_path.md"):
    p = f"gpurun_out/{tag}_{f}"
    try:
        body = open(p).read()
    except OSError:
        continue
    open(p, "w").write(f"# commit {commit}\n" + body)
for f in ("traffic.json", "mfma.json"):
    p = f"gpurun_out/{tag}_{f}"
    try:
        d = json.load(open(p))
    except (OSError, ValueError):
        continue
    d["commit"] = commit
    json.dump(d, open(p, "w"), indent=1)
p = f"gpurun_out/{tag}_bench.json"
lines = open(p).read().strip().splitlines()
d = json.loads(lines[-1]); d["commit"] = commit
open(p, "w").write(json.dumps(d) + "\n")
PYEOF
tail -1 gpurun_out/${TAG}_bench.json | cut -c1-300
