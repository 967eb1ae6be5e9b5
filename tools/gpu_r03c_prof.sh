# Round 3 (end): C2 profile set (bench line, kernel stats, PMC traffic / MFMA busy, streams, configs),
# C4 / C5 bench lines, isolated per-layer table.
set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
bash tools/gpu_profile_round.sh r03 unet_resnet50 16 lovasz_hinge || exit 1
python tools/trace_gaps.py gpurun_out/r03_prof 4 > gpurun_out/r03_gaps.txt 2>&1 || echo "gaps failed"
timeout -k 10 300 python bench.py --model attention_unet --batch 8 > gpurun_out/r03_attention_bench.json 2> gpurun_out/r03_attention_bench.err || { echo C4 bench failed; exit 1; }
timeout -k 10 300 python bench.py --model multitask_unet --batch 8 > gpurun_out/r03_multitask_bench.json 2> gpurun_out/r03_multitask_bench.err || { echo C5 bench failed; exit 1; }
cut -c1-200 gpurun_out/r03_attention_bench.json gpurun_out/r03_multitask_bench.json
timeout -k 10 300 python tools/layer_table.py --top 120 > gpurun_out/r03_layers.txt 2>&1 || echo "layer table failed"
echo done
