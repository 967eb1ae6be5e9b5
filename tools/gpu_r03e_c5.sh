# Round 3 (end): the C5 bench line at its BASELINE loss (multitask_unet B=8, seg BCE + cls CE).
set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
timeout -k 10 200 python bench.py --model multitask_unet --batch 8 --loss bce > gpurun_out/r03_multitask_bench.json 2> gpurun_out/r03_multitask_bench.err || { echo C5 bench failed; exit 1; }
cut -c1-200 gpurun_out/r03_multitask_bench.json
