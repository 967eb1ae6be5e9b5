# Round 3 (end): the C5 bench line at its BASELINE loss (multitask_unet B=8, seg BCE + cls CE).
set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
timeout -k 10 200 python bench.py --model multitask_unet --batch 8 --loss bce > gpurun_out/r03_multitask_bench.json 2> gpurun_out/r03_multitask_bench.err || { echo C5 bench failed; exit 1; }
cut -c1-200 gpurun_out/r03_multitask_bench.json
# the N>1 bench path end to end on ONE MI355X (two ranks share the card; gloo moves the gradient buckets
# through the host, so the rate says nothing about scaling): bucketed all-reduce, params in sync
UNETSEG_DIST_BACKEND=gloo timeout -k 10 300 python -m torch.distributed.run --nnodes=1 --nproc-per-node 2 --master-addr 127.0.0.1 --master-port 29531 bench.py --gpus 2 --steps 3 --warmup 1 --cpu-baseline 0 > gpurun_out/r03_ddp2_rehearsal_gloo_1gpu.json 2> gpurun_out/r03_ddp2.err || { echo ddp2 rehearsal failed; tail -20 gpurun_out/r03_ddp2.err; exit 1; }
cut -c1-300 gpurun_out/r03_ddp2_rehearsal_gloo_1gpu.json
echo done
