# N=2 rehearsal of the data-parallel bench on ONE GPU (both ranks share it; gloo moves the buckets):
# exercises GradBuckets + the weight-gradient stream + the joins with real device tensors.
set -o pipefail
cd $GRAFT_REPO_ROOT
UNETSEG_DIST_BACKEND=gloo timeout -k 10 300 python -m torch.distributed.run --nnodes=1 --nproc-per-node 2 \
  --master-addr 127.0.0.1 --master-port 29517 bench.py --gpus 2 --steps 3 --warmup 2 --batch 4 --cpu-baseline 0 \
  > gpurun_out/ddp2.json 2> gpurun_out/ddp2.err
rc=$?
tail -3 gpurun_out/ddp2.err; tail -1 gpurun_out/ddp2.json | cut -c1-250
exit $rc
