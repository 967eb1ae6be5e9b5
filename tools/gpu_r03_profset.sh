set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
bash tools/gpu_profile_round.sh r03 unet_resnet50 16 lovasz_hinge
