# Round 3: profile sets of the B=8 configurations (C4 attention_unet, C5 multitask_unet).
set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
bash tools/gpu_profile_round.sh r03_attention attention_unet 8 lovasz_hinge && bash tools/gpu_profile_round.sh r03_multitask multitask_unet 8 bce
