# Round 3 (end): C5 (multitask_unet B=8, BCE + CE) interleaved A/B of this round's late changes.
set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
for i in 1 2; do for v in on stemtn nomulti nobits; do
  case $v in on) E="UNETSEG_X=0";; stemtn) E="UNETSEG_STEM_TN=1";; nomulti) E="UNETSEG_NO_POST_RES_MULTI=1";; nobits) E="UNETSEG_NO_RELU_BITS=1";; esac
  env $E timeout -k 10 200 python bench.py --model multitask_unet --batch 8 --loss bce --cpu-baseline 0 --probe 0 --steps 20 2>/dev/null | python -c "import json,sys; d=json.loads(sys.stdin.read()); print('$v', d['value'], d['ms_per_step'])" || exit 1
done; done
echo done
