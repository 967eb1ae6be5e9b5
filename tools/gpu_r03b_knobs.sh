# Round 3: step A/B of the opt-in kernel knobs left by the previous session (register-resident-weight
# halo kernel, ring DMA issue stagger), interleaved, three rounds on one box.
set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
for i in 1 2 3; do for v in base haloR sched both; do
  case $v in base) E="UNETSEG_X=0";; haloR) E="UNETSEG_HALO_R=1";; sched) E="UNETSEG_TN_SCHED=1";; both) E="UNETSEG_HALO_R=1 UNETSEG_TN_SCHED=1";; esac
  env $E timeout -k 10 200 python bench.py --cpu-baseline 0 --probe 0 --steps 20 2>/dev/null | python -c "import json,sys; d=json.loads(sys.stdin.read()); print('$v', d['value'], d['ms_per_step'])" || exit 1
done; done
echo done
