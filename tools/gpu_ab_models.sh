# C4 / C5 bench A/B: tools/ab/A/ (library + fast-call binding) vs the tree's library, interleaved
cd $GRAFT_REPO_ROOT
for M in "attention_unet --batch 8" "multitask_unet --batch 8 --loss bce"; do
for i in 1 2 3; do
for v in A B; do
  case $v in A) E="UNETSEG_LIB_PATH=tools/ab/A/libunetseg_hip.so";; B) E="X=1";; esac
  r=$(env $E timeout -k 10 300 python bench.py --model $M --cpu-baseline 0 --probe 0 2>/dev/null | tail -1 | python -c "import json,sys; d=json.load(sys.stdin); print(d['value'], d['ms_per_step'])") || exit 1
  echo "$M $v: $r"
done
done
done
