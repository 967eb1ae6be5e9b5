# stream-priority A/B: compute stream priority x weight-gradient stream priority
cd $GRAFT_REPO_ROOT
python -c "import torch; print('priority range', torch.cuda.Stream.priority_range())"
for i in 1 2; do
for cfg in "0 0" "-1 0" "0 -1"; do
  set -- $cfg
  r=$(UNETSEG_SIDE_PRIORITY=$2 timeout -k 10 300 python bench.py --cpu-baseline 0 --probe 0 --priority $1 2>/dev/null | tail -1 | python -c "import json,sys; d=json.load(sys.stdin); print(d['value'], d['ms_per_step'])")
  echo "compute=$1 side=$2: $r"
done
done
