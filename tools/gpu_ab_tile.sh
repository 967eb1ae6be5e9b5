# halo wgrad split-count model: seconds per tile (UNETSEG_HALO_WG_TILE_US) A/B, interleaved
cd $GRAFT_REPO_ROOT
for i in 1 2 3; do
for v in 2.0 1.0 4.0; do
  r=$(UNETSEG_HALO_WG_TILE_US=$v timeout -k 10 300 python bench.py --cpu-baseline 0 --probe 0 2>/dev/null | tail -1 | python -c "import json,sys; d=json.load(sys.stdin); print(d['value'], d['ms_per_step'])") || exit 1
  echo "tile_us=$v: $r"
done
done
