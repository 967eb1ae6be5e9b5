# Round 3: stem forward TN configuration sweep (UNETSEG_STEM_CFG), per-call time from the layer table.
set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
for c in 6 1 2 3 5 11 12 13 14; do
  UNETSEG_STEM_CFG=$c timeout -k 10 200 python tools/layer_table.py --top 300 > gpurun_out/stem_$c.txt 2>&1 || { echo "cfg $c failed"; tail -5 gpurun_out/stem_$c.txt; exit 1; }
  echo "cfg $c: $(grep -h "^stem_" gpurun_out/stem_$c.txt | tr -s ' ' | cut -c1-120 | tr '\n' ' ')"
done
echo done
