# Round 3: per-call conv tables of one bench step (overlapped probe; isolated layer table), A/B of
# overlap-adam and of the opt-in kernel knobs, DeviceLoader throughput.
set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
UNETSEG_PROBE_DUMP=gpurun_out/r03b_probe_ov.txt timeout -k 10 200 python bench.py --cpu-baseline 0 --steps 5 > /dev/null 2>&1 || { echo probe failed; exit 1; }
timeout -k 10 300 python tools/layer_table.py --top 300 > gpurun_out/r03b_layers.txt 2>&1 || { echo layer table failed; exit 1; }
for i in 1 2 3; do for v in base noov haloR sched; do
  case $v in base) E="UNETSEG_X=0"; O=1;; noov) E="UNETSEG_X=0"; O=0;; haloR) E="UNETSEG_HALO_R=1"; O=1;; sched) E="UNETSEG_TN_SCHED=1"; O=1;; esac
  env $E timeout -k 10 200 python bench.py --cpu-baseline 0 --probe 0 --steps 20 --overlap-adam $O 2>/dev/null | python -c "import json,sys; d=json.loads(sys.stdin.read()); print('$v', d['value'], d['ms_per_step'])" || exit 1
done; done
timeout -k 10 400 python tools/loader_bench.py --out gpurun_out/r03_loader.json 2> gpurun_out/loader.err | cut -c1-600 || { echo loader failed; tail gpurun_out/loader.err; exit 1; }
echo done
