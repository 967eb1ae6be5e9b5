# Round 3: per-call conv table of one bench step (overlapped and serialised), overlap-adam A/B,
# DeviceLoader throughput.
set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
UNETSEG_PROBE_DUMP=gpurun_out/r03b_probe_ov.txt timeout -k 10 200 python bench.py --cpu-baseline 0 --steps 5 > /dev/null 2>&1 || { echo probe failed; exit 1; }
UNETSEG_NO_OVERLAP=1 UNETSEG_PROBE_DUMP=gpurun_out/r03b_probe_serial.txt timeout -k 10 200 python bench.py --cpu-baseline 0 --steps 5 > /dev/null 2>&1 || { echo probe2 failed; exit 1; }
for i in 1 2; do for o in 0 1; do
  timeout -k 10 200 python bench.py --cpu-baseline 0 --probe 0 --steps 20 --overlap-adam $o 2>/dev/null | python -c "import json,sys; d=json.loads(sys.stdin.read()); print('overlap', d['overlap_adam'], d['value'], d['ms_per_step'])"
done; done
timeout -k 10 500 python tools/loader_bench.py --out gpurun_out/r03_loader.json 2> gpurun_out/loader.err | cut -c1-600 || { echo loader failed; tail gpurun_out/loader.err; exit 1; }
echo done
