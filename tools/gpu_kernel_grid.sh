# per-(kernel, grid) durations of one configuration's steps under rocprofv3 --kernel-trace, for the
# kernels whose name matches $PAT (BENCH_ARGS: the bench configuration; LIB: library build, default in-tree)
set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
L=${LIB:-unet-embroidery-seg_amd/unetseg_hip/libunetseg_hip.so}
rm -rf gpurun_out/kg
UNETSEG_LIB_PATH=$L timeout -k 10 300 rocprofv3 --kernel-trace --output-format csv -d gpurun_out/kg -o run -- python3 bench.py $BENCH_ARGS --steps 3 --warmup 1 --extra-configs 0 --cpu-baseline 0 --probe 0 --card-probe 0 --host-probe 0 > gpurun_out/kg.log 2>&1 || { echo rocprof failed; tail -5 gpurun_out/kg.log; exit 1; }
python3 - "$PAT" <<'PY'
import csv, glob, collections, sys
pat = sys.argv[1]
f = glob.glob("gpurun_out/kg/**/run_kernel_trace.csv", recursive=True)[0]
d = collections.defaultdict(list)
for r in csv.DictReader(open(f)):
    if pat in r["Kernel_Name"]:
        d[(r["Kernel_Name"][:70], r["Grid_Size_X"])].append((int(r["End_Timestamp"]) - int(r["Start_Timestamp"])) / 1000)
for k, v in sorted(d.items()):
    print(k, len(v), "avg %.1f us min %.1f" % (sum(v) / len(v), min(v)))
PY
rm -rf gpurun_out/kg
