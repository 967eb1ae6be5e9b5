# kernel durations of one bench run (kernel-trace only): KPAT = regex of kernels to print
set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
timeout -k 10 300 rocprofv3 --kernel-trace --output-format csv -d gpurun_out/ks -o run -- python bench.py --steps 3 --warmup 1 --cpu-baseline 0 --probe 0 $BENCH_ARGS > gpurun_out/ks.log 2>&1 || { echo PROF FAILED; tail -20 gpurun_out/ks.log; exit 1; }
python - <<'PY'
import csv, glob, os, re, collections
rows = list(csv.DictReader(open(glob.glob("gpurun_out/ks/**/run_kernel_trace.csv", recursive=True)[0])))
agg = collections.defaultdict(list)
grids = {}
for r in rows:
    if re.search(os.environ.get("KPAT", "pack|adam"), r["Kernel_Name"]):
        agg[r["Kernel_Name"][:70]].append((int(r["End_Timestamp"]) - int(r["Start_Timestamp"])) / 1e3)
        grids.setdefault(r["Kernel_Name"][:70], []).append(r["Grid_Size_X"])
for k, v in agg.items():
    print(f"{len(v):4d} x avg {sum(v)/len(v):8.1f} us min {min(v):8.1f}  {k}")
    if os.environ.get("KPER"):
        n = int(os.environ["KPER"])
        print("   per call (last step):", " ".join(f"{x:.1f}[grid {g}]" for x, g in zip(v[-n:], grids[k][-n:])))
PY
rm -rf gpurun_out/ks
