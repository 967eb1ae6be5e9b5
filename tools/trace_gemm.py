"""Per-launch GEMM kernel durations of one training step from a rocprofv3 kernel trace."""
import csv
import sys

rows = list(csv.DictReader(open(f"{sys.argv[1]}/run_kernel_trace.csv")))
idx = [i for i, r in enumerate(rows) if "lovasz_scan" in r["Kernel_Name"]]
step = rows[idx[-2]:idx[-1]]
tot = sum(int(r["End_Timestamp"]) - int(r["Start_Timestamp"]) for r in step)
print("kernels/step", len(step), "ms", tot / 1e6)
agg = {}
for r in step:
    n = r["Kernel_Name"]
    d = (int(r["End_Timestamp"]) - int(r["Start_Timestamp"])) / 1e3
    key = n.replace("void (anonymous namespace)::", "").replace("(anonymous namespace)::", "")
    key = key.split("(")[0][:48]
    agg.setdefault(key, []).append((d, r["Grid_Size_X"], r["Grid_Size_Y"], r["Grid_Size_Z"], r["Workgroup_Size_X"]))
pat = sys.argv[2] if len(sys.argv) > 2 else "tn_fast"
for k, v in agg.items():
    if pat in k:
        print(k, "total %.1f us" % sum(x[0] for x in v))
        for d, gx, gy, gz, wg in v:
            print("   %8.1f us  grid=(%d,%s,%s)" % (d, int(gx) // int(wg), gy, gz))
