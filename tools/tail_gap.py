"""Print the end of the last full step of a kernel trace (both streams) and the gap before Adam."""
import csv
import sys

rows = list(csv.DictReader(open(f"{sys.argv[1]}/run_kernel_trace.csv")))
ks = sorted((int(r["Start_Timestamp"]), int(r["End_Timestamp"]), r["Stream_Id"], r["Kernel_Name"]) for r in rows)
adam = [i for i, k in enumerate(ks) if "adam" in k[3]]
lo, hi = adam[-2], adam[-1]
step = ks[lo:hi + 1]
t0 = step[0][0]
for k in step[-int(sys.argv[2]) if len(sys.argv) > 2 else -10:]:
    n = k[3].replace("void (anonymous namespace)::", "").replace("(anonymous namespace)::", "")[:55]
    print(f"{(k[0] - t0) / 1e6:8.3f} {(k[1] - k[0]) / 1e3:7.1f}us s{k[2]} {n}")
