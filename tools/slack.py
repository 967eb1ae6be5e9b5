"""Host slack per kernel in the last full step: GPU start minus the host launch call's end
(rocprofv3 --kernel-trace --hip-trace csv).  Small slack before a gap = host-bound launch."""
import csv
import glob
import sys

d = sys.argv[1]
kt = list(csv.DictReader(open(glob.glob(f"{d}/**/*kernel_trace.csv", recursive=True)[0])))
ht = list(csv.DictReader(open(glob.glob(f"{d}/**/*hip_api_trace.csv", recursive=True)[0])))
api = {r["Correlation_Id"]: (int(r["Start_Timestamp"]), int(r["End_Timestamp"]), r["Function"]) for r in ht}
ks = sorted((int(r["Start_Timestamp"]), int(r["End_Timestamp"]), r["Stream_Id"], r["Kernel_Name"], r["Correlation_Id"]) for r in kt)
adam = [i for i, k in enumerate(ks) if "adam" in k[3]]
step = ks[adam[-2]:adam[-1] + 1]
t0 = step[0][0]
nm = lambda n: n.replace("void (anonymous namespace)::", "").replace("(anonymous namespace)::", "")[:40]  # noqa: E731
prev_end = {}
rows = []
for k in step:
    a = api.get(k[4])
    slack = (k[0] - a[1]) / 1e3 if a else float("nan")
    gap = (k[0] - prev_end[k[2]]) / 1e3 if k[2] in prev_end else 0.0
    prev_end[k[2]] = k[1]
    rows.append((gap, slack, (k[0] - t0) / 1e6, k[2], nm(k[3]), a[2] if a else "?"))
sl = sorted(r[1] for r in rows if r[1] == r[1])
print(f"kernels {len(rows)}; host slack (us) min {sl[0]:.1f} p10 {sl[len(sl)//10]:.1f} median {sl[len(sl)//2]:.1f}")
print("largest gaps on their stream (gap us, slack us, t ms, stream, kernel):")
for r in sorted(rows, reverse=True)[:int(sys.argv[2]) if len(sys.argv) > 2 else 25]:
    print(f"{r[0]:8.1f} {r[1]:9.1f} {r[2]:8.3f} s{r[3]} {r[4]} [{r[5]}]")
