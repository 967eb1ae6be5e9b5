"""Largest idle gaps of the busiest stream in the last full step of a rocprofv3 kernel trace."""
import collections
import csv
import sys

rows = list(csv.DictReader(open(f"{sys.argv[1]}/run_kernel_trace.csv")))
ks = sorted((int(r["Start_Timestamp"]), int(r["End_Timestamp"]), r["Stream_Id"], r["Kernel_Name"]) for r in rows)
adam = [i for i, k in enumerate(ks) if "adam" in k[3]]
step = ks[adam[-2]:adam[-1] + 1]
t0 = step[0][0]
cnt = collections.Counter(k[2] for k in step)
main_s = cnt.most_common(1)[0][0]
main = [k for k in step if k[2] == main_s]
gaps = sorted(((b[0] - a[1], (a[1] - t0) / 1e6, a[3], b[3]) for a, b in zip(main, main[1:])), reverse=True)
nm = lambda n: n.replace("void (anonymous namespace)::", "").replace("(anonymous namespace)::", "")[:45]  # noqa: E731
print(f"stream {main_s}: total gap {sum(g[0] for g in gaps) / 1e6:.3f} ms over {len(gaps)} boundaries")
hist = collections.Counter(min(int(g[0] / 2000) * 2, 40) for g in gaps)
print("gap histogram (us bucket: count):", sorted(hist.items()))
for g in gaps[:int(sys.argv[2]) if len(sys.argv) > 2 else 12]:
    print(f"{g[0] / 1e3:8.1f} us at {g[1]:7.3f}  {nm(g[2])} -> {nm(g[3])}")
