"""Summarise a rocprofv3 --kernel-trace --stats run: per-kernel totals and per-step GEMM launches."""
import csv
import sys

d = sys.argv[1]
rows = list(csv.DictReader(open(f"{d}/run_kernel_stats.csv")))
tot = sum(float(r["TotalDurationNs"]) for r in rows)
steps = sys.argv[2] if len(sys.argv) > 2 else "1"
if steps == "auto":  # training steps in the trace: one input pack (stem or plain) per step
    steps = sum(1 for r in csv.DictReader(open(f"{d}/run_kernel_trace.csv")) if "pack_input" in r["Kernel_Name"])
steps = max(int(steps), 1)
print(f"total kernel ms: {tot / 1e6:.2f}  per step ({steps}): {tot / 1e6 / steps:.2f}")
for r in sorted(rows, key=lambda r: -float(r["TotalDurationNs"]))[:int(sys.argv[3]) if len(sys.argv) > 3 else 30]:
    print("%8.2f ms %6s calls avg %8.1f us %5.1f%%  %s" % (float(r["TotalDurationNs"]) / 1e6, r["Calls"],
          float(r["AverageNs"]) / 1e3, float(r["Percentage"]), r["Name"][:100]))
