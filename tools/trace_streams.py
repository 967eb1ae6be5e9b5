"""Per-stream busy time and critical-path view of a rocprofv3 --kernel-trace run.

    python tools/trace_streams.py <dir with run_kernel_trace.csv> [steps]

Takes the last `steps` training steps (split at the input pack: pack_input_stem or pack_input), and prints per stream: summed
kernel time, union-of-intervals wall, and the top kernels by time on each stream; plus the idle
gaps of the compute stream (time where no kernel of that stream runs).
"""
import csv
import sys
from collections import defaultdict


def main():
    d = sys.argv[1]
    steps = int(sys.argv[2]) if len(sys.argv) > 2 else 3
    top = int(sys.argv[3]) if len(sys.argv) > 3 else 14
    rows = list(csv.DictReader(open(f"{d}/run_kernel_trace.csv")))
    ks = [(int(r["Start_Timestamp"]), int(r["End_Timestamp"]), r["Stream_Id"], r["Kernel_Name"]) for r in rows]
    ks.sort()
    # a step starts at the stem input pack (Adam runs once per gradient bucket with --overlap-adam);
    # the last step is closed by the final kernel of the trace
    mark = [i for i, k in enumerate(ks) if "pack_input" in k[3]]  # the step's first kernel: the input pack (stem or plain)
    if len(mark) < steps:
        print("not enough steps", len(mark))
        return
    lo, hi = mark[-steps], len(ks)
    sel = ks[lo:hi]
    t0, t1 = sel[0][0], max(k[1] for k in sel)
    wall = (t1 - t0) / 1e6 / steps
    print(f"wall per step {wall:.3f} ms over {steps} steps")
    by = defaultdict(list)
    for k in sel:
        by[k[2]].append(k)
    # union of all streams
    def union(iv):
        iv = sorted((a, b) for a, b, *_ in iv)
        tot, cs, ce = 0, None, None
        for a, b in iv:
            if cs is None or a > ce:
                if cs is not None:
                    tot += ce - cs
                cs, ce = a, b
            else:
                ce = max(ce, b)
        if cs is not None:
            tot += ce - cs
        return tot
    print(f"any-stream busy {union(sel) / 1e6 / steps:.3f} ms/step")
    for s, lst in sorted(by.items()):
        tot = sum(b - a for a, b, *_ in lst) / 1e6 / steps
        print(f"stream {s}: {len(lst) // steps} kernels/step, sum {tot:.3f} ms, busy {union(lst) / 1e6 / steps:.3f} ms")
        agg = defaultdict(lambda: [0, 0.0])
        for a, b, _, n in lst:
            key = n.replace("void (anonymous namespace)::", "").replace("(anonymous namespace)::", "").split("(")[0][:70]
            agg[key][0] += 1
            agg[key][1] += (b - a) / 1e6 / steps
        for n, (c, t) in sorted(agg.items(), key=lambda kv: -kv[1][1])[:top]:
            print(f"   {t:7.3f} ms {c // steps:4d}x  {n}")


if __name__ == "__main__":
    main()
