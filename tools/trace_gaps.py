"""Idle gaps of the compute stream in a rocprofv3 --kernel-trace run, and what sits around the
non-library kernels (copies / fills) of a training step.

    python tools/trace_gaps.py <dir with run_kernel_trace.csv> [steps]

Per step (split at the stem's input pack): the compute stream's summed kernel time, its idle time between
consecutive kernels (histogram, and the largest gaps with the kernels on either side), and for every
copyBuffer / FillFunctor / elementwise launch the kernel before and after it on its stream.
"""
import csv
import sys
from collections import Counter, defaultdict


def short(n):
    return n.replace("void (anonymous namespace)::", "").replace("(anonymous namespace)::", "").split("(")[0][:60]


def main():
    d = sys.argv[1]
    steps = int(sys.argv[2]) if len(sys.argv) > 2 else 2
    rows = list(csv.DictReader(open(f"{d}/run_kernel_trace.csv")))
    ks = sorted((int(r["Start_Timestamp"]), int(r["End_Timestamp"]), r["Stream_Id"], r["Kernel_Name"]) for r in rows)
    # a step starts at the stem input pack (Adam runs once per gradient bucket with --overlap-adam)
    mark = [i for i, k in enumerate(ks) if "pack_input" in k[3]]  # the step's first kernel: the input pack (stem or plain)
    lo, hi = mark[-steps], len(ks)
    sel = ks[lo:hi]
    main_stream = ks[mark[-1]][2]
    by = defaultdict(list)
    for k in sel:
        by[k[2]].append(k)
    cs = by[main_stream]
    gaps = [(cs[i][0] - cs[i - 1][1], short(cs[i - 1][3]), short(cs[i][3])) for i in range(1, len(cs))]
    busy = sum(b - a for a, b, *_ in cs)
    idle = sum(max(g, 0) for g, *_ in gaps)
    print(f"compute stream {main_stream}: {len(cs) / steps:.0f} kernels/step, busy {busy / 1e6 / steps:.3f} ms, "
          f"idle between kernels {idle / 1e6 / steps:.3f} ms/step")
    hist = Counter()
    for g, *_ in gaps:
        us = g / 1e3
        hist["<1us" if us < 1 else "1-2us" if us < 2 else "2-5us" if us < 5 else "5-20us" if us < 20 else ">=20us"] += 1
    print("gap histogram (per step):", {k: round(v / steps, 1) for k, v in sorted(hist.items())})
    print("largest gaps:")
    for g, a, b in sorted(gaps, reverse=True)[:12]:
        print(f"  {g / 1e3:8.1f} us  after {a}  before {b}")
    agg = defaultdict(lambda: [0, 0.0])
    for g, a, b in gaps:
        agg[b][0] += 1
        agg[b][1] += max(g, 0) / 1e3
    print("idle before each kernel type (us/step, count/step):")
    for n, (c, t) in sorted(agg.items(), key=lambda kv: -kv[1][1])[:15]:
        print(f"  {t / steps:8.1f} us {c / steps:5.1f}x  {n}")
    # which other-stream kernels ran while the compute stream sat idle: for every
    # gap >= 20 us, the overlapping kernels of the other streams and how much of the gap each covers
    others = [k for s, lst in by.items() if s != main_stream for k in lst]
    held = defaultdict(lambda: [0, 0.0])
    print("gaps >= 20 us and the other streams' kernels running inside them:")
    shown = 0
    for i in range(1, len(cs)):
        g0, g1 = cs[i - 1][1], cs[i][0]
        if g1 - g0 < 20_000:
            continue
        cov = []
        for a, b, s, n in others:
            ov = min(b, g1) - max(a, g0)
            if ov > 0:
                cov.append((ov, short(n)))
                held[short(n)][0] += 1
                held[short(n)][1] += ov / 1e3
        if shown < 16:
            desc = ", ".join(f"{n} {ov / 1e3:.0f}" for ov, n in sorted(cov, reverse=True)[:3]) or "nothing (host / launch)"
            print(f"  {(g1 - g0) / 1e3:7.1f} us before {short(cs[i][3])}: {desc}")
            shown += 1
    print("other-stream kernels overlapping compute-stream gaps >= 20 us (us/step, gaps/step):")
    for n, (c, t) in sorted(held.items(), key=lambda kv: -kv[1][1])[:10]:
        print(f"  {t / steps:8.1f} us {c / steps:5.1f}x  {n}")
    print("non-library launches (per stream: before -> this -> after):")
    seen = Counter()
    for s, lst in by.items():
        for i, k in enumerate(lst):
            n = k[3]
            if "rocclr" in n or "at::native" in n or "Functor" in n:
                ctx = (short(lst[i - 1][3]) if i else "-", short(n), short(lst[i + 1][3]) if i + 1 < len(lst) else "-")
                seen[(s,) + ctx] += 1
    for (s, a, n, b), c in sorted(seen.items(), key=lambda kv: -kv[1]):
        print(f"  stream {s} {c / steps:4.1f}x  {a}  ->  {n[:40]}  ->  {b}")


if __name__ == "__main__":
    main()
