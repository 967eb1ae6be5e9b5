"""Per-step timeline of a rocprofv3 --kernel-trace run: every kernel of both streams of one step with
its start offset from the step start, duration and stream, plus per-phase sums.

    python tools/trace_timeline.py <dir with run_kernel_trace.csv> [step index from the end, default 2]
        [--from MS] [--to MS]

A step starts at the stem's input pack (pack_input_stem).  The compute stream is the one that runs
that kernel; everything else is reported as the side (weight-gradient) stream.  Useful to read the
step's tail (what the compute stream waits for before the next step) and the overlap of the two
streams.
"""
import argparse
import csv
import glob
import os


def short(n):
    return n.replace("void (anonymous namespace)::", "").replace("(anonymous namespace)::", "").split("(")[0][:70]


def load(d):
    f = os.path.join(d, "run_kernel_trace.csv")
    if not os.path.exists(f):
        f = glob.glob(os.path.join(d, "**", "*kernel_trace.csv"), recursive=True)[0]
    rows = list(csv.DictReader(open(f)))
    return sorted((int(r["Start_Timestamp"]), int(r["End_Timestamp"]), r["Stream_Id"], r["Kernel_Name"]) for r in rows)


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("dir")
    ap.add_argument("step", nargs="?", type=int, default=2)
    ap.add_argument("--from", dest="t0", type=float, default=None)
    ap.add_argument("--to", dest="t1", type=float, default=None)
    a = ap.parse_args()
    ks = load(a.dir)
    marks = [i for i, k in enumerate(ks) if "pack_input_stem" in k[3]]
    i0, i1 = marks[-a.step - 1], marks[-a.step]
    main = ks[i0][2]
    t0 = ks[i0][0]
    t_end = ks[i1][0]
    sel = [k for k in ks if t0 <= k[0] < t_end]
    print(f"step {(t_end - t0) / 1e6:.3f} ms  compute stream {main}")
    busy = {}
    for s, e, st, n in sel:
        busy[st == main] = busy.get(st == main, 0) + (e - s)
    print(f"compute busy {busy.get(True, 0) / 1e6:.3f} ms  side busy {busy.get(False, 0) / 1e6:.3f} ms")
    for s, e, st, n in sel:
        off = (s - t0) / 1e6
        if a.t0 is not None and off < a.t0:
            continue
        if a.t1 is not None and off > a.t1:
            continue
        col = "C" if st == main else "      S"
        print(f"{off:8.3f} {(e - s) / 1e3:8.1f}us {col} {short(n)}")


if __name__ == "__main__":
    main()
