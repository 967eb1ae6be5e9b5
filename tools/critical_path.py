"""Critical-path budget of one training step: the compute stream's time per kernel
class against that class's floor.

    python tools/critical_path.py <prof dir (run_kernel_trace.csv)> <traffic.json> <bench.json> [steps]

* ms/step: summed kernel time of the class on the compute stream (the stream of the step's input
  pack) over the last `steps` steps of a rocprofv3 --kernel-trace run (profiled clocks: a few % slow);
* floor: the conv GEMMs (fwd + data gradient) take bench.py's probe floor, the sum over calls of
  max(algorithmic flop / 2516.6 TF/s, compulsory bytes / 6.3 TB/s); every other class takes its PMC
  bytes (FETCH_SIZE x2 + WRITE_SIZE per launch, tools/pmc_traffic.py) / 6.3 TB/s, and at least 2 us per
  launch (an empty launch's cost on this card);
* the compute stream's idle time between kernels is a row of its own (floor 0).
Prints a markdown table and the sum of floors as a step time and images/s.
"""
import csv
import json
import re
import sys
from collections import defaultdict

HBM = 6.3e12
LAUNCH_US = 2.0
CLASSES = [
    ("conv fwd + data gradient (MFMA)", r"tn_fast_kernel|tn_multi_kernel|halo3_kernel<|stem_halo|first3x3|tn_halo_persist|igemm_tn"),
    ("weight gradient on the compute stream", r"wgrad|stem_wgrad_remap"),
    ("BN apply (forward)", r"bn_apply"),
    ("BN backward apply / reduce", r"bn_bwd_apply|bn_bwd_reduce"),
    ("BN / bias finalize", r"finalize|colsum|fin_merge"),
    ("upsample fwd / bwd", r"upsample"),
    ("maxpool fwd / bwd", r"maxpool"),
    ("ReLU backward + bias", r"relu_bwd"),
    ("attention gate", r"attn_|pw_small"),
    ("loss (Lovasz sort, BCE, CE)", r"lovasz|radix|bce|ce_|scale_grad|mc_loss"),
    ("input pack / weight pack / Adam", r"pack|adam"),
]


def short(n):
    return n.replace("void (anonymous namespace)::", "").replace("(anonymous namespace)::", "").split("(")[0][:80]


def main():
    d, traffic_p, bench_p = sys.argv[1:4]
    steps = int(sys.argv[4]) if len(sys.argv) > 4 else 3
    rows = list(csv.DictReader(open(f"{d}/run_kernel_trace.csv")))
    ks = sorted((int(r["Start_Timestamp"]), int(r["End_Timestamp"]), r["Stream_Id"], r["Kernel_Name"]) for r in rows)
    mark = [i for i, k in enumerate(ks) if "pack_input" in k[3]]
    sel = ks[mark[-steps]:]
    cs = [k for k in sel if k[2] == ks[mark[-1]][2]]
    tr = json.load(open(traffic_p)).get("kernels", {})
    line = [ln for ln in open(bench_p).read().splitlines() if ln.startswith("{")][-1]
    bj = json.loads(line)
    roof = bj.get("roofline") or {}
    wl = (bj.get("config") or {}).get("workload", "")
    model = wl.split()[0] if wl else "unet_resnet50"
    m = re.search(r"per-GPU batch (\d+)", wl)
    batch = int(m.group(1)) if m else 16
    gflop = {"unet_resnet50": 547.46, "multitask_unet": 547.36, "attention_unet": 1374.35}.get(model, 547.46)
    conv_floor = roof.get("floor_ms_per_step")
    agg = defaultdict(lambda: [0, 0.0, 0.0, 0])  # launches, ms, floor ms, launches without PMC bytes
    for a, b, _, n in cs:
        cls = next((c for c, pat in CLASSES if re.search(pat, n)), "other")
        e = agg[cls]
        e[0] += 1
        e[1] += (b - a) / 1e6
        t = tr.get(short(n))
        if t is not None:
            e[2] += max((t["fetch_bytes_per_launch"] + t["write_bytes_per_launch"]) / HBM * 1e3, LAUNCH_US * 1e-3)
        else:
            e[2] += LAUNCH_US * 1e-3
            e[3] += 1
    idle = sum(max(cs[i][0] - cs[i - 1][1], 0) for i in range(1, len(cs))) / 1e6
    out = []
    tot_ms = tot_floor = 0.0
    for cls, (c, ms, fl, miss) in sorted(agg.items(), key=lambda kv: -kv[1][1]):
        ms /= steps
        fl /= steps
        if cls.startswith("conv") and conv_floor is not None:
            fl = conv_floor
        tot_ms += ms
        tot_floor += fl
        note = f" ({miss // steps} launches without PMC bytes: launch floor)" if miss else ""
        out.append((cls + note, c / steps, ms, fl))
    print("| kernel class (compute stream) | launches/step | ms/step | floor ms | gap ms |")
    print("|---|---|---|---|---|")
    for cls, c, ms, fl in out:
        print(f"| {cls} | {c:.0f} | {ms:.3f} | {fl:.3f} | {ms - fl:.3f} |")
    print(f"| idle between kernels | - | {idle / steps:.3f} | 0 | {idle / steps:.3f} |")
    step = tot_ms + idle / steps
    print(f"| **step (compute stream)** | {len(cs) / steps:.0f} | **{step:.3f}** | **{tot_floor:.3f}** | {step - tot_floor:.3f} |")
    need = gflop * batch / 2516.6 / 0.35
    print(f"\nsum of floors {tot_floor:.3f} ms = {batch / tot_floor * 1e3:.0f} img/s ({model}, B={batch}; "
          f"step fraction {gflop * batch / tot_floor / 2516.6:.3f}); 0.35 needs <= {need:.2f} ms per step")


if __name__ == "__main__":
    main()
