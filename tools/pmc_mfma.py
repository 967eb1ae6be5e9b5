"""MFMA utilisation per kernel group from one rocprofv3 PMC pass.

    rocprofv3 --pmc SQ_VALU_MFMA_BUSY_CYCLES SQ_INSTS_MFMA GRBM_GUI_ACTIVE SQ_WAVES --kernel-trace \
        --output-format csv -d <D> -o run -- python bench.py --steps 2 --warmup 1 --cpu-baseline 0 --probe 0
    python tools/pmc_mfma.py <D> <out.json> "<workload string printed by bench.py>"

Per dispatch (MI355X_MICROARCH.md, PMC rows): SQ_VALU_MFMA_BUSY_CYCLES is summed over every SIMD
(256 CUs x 4) and counts cycles; GRBM_GUI_ACTIVE is the dispatch's active cycles summed over the 8
XCDs.  MFMA busy fraction of a group = sum(MFMA busy) / (1024 x sum(GRBM_GUI_ACTIVE) / 8), i.e. the
share of all SIMD-cycles, during that group's kernels, in which the matrix pipe was busy.  Counter
FLOPs = SQ_INSTS_MFMA x 16384 (every MFMA here is v_mfma_f32_16x16x32_bf16: 16*16*32*2 flops; the
generic fp32 kernels are not in the bf16 bench).  Kernel groups as in bench.py's probe.
"""
import csv
import json
import re
import sys
from collections import defaultdict

GROUPS = {
    "igemm_tn": re.compile(r"(tn_fast_kernel|tn_multi_kernel|tn_halo_persist_kernel|halo3_kernel<|stem_halo_kernel|first3x3_fwd_kernel|igemm_tn_kernel)"),
    "wgrad": re.compile(r"(wgrad_fast_kernel|wgrad_ring_kernel|halo3_wgrad_kernel|wgrad_kernel<)"),
}
SIMDS = 256 * 4
FLOP_PER_MFMA = 16 * 16 * 32 * 2


def main():
    d, out, workload = sys.argv[1:4]
    rows = list(csv.DictReader(open(f"{d}/run_counter_collection.csv")))
    per = defaultdict(lambda: defaultdict(float))  # dispatch -> counter -> value
    names = {}
    for r in rows:
        key = r.get("Dispatch_Id") or r.get("Correlation_Id")
        per[key][r["Counter_Name"]] += float(r["Counter_Value"])
        names[key] = r["Kernel_Name"]
    res = {"workload": workload, "source": d, "simds": SIMDS,
           "formula": "mfma_busy = sum(SQ_VALU_MFMA_BUSY_CYCLES) / (1024 * sum(GRBM_GUI_ACTIVE) / 8)",
           "groups": {}, "kernels": {}}
    for g, pat in GROUPS.items():
        busy = act = insts = 0.0
        n = 0
        for k, c in per.items():
            if pat.search(names[k]):
                busy += c["SQ_VALU_MFMA_BUSY_CYCLES"]
                act += c["GRBM_GUI_ACTIVE"]
                insts += c["SQ_INSTS_MFMA"]
                n += 1
        if n:
            res["groups"][g] = {"launches": n, "mfma_busy": busy / (SIMDS * act / 8.0) if act else None,
                                "counter_gflop": insts * FLOP_PER_MFMA / 1e9}
    agg = defaultdict(lambda: [0, 0.0, 0.0, 0.0])
    for k, c in per.items():
        kn = names[k].replace("void (anonymous namespace)::", "").replace("(anonymous namespace)::", "").split("(")[0][:80]
        a = agg[kn]
        a[0] += 1
        a[1] += c["SQ_VALU_MFMA_BUSY_CYCLES"]
        a[2] += c["GRBM_GUI_ACTIVE"]
        a[3] += c["SQ_INSTS_MFMA"]
    top = sorted(agg.items(), key=lambda kv: -kv[1][2])[:30]
    res["kernels"] = {k: {"launches": n, "mfma_busy": (b / (SIMDS * a / 8.0)) if a else None,
                          "active_cycles_per_launch": a / 8.0 / n, "counter_gflop_per_launch": i * FLOP_PER_MFMA / 1e9 / n}
                      for k, (n, b, a, i) in top}
    json.dump(res, open(out, "w"), indent=1)
    print(json.dumps(res["groups"], indent=1))


if __name__ == "__main__":
    main()
