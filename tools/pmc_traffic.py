"""HBM traffic per launch of the roofline kernel from two rocprofv3 PMC passes (FETCH_SIZE, WRITE_SIZE).

    rocprofv3 --pmc FETCH_SIZE --kernel-trace --output-format csv -d <F> -o run -- python bench.py ...
    rocprofv3 --pmc WRITE_SIZE --kernel-trace --output-format csv -d <W> -o run -- python bench.py ...
    python tools/pmc_traffic.py <F> <W> <out.json> <workload string printed by bench.py>

Corrections (MI355X_MICROARCH.md, HBM section): both counters are in KiB; on gfx950 FETCH_SIZE counts
half the bytes of 16-B/lane streaming reads (the loads of every conv kernel here), so it is doubled;
WRITE_SIZE is exact for 16-B and 8-B/lane stores.  Kernels are grouped the way bench.py's probe
groups launches: "igemm_tn" = conv fwd + dgrad GEMMs, "wgrad" = weight-gradient GEMM + its reduce.
"""
import csv
import json
import re
import sys

GROUPS = {
    "igemm_tn": re.compile(r"(tn_fast_kernel|tn_multi_kernel|tn_halo_persist_kernel|halo3_kernel<|stem_halo_kernel|first3x3_fwd_kernel|igemm_tn_kernel)"),
    "wgrad": re.compile(r"(wgrad_fast_kernel|wgrad_ring_kernel|wgrad_kernel|wgrad_reduce_kernel)"),
}


def _load(d, counter):
    rows = [r for r in csv.DictReader(open(f"{d}/run_counter_collection.csv")) if r["Counter_Name"] == counter]
    return [(r["Kernel_Name"], float(r["Counter_Value"]) * 1024.0) for r in rows]


def main():
    fdir, wdir, out, workload = sys.argv[1:5]
    fetch, write = _load(fdir, "FETCH_SIZE"), _load(wdir, "WRITE_SIZE")
    res = {"workload": workload, "source": {"fetch": fdir, "write": wdir}, "unit": "bytes",
           "corrections": "FETCH_SIZE KiB x1024 x2 (gfx950 half-count of wide reads); WRITE_SIZE KiB x1024",
           "groups": {}, "kernels": {}}
    for g, pat in GROUPS.items():
        fb = [v for n, v in fetch if pat.search(n)]
        wb = [v for n, v in write if pat.search(n)]
        if not fb or not wb:
            continue
        # launches of the main GEMM kernels (reduce kernels fold into their wgrad launch)
        main_pat = re.compile(r"(tn_fast_kernel|tn_multi_kernel|tn_halo_persist_kernel|halo3_kernel<|stem_halo_kernel|first3x3_fwd_kernel|igemm_tn_kernel|wgrad_fast_kernel<|wgrad_ring_kernel<|wgrad_kernel<)")
        nl = sum(1 for n, _ in fetch if main_pat.search(n) and pat.search(n))
        f2, w = 2.0 * sum(fb), sum(wb)
        res["groups"][g] = {"launches": nl, "fetch_bytes_per_launch": f2 / nl, "write_bytes_per_launch": w / nl,
                            "traffic_bytes_per_launch": (f2 + w) / nl}
    per = {}
    for n, v in fetch:
        k = n.replace("void (anonymous namespace)::", "").replace("(anonymous namespace)::", "").split("(")[0][:80]
        e = per.setdefault(k, [0, 0.0, 0.0])
        e[0] += 1
        e[1] += 2.0 * v
    for n, v in write:
        k = n.replace("void (anonymous namespace)::", "").replace("(anonymous namespace)::", "").split("(")[0][:80]
        if k in per:
            per[k][2] += v
    top = sorted(per.items(), key=lambda kv: -(kv[1][1] + kv[1][2]))[:120]
    res["kernels"] = {k: {"launches": c, "fetch_bytes_per_launch": f / c, "write_bytes_per_launch": w / c}
                      for k, (c, f, w) in top}
    json.dump(res, open(out, "w"), indent=1)
    print(json.dumps(res["groups"], indent=1))


if __name__ == "__main__":
    main()
