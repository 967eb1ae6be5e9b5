"""Conv-group HBM traffic per kernel family against the compulsory bytes of the calls that family runs
(which kernels carry the excess over compulsory).

    python tools/conv_traffic_families.py <traffic.json> <conv_configs.json>

traffic.json: tools/pmc_traffic.py (PMC FETCH_SIZE x 2 + WRITE_SIZE per launch, launches over the PMC
run); conv_configs.json: tools/bench_conv_configs.py (calls and compulsory MB per configuration key,
one step).  The PMC run's step count is its halo weight-gradient launches over that kernel's calls per
step.  Families: a kernel-name pattern on the PMC side, a configuration-key pattern on the call side;
forward and data-gradient calls only (the weight gradients' split-K slabs are their own traffic)."""
import json
import re
import sys

FAMILIES = [
    ("halo3 (3x3 64->64, weights in LDS)", r"^halo3_kernel<", r":halo3$"),
    ("persistent halo-A ring", r"^tn_halo_persist_kernel<", r"_hp$"),
    ("TN tiles and rings (tn_fast / tn_multi)", r"^(tn_fast_kernel|tn_multi_kernel)<",
     r":(tn|ring|multi)[0-9]\w*(?<!_hp)$"),
    ("stem and first 3x3", r"^(stem_halo|first3x3)", r"^(stem_fwd|fwd):(stem_halo|first3x3)"),
]


def main():
    tr = json.load(open(sys.argv[1]))["kernels"]
    cf = json.load(open(sys.argv[2]))
    wg_calls = sum(v["calls"] for k, v in cf.items() if k == "wgrad:halo3_wgrad")
    wg_launch = sum(v["launches"] for n, v in tr.items() if n.startswith("halo3_wgrad_kernel"))
    steps = wg_launch / wg_calls if wg_calls else 1.0
    print(f"PMC run: {steps:.1f} steps (halo weight-gradient launches {wg_launch} / {wg_calls} per step)")
    print(f"{'family':40s} {'PMC MB/step':>11s} {'compulsory':>10s} {'ratio':>6s} {'excess MB':>9s}")
    tot_p = tot_c = 0.0
    rows = []
    for name, kpat, cpat in FAMILIES:
        pmc = sum((v["fetch_bytes_per_launch"] + v["write_bytes_per_launch"]) * v["launches"]
                  for n, v in tr.items() if re.search(kpat, n)) / steps / 1e6
        comp = sum(v.get("compulsory_mb", 0.0) for k, v in cf.items()
                   if re.search(cpat, k) and not k.startswith("wgrad"))
        rows.append((pmc - comp, name, pmc, comp))
        tot_p += pmc
        tot_c += comp
    for ex, name, pmc, comp in sorted(rows, reverse=True):
        print(f"{name:40s} {pmc:11.1f} {comp:10.1f} {pmc / comp if comp else 0:6.2f} {ex:9.1f}")
    print(f"{'conv fwd + data gradient':40s} {tot_p:11.1f} {tot_c:10.1f} {tot_p / tot_c if tot_c else 0:6.2f} "
          f"{tot_p - tot_c:9.1f}")


if __name__ == "__main__":
    main()
