"""Kernel configurations one benchmark step runs, with their HIP-event time (GPU).

    python tools/bench_conv_configs.py [--model unet_resnet50] [--batch 16] [--size 512] [--out FILE]

Runs one warmup step and one probe step of bench.py's workload and prints, per kernel
configuration (conv fwd / dgrad / fused dgrad / wgrad + split-K reduce), the calls per step and
their summed HIP-event time.  DESIGN.md's coverage table maps each row to the test that covers it.
"""
import argparse
import contextlib
import json
import os
import sys

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
for p in (REPO, os.path.join(REPO, "unet-embroidery-seg_amd")):
    sys.path.insert(0, p)

import torch  # noqa: E402


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--model", default="unet_resnet50")
    ap.add_argument("--batch", type=int, default=16)
    ap.add_argument("--size", type=int, default=512)
    ap.add_argument("--out", default=None)
    args = ap.parse_args()
    from model.model_factory import create_model
    from unetseg_hip import introspect, ops
    from unetseg_hip.arena import FusedAdam
    from unetseg_hip.losses import binary_segmentation_loss, multitask_loss
    from utils.synthetic import make_batch

    dev = torch.device("cuda", 0)
    torch.cuda.set_stream(torch.cuda.Stream(dev))
    kw = dict(num_classes=1) if args.model == "multitask_unet" else dict(num_classes=2)
    with contextlib.redirect_stdout(sys.stderr):
        model = create_model(args.model, weights="", **kw).to(dev).train()
    model.compute_dtype = "bf16"
    opt = FusedAdam(model, lr=1e-4)
    x, y, c = make_batch(args.batch, args.size, seed=5, with_cls=True)
    x, y, c = x.to(dev), y.to(dev), c.to(dev)

    def step():
        opt.zero_grad()
        with torch.autocast("cuda", dtype=torch.bfloat16):
            if args.model == "multitask_unet":
                seg, cls = model(x)
                loss = multitask_loss(seg, cls, y, c, 1.0, "bce")[0]
            else:
                loss = binary_segmentation_loss(model(x), y, "lovasz_hinge")
        loss.backward()
        opt.step()

    step()
    ops.PROBE = []
    step()
    torch.cuda.synchronize()
    table = introspect.probe_table(ops.PROBE)
    # compulsory HBM bytes per configuration (bench.compulsory_bytes of each call, charged to the
    # call's first key like its time): the denominator of a per-configuration traffic ratio
    import bench
    comp = {}
    for kind, flops, nl, e0, e1, desc in ops.PROBE:
        keys = introspect.call_configs(desc)
        if keys and not desc[0].startswith("wgrad"):
            comp[keys[0]] = comp.get(keys[0], 0) + bench.compulsory_bytes(desc)
    ops.PROBE = None
    rows = sorted(table.items(), key=lambda kv: -kv[1][1])
    lines = [f"# {args.model} {args.size}x{args.size} batch {args.batch} bf16: kernel configurations of one step"]
    lines.append(f"{'configuration':40s} {'calls':>6s} {'ms/step':>9s}")
    for k, (n, t) in rows:
        lines.append(f"{k:40s} {n:6d} {1e3 * t:9.3f}")
    text = "\n".join(lines)
    print(text)
    if args.out:
        with open(args.out, "w") as f:
            f.write(text + "\n")
        with open(os.path.splitext(args.out)[0] + ".json", "w") as f:
            json.dump({k: {"calls": n, "ms": round(1e3 * t, 4), "compulsory_mb": round(comp.get(k, 0) / 1e6, 2)}
                       for k, (n, t) in rows}, f, indent=1)


if __name__ == "__main__":
    main()
