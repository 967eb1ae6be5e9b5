"""Per-conv-call timing table of one bf16 training step (HIP events around every conv launch).

    python tools/layer_table.py [--model unet_resnet50] [--batch 16] [--size 512] [--top 60]

Prints one row per fwd / dgrad / wgrad call: shape (N,H,W,C1,C2,K,R,S,stride), time, TFLOP/s,
sorted by time; then totals per kind.  Used to pick the next kernel to optimise.
"""
import argparse
import os
import sys

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
for p in (REPO, os.path.join(REPO, "unet-embroidery-seg_amd")):
    sys.path.insert(0, p)

os.environ.setdefault("UNETSEG_NO_OVERLAP", "1")  # per-op timing: no wgrad/dgrad concurrency
import torch  # noqa: E402


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--model", default="unet_resnet50")
    ap.add_argument("--batch", type=int, default=16)
    ap.add_argument("--size", type=int, default=512)
    ap.add_argument("--top", type=int, default=60)
    a = ap.parse_args()
    from model.model_factory import create_model
    from unetseg_hip import ops
    from unetseg_hip.arena import FusedAdam
    from unetseg_hip.losses import binary_segmentation_loss
    from utils.synthetic import make_batch

    kw = dict(num_classes=1) if a.model == "multitask_unet" else dict(num_classes=2)
    m = create_model(a.model, weights="", **kw).cuda().train()
    m.compute_dtype = "bf16"
    opt = FusedAdam(m, lr=1e-4, weight_decay=1e-4)
    x, y = make_batch(a.batch, a.size, seed=5)
    x, y = x.cuda(), y.cuda()

    def step():
        opt.zero_grad()
        with torch.autocast("cuda", dtype=torch.bfloat16):
            loss = binary_segmentation_loss(m(x), y, "lovasz_hinge")
        loss.backward()
        opt.step()

    for _ in range(3):
        step()
    torch.cuda.synchronize()
    ops.PROBE = []
    step()
    torch.cuda.synchronize()
    rows = []
    for kind, fl, nl, e0, e1, desc in ops.PROBE:
        t = e0.elapsed_time(e1) * 1e-3
        rows.append((t, desc, fl))
    ops.PROBE = None
    tot = {}
    for t, d, fl in rows:
        e = tot.setdefault(d[0], [0.0, 0.0, 0])
        e[0] += t
        e[1] += fl
        e[2] += 1
    print("%-6s %-34s %9s %8s" % ("kind", "N,H,W,C1,C2,K,R,S,st", "us", "TF/s"))
    for t, d, fl in sorted(rows, key=lambda r: -r[0])[:a.top]:
        print("%-6s %-34s %9.1f %8.1f" % (d[0], ",".join(str(v) for v in d[1:]), t * 1e6, fl / t / 1e12))
    for k, (t, fl, n) in tot.items():
        print(f"TOTAL {k}: {n} calls {t * 1e3:.3f} ms {fl / t / 1e12:.1f} TF/s")


if __name__ == "__main__":
    main()
