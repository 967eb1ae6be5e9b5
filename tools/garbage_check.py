"""Uninitialised-memory screen: gradients of one model step after the caching allocator has been
filled with NaN blocks must equal (bitwise) those of a step on fresh memory, and be finite.

    python tools/garbage_check.py [model] [fp32|bf16]
Any kernel that reads an output / partial buffer it did not write (torch.empty contents) turns the
NaN poison into a visible difference.
"""
import os
import sys

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
for p in (REPO, os.path.join(REPO, "unet-embroidery-seg_amd")):
    sys.path.insert(0, p)

import torch  # noqa: E402


def step(m, x, y):
    torch.manual_seed(0)
    from unetseg_hip import losses
    for p in m.parameters():
        p.grad = None
    out = m(x)
    loss = losses.binary_segmentation_loss(out, y, "lovasz_hinge")
    loss.backward()
    torch.cuda.synchronize()
    return out.detach().clone(), {k: p.grad.detach().clone() for k, p in m.named_parameters() if p.grad is not None}


def poison():
    blocks = []
    for mb in (1, 2, 3, 5, 8, 13, 21, 34, 55, 89, 144):
        for _ in range(3):
            blocks.append(torch.full((mb << 18,), float("nan"), device="cuda"))
    small = [torch.full((k * 97 + 1,), float("nan"), device="cuda") for k in range(1, 400)]
    torch.cuda.synchronize()
    del blocks, small  # back to the cache, contents NaN


def main():
    name = sys.argv[1] if len(sys.argv) > 1 else "unet_plain"
    dtn = sys.argv[2] if len(sys.argv) > 2 else "fp32"
    from model.model_factory import build_model
    from utils.synthetic import make_batch

    torch.manual_seed(0)
    m = build_model(name, num_classes=2).cuda().train()
    m.compute_dtype = dtn
    x, y = make_batch(2, 64, seed=21)
    x, y = x.cuda(), y.cuda()
    o0, g0 = step(m, x, y)
    bad = []
    for it in range(3):
        if it == 2 and os.environ.get("AFTER_RESNET"):
            # the eval-mode 512x512 unet_resnet50 workload of the mIoU test, then a fresh model
            r = build_model("unet_resnet50", num_classes=2).cuda().eval()
            r.compute_dtype = "fp32"
            xr, _ = make_batch(8, 512, seed=50_000)
            with torch.no_grad():
                r(xr.cuda())
            torch.cuda.synchronize()
            del r
            m2 = build_model(name, num_classes=2).cuda().train()
            m2.load_state_dict(m.state_dict())
            m2.compute_dtype = dtn
            mm = m2
        else:
            poison()
            mm = m
        o1, g1 = step(mm, x, y)
        if not torch.equal(o0, o1):
            bad.append(f"iter {it}: logits differ (finite: {bool(torch.isfinite(o1).all())})")
        for k in g0:
            if not torch.equal(g0[k], g1[k]):
                fin = bool(torch.isfinite(g1[k]).all())
                bad.append(f"iter {it}: grad {k} differs (finite: {fin})")
    print(f"{name} {dtn}: {'OK' if not bad else str(len(bad)) + ' differences'}")
    for b in bad[:30]:
        print("  ", b)


if __name__ == "__main__":
    main()
