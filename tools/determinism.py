"""Run-to-run determinism of one model's gradients in one process (cross-stream race screen).

    python tools/determinism.py [model] [fp32|bf16] [iters]
Runs forward+backward `iters` times on the same inputs, with unrelated allocations of varying
size in between (so the caching allocator hands out different blocks each time), and reports
every parameter whose gradient differs bitwise from the first run's.
"""
import os
import sys

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
for p in (REPO, os.path.join(REPO, "unet-embroidery-seg_amd")):
    sys.path.insert(0, p)

import torch  # noqa: E402


def main():
    name = sys.argv[1] if len(sys.argv) > 1 else "unet_plain"
    dtn = sys.argv[2] if len(sys.argv) > 2 else "fp32"
    iters = int(sys.argv[3]) if len(sys.argv) > 3 else 8
    from model.model_factory import build_model
    from unetseg_hip import losses
    from utils.synthetic import make_batch

    torch.manual_seed(0)
    m = build_model(name, num_classes=2).cuda().train()
    m.compute_dtype = dtn
    x, y = make_batch(2, 64, seed=21)
    x, y = x.cuda(), y.cuda()
    ref = None
    bad = 0
    junk = []
    for it in range(iters):
        for p in m.parameters():
            p.grad = None
        out = m(x)
        loss = losses.binary_segmentation_loss(out, y, "lovasz_hinge")
        loss.backward()
        g = {k: p.grad.detach().clone() for k, p in m.named_parameters() if p.grad is not None}
        torch.cuda.synchronize()
        if ref is None:
            ref = g
        else:
            diff = [k for k in ref if not torch.equal(ref[k], g[k])]
            if diff:
                bad += 1
                worst = max(diff, key=lambda k: ((ref[k] - g[k]).norm() / (ref[k].norm() + 1e-30)).item())
                rel = ((ref[worst] - g[worst]).norm() / (ref[worst].norm() + 1e-30)).item()
                print(f"iter {it}: {len(diff)} params differ; worst {worst} rel {rel:.3e}", flush=True)
        # perturb the allocator: free some junk, allocate blocks of other sizes
        junk = junk[len(junk) // 2:] + [torch.empty((it + 1) * 1234567, dtype=torch.uint8, device="cuda")]
    print(f"{name} {dtn}: {bad} of {iters - 1} runs differ from the first")


if __name__ == "__main__":
    main()
