"""Host enqueue time of one training step vs its GPU time (is the Python op layer the bottleneck?).

    python tools/host_overhead.py [--model unet_resnet50] [--batch 16]
Prints, per step: host time from step start to the return of opt.step() (all kernels enqueued),
and the time until the GPU finished.  Also a cProfile summary of one step's host side.
"""
import argparse
import cProfile
import os
import pstats
import sys
import time

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
for p in (REPO, os.path.join(REPO, "unet-embroidery-seg_amd")):
    sys.path.insert(0, p)

import torch  # noqa: E402


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--model", default="unet_resnet50")
    ap.add_argument("--batch", type=int, default=16)
    a = ap.parse_args()
    from model.model_factory import create_model
    from unetseg_hip.arena import FusedAdam
    from unetseg_hip.losses import binary_segmentation_loss
    from utils.synthetic import make_batch

    m = create_model(a.model, weights="", num_classes=2).cuda().train()
    m.compute_dtype = "bf16"
    opt = FusedAdam(m, lr=1e-4, weight_decay=1e-4)
    x, y = make_batch(a.batch, 512, seed=5)
    x, y = x.cuda(), y.cuda()

    def step():
        opt.zero_grad()
        with torch.autocast("cuda", dtype=torch.bfloat16):
            loss = binary_segmentation_loss(m(x), y, "lovasz_hinge")
        t_f = time.perf_counter()
        loss.backward()
        opt.step()
        return t_f

    for _ in range(3):
        step()
    torch.cuda.synchronize()
    for _ in range(3):
        t0 = time.perf_counter()
        tf = step()
        t1 = time.perf_counter()
        torch.cuda.synchronize()
        t2 = time.perf_counter()
        print(f"host fwd {1e3 * (tf - t0):.2f} ms, host fwd+bwd+adam {1e3 * (t1 - t0):.2f} ms, "
              f"gpu done {1e3 * (t2 - t0):.2f} ms", flush=True)
    pr = cProfile.Profile()
    pr.enable()
    step()
    pr.disable()
    torch.cuda.synchronize()
    pstats.Stats(pr).sort_stats("tottime").print_stats(25)


if __name__ == "__main__":
    main()
