"""Host enqueue cost of one training step vs its GPU time, per bench configuration.

    python tools/host_cost.py [--configs c2,c4,c5] [--steps 5]

The Python op layer enqueues every kernel of a step; when that takes longer than the GPU needs to run
them, the step is host-bound and kernel work no longer shows in the step time.  Host cost: the GPU is
first parked on a long spin kernel (torch.cuda._sleep), so the launch queue never throttles the host,
and the wall time of enqueueing `steps` steps is divided by `steps`.  GPU time: the median of
per-step HIP-event times in a normal back-to-back loop (bench.py's measurement).
"""
import argparse
import os
import sys
import time
import types

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
for p in (REPO, os.path.join(REPO, "unet-embroidery-seg_amd")):
    sys.path.insert(0, p)

import torch  # noqa: E402

CONFIGS = {"c2": ("unet_resnet50", 16, "lovasz_hinge"), "c4": ("attention_unet", 8, "lovasz_hinge"),
           "c5": ("multitask_unet", 8, "bce")}


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--configs", default="c2,c4,c5")
    ap.add_argument("--steps", type=int, default=3)
    ap.add_argument("--graph", type=int, default=0)
    a = ap.parse_args()
    import bench

    dev = torch.device("cuda", 0)
    torch.cuda.set_stream(torch.cuda.Stream(dev))
    args = types.SimpleNamespace(bucket_mb=25.0, ddp_bf16=False, graph=a.graph, overlap_adam=1, warmup=3)
    for tag in a.configs.split(","):
        name, batch, loss = CONFIGS[tag]
        model, step, run, _, _ = bench.build_step(name, batch, 512, loss, dev, 0, 1, args)
        for i in range(3):
            run(i)
        torch.cuda.synchronize()
        # host cost with the GPU parked (the queue never blocks the host)
        torch.cuda._sleep(2_000_000_000)
        t0 = time.perf_counter()
        for i in range(a.steps):
            run(i)
        host = (time.perf_counter() - t0) / a.steps * 1e3
        torch.cuda.synchronize()
        # GPU time per step, back to back
        evs = [torch.cuda.Event(enable_timing=True) for _ in range(a.steps + 1)]
        evs[0].record()
        for i in range(a.steps):
            run(i)
            evs[i + 1].record()
        torch.cuda.synchronize()
        gpu = sorted(evs[i].elapsed_time(evs[i + 1]) for i in range(a.steps))[a.steps // 2]
        print(f"{tag} {name} B={batch}: host enqueue {host:.2f} ms/step, GPU {gpu:.2f} ms/step "
              f"({'host-bound' if host > gpu else 'GPU-bound'})", flush=True)
        del model, step, run
        torch.cuda.empty_cache()


if __name__ == "__main__":
    main()
