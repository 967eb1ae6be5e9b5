"""Python garbage-collector pauses during training steps, and what gc.freeze() does to them.

    python tools/gc_probe.py [c2|c4|c5] [steps]

The op layer allocates Python objects per step (tape closures, Nodes); a collection of the oldest
generation traverses every tracked object of the process (the model, torch's module tree, ...), and
while it runs the host enqueues nothing.  Prints, per arm (default / gc.freeze() after warm-up), the
collections per generation, their summed and largest pause, and the GPU time per step.
"""
import gc
import os
import sys
import time
import types

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
for p in (REPO, os.path.join(REPO, "unet-embroidery-seg_amd")):
    sys.path.insert(0, p)

import torch  # noqa: E402

from host_cost import CONFIGS  # noqa: E402


def main():
    tag = sys.argv[1] if len(sys.argv) > 1 else "c5"
    steps = int(sys.argv[2]) if len(sys.argv) > 2 else 40
    import bench

    dev = torch.device("cuda", 0)
    torch.cuda.set_stream(torch.cuda.Stream(dev))
    args = types.SimpleNamespace(bucket_mb=25.0, ddp_bf16=False, graph=0, overlap_adam=1, warmup=3)
    name, batch, loss = CONFIGS[tag]
    model, step, run, _, _ = bench.build_step(name, batch, 512, loss, dev, 0, 1, args)
    pauses = []
    t_start = {}

    def cb(phase, info):
        if phase == "start":
            t_start["t"] = time.perf_counter()
        else:
            pauses.append((info["generation"], time.perf_counter() - t_start["t"]))

    gc.callbacks.append(cb)
    for arm in ("default", "freeze"):
        for i in range(5):
            run(i)
        torch.cuda.synchronize()
        if arm == "freeze":
            gc.collect()
            gc.freeze()
        pauses.clear()
        evs = [torch.cuda.Event(enable_timing=True) for _ in range(steps + 1)]
        evs[0].record()
        t0 = time.perf_counter()
        for i in range(steps):
            run(i)
            evs[i + 1].record()
        torch.cuda.synchronize()
        wall = (time.perf_counter() - t0) / steps * 1e3
        per = sorted(evs[i].elapsed_time(evs[i + 1]) for i in range(steps))
        by = {g: [p for gg, p in pauses if gg == g] for g in (0, 1, 2)}
        desc = ", ".join(f"gen{g}: {len(v)}x sum {sum(v) * 1e3:.1f} ms max {max(v, default=0) * 1e3:.2f} ms"
                         for g, v in by.items())
        print(f"{tag} {arm:8s} wall {wall:.2f} ms/step, GPU median {per[steps // 2]:.2f} max {per[-1]:.2f} ms | {desc}",
              flush=True)
    gc.callbacks.remove(cb)


if __name__ == "__main__":
    main()
