"""GPU idle at the training-step boundary caused by the host (no profiler attached).

    python tools/boundary_gap.py [c2|c4|c5] [steps]

Event A is recorded on the compute stream right after step i returns on the host (the backward has
been enqueued and joined), event B right before step i+1 enqueues its first kernel (after
zero_grad).  Nothing runs on the compute stream between the two records, so B - A (GPU clock) is
time the compute stream sat idle because the host had not yet reached step i+1; a host that runs
ahead of the GPU gives ~0.  Also prints the per-step GPU time for scale.
"""
import os
import sys
import types

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
for p in (REPO, os.path.join(REPO, "unet-embroidery-seg_amd")):
    sys.path.insert(0, p)

import torch  # noqa: E402

from host_cost import CONFIGS  # noqa: E402


def main():
    tag = sys.argv[1] if len(sys.argv) > 1 else "c2"
    steps = int(sys.argv[2]) if len(sys.argv) > 2 else 20
    import bench
    from unetseg_hip import nn as unn

    dev = torch.device("cuda", 0)
    torch.cuda.set_stream(torch.cuda.Stream(dev))
    args = types.SimpleNamespace(bucket_mb=25.0, ddp_bf16=False, graph=0, overlap_adam=1, warmup=3)
    name, batch, loss = CONFIGS[tag]
    model, step, run, _, _ = bench.build_step(name, batch, 512, loss, dev, 0, 1, args)
    for i in range(5):
        run(i)
    torch.cuda.synchronize()
    # event B: recorded when the model's forward starts (before its first kernel)
    marks = []
    orig = unn._ModelFn.forward

    def fwd(fctx, *a):
        ev = torch.cuda.Event(enable_timing=True)
        ev.record()
        marks.append(ev)
        return orig(fctx, *a)

    unn._ModelFn.forward = staticmethod(fwd)
    ends = []
    for i in range(steps):
        run(i)
        ev = torch.cuda.Event(enable_timing=True)
        ev.record()
        ends.append(ev)
    torch.cuda.synchronize()
    unn._ModelFn.forward = staticmethod(orig)
    gaps = sorted(ends[i].elapsed_time(marks[i + 1]) for i in range(steps - 1))
    per = sorted(ends[i].elapsed_time(ends[i + 1]) for i in range(steps - 1))
    print(f"{tag} {name} B={batch}: step {per[len(per) // 2]:.3f} ms median; boundary idle median "
          f"{gaps[len(gaps) // 2] * 1e3:.0f} us, max {gaps[-1] * 1e3:.0f} us, mean {sum(gaps) / len(gaps) * 1e3:.0f} us",
          flush=True)


if __name__ == "__main__":
    main()
