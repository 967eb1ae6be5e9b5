"""Where the compute stream waits in a training step (no profiler: HIP events only).

    python tools/tail_probe.py [--model unet_resnet50] [--batch 16] [--steps 6]

Hooks the end of ops.Ctx.backward (ops.ON_JOIN) to record, per step: c = the compute stream's last
backward kernel done, s = the weight-gradient stream's last kernel done (held-back weight gradients
and the last buckets' overlapped Adam included; both before the join), a = opt.step() done, and the
next step's first forward kernel start f.  Prints the averages of s - c (the side-stream tail the
join waits for), a - max(c, s) (Adam), f - a (step boundary: zero_grad + host) and the step time.
"""
import argparse
import contextlib
import io
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
    ap.add_argument("--steps", type=int, default=6)
    a = ap.parse_args()
    from model.model_factory import create_model
    from unetseg_hip import ops
    from unetseg_hip.arena import FusedAdam
    from unetseg_hip.losses import binary_segmentation_loss
    from utils.synthetic import make_batch

    dev = torch.device("cuda", 0)
    torch.cuda.set_stream(torch.cuda.Stream(dev))
    with contextlib.redirect_stdout(io.StringIO()):
        m = create_model(a.model, num_classes=2, weights="").to(dev).train()
    m.compute_dtype = "bf16"
    opt = FusedAdam(m, lr=1e-4, weight_decay=1e-4, overlap=True)  # bench.py's optimizer
    x, y = make_batch(a.batch, 512, seed=5)
    x, y = x.to(dev), y.to(dev)
    marks = []

    def on_join(ctx):
        # the real Ctx.backward (tape, held-back weight gradients, last buckets' Adam) has run;
        # the compute stream joins the side stream right after this
        ec, es = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        ec.record(torch.cuda.current_stream(ctx.device))
        es.record(ctx.side if ctx.side is not None else torch.cuda.current_stream(ctx.device))
        marks[-1]["c"], marks[-1]["s"] = ec, es

    ops.ON_JOIN = on_join
    for i in range(a.steps + 2):
        e0 = torch.cuda.Event(enable_timing=True)
        e0.record()
        marks.append({"f": e0})
        opt.zero_grad()
        loss = binary_segmentation_loss(m(x), y, "lovasz_hinge")
        loss.backward()
        opt.step()
        ea = torch.cuda.Event(enable_timing=True)
        ea.record()
        marks[-1]["a"] = ea
    torch.cuda.synchronize()
    ops.ON_JOIN = None
    tails, adams, bounds, steps = [], [], [], []
    for i in range(2, len(marks) - 1):
        mk, nx = marks[i], marks[i + 1]
        t_c = mk["f"].elapsed_time(mk["c"])
        t_s = mk["f"].elapsed_time(mk["s"])
        t_a = mk["f"].elapsed_time(mk["a"])
        tails.append(t_s - t_c)
        adams.append(t_a - max(t_c, t_s))
        bounds.append(mk["a"].elapsed_time(nx["f"]))
        steps.append(mk["f"].elapsed_time(nx["f"]))
    n = len(steps)
    print(f"{a.model} B={a.batch}: step {sum(steps) / n:.3f} ms; side-stream tail after the compute stream's "
          f"backward {sum(tails) / n * 1e3:.0f} us; Adam + join {sum(adams) / n * 1e3:.0f} us; "
          f"Adam end -> next step start {sum(bounds) / n * 1e3:.0f} us")


if __name__ == "__main__":
    main()
