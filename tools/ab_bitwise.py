"""Bitwise A/B of one bench training step under two library builds (a kernel change that must not move
a bit: run once per build, compare the dumps).

    UNETSEG_LIB_PATH=<dir>/libunetseg_hip.so python tools/ab_bitwise.py dump <out.pt> [model] [batch]
    python tools/ab_bitwise.py compare <a.pt> <b.pt>

dump: two eager steps of bench.py's step (batches 0 and 1: fwd + loss + bwd + Adam) and saves the loss,
every parameter, gradient, Adam moment and BN buffer.  compare: lists every tensor that differs."""
import os
import sys
import types

import torch

ROOT = os.path.join(os.path.dirname(os.path.abspath(__file__)), "..")
sys.path.insert(0, ROOT)
sys.path.insert(0, os.path.join(ROOT, "unet-embroidery-seg_amd"))


def dump(out, model, batch):
    import bench

    args = types.SimpleNamespace(bucket_mb=64, ddp_bf16=0, graph=0, overlap_adam=1, plan=0)
    loss = "bce" if model == "multitask_unet" else "lovasz_hinge"
    m, step, _, _, _ = bench.build_step(model, batch, 512, loss, "cuda", 0, 1, args)
    losses = [step(0).detach().float().cpu(), step(1).detach().float().cpu()]
    torch.cuda.synchronize()
    state = {"loss": torch.stack(losses)}
    for n, p in m.named_parameters():
        state["p." + n] = p.detach().float().cpu()
        if p.grad is not None:
            state["g." + n] = p.grad.detach().float().cpu()
    for n, b in m.named_buffers():
        state["b." + n] = b.detach().cpu()
    torch.save(state, out)
    print(f"{model} B={batch}: {len(state)} tensors, losses {losses[0].item():.6f} {losses[1].item():.6f}")


def compare(a, b):
    A = torch.load(a, weights_only=True)
    B = torch.load(b, weights_only=True)
    bad = [k for k in A if k not in B or not torch.equal(A[k], B[k])]
    print(f"{len(A)} tensors, {len(bad)} differ" + (": " + ", ".join(bad[:20]) if bad else " (bit-identical)"))
    return 1 if bad else 0


if __name__ == "__main__":
    if sys.argv[1] == "dump":
        dump(sys.argv[2], sys.argv[3] if len(sys.argv) > 3 else "unet_resnet50",
             int(sys.argv[4]) if len(sys.argv) > 4 else 16)
    else:
        sys.exit(compare(sys.argv[2], sys.argv[3]))
