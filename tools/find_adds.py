"""Which op-layer calls launch the generic add kernel in one training step (and with what shapes)."""
import collections
import os
import sys
import traceback

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
for p in (REPO, os.path.join(REPO, "unet-embroidery-seg_amd")):
    sys.path.insert(0, p)
import torch  # noqa: E402


def main():
    import types
    import bench
    from unetseg_hip import lib as L
    name, batch, loss = sys.argv[1], int(sys.argv[2]), sys.argv[3]
    dev = torch.device("cuda", 0)
    torch.cuda.set_stream(torch.cuda.Stream(dev))
    args = types.SimpleNamespace(bucket_mb=8.0, ddp_bf16=False, graph=0, overlap_adam=1, warmup=1, plan=0)
    model, step, run, _, _ = bench.build_step(name, batch, 512, loss, dev, 0, 1, args)
    step(0)
    torch.cuda.synchronize()
    seen = collections.Counter()
    real = L.lib.add

    def add(*a):
        st = traceback.extract_stack(limit=6)[:-1]
        where = " <- ".join(f"{os.path.basename(f.filename)}:{f.lineno}:{f.name}" for f in reversed(st))
        seen[(a[0], a[5], a[6], where)] += 1  # dtype, rows, channels
        return real(*a)
    L.lib.__dict__["add"] = add
    step(1)
    torch.cuda.synchronize()
    for k, v in seen.most_common():
        print(v, k)


if __name__ == "__main__":
    main()
