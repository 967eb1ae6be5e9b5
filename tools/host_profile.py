"""cProfile of the host side of training steps (the Python op layer's enqueue cost).

    python tools/host_profile.py [c2|c4|c5] [steps]

The GPU is parked on a spin kernel first (as tools/host_cost.py does), so the profile shows pure
enqueue work, not waits on a full launch queue.  Prints the top functions by own time and by
cumulative time.
"""
import cProfile
import os
import pstats
import sys
import types

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
for p in (REPO, os.path.join(REPO, "unet-embroidery-seg_amd")):
    sys.path.insert(0, p)

import torch  # noqa: E402

from host_cost import CONFIGS  # noqa: E402


def main():
    tag = sys.argv[1] if len(sys.argv) > 1 else "c5"
    steps = int(sys.argv[2]) if len(sys.argv) > 2 else 3
    import bench

    dev = torch.device("cuda", 0)
    torch.cuda.set_stream(torch.cuda.Stream(dev))
    args = types.SimpleNamespace(bucket_mb=25.0, ddp_bf16=False, graph=0, overlap_adam=1, warmup=3)
    name, batch, loss = CONFIGS[tag]
    model, step, run, _, _ = bench.build_step(name, batch, 512, loss, dev, 0, 1, args)
    for i in range(3):
        run(i)
    torch.cuda.synchronize()
    # the op layer's backward runs in autograd's worker thread: profile it there separately
    from unetseg_hip import nn as unn

    bprof = cProfile.Profile()
    orig = unn._ModelFn.backward

    def backward(fctx, *grads):
        bprof.enable()
        try:
            return orig(fctx, *grads)
        finally:
            bprof.disable()

    unn._ModelFn.backward = staticmethod(backward)
    torch.cuda._sleep(2_000_000_000)
    prof = cProfile.Profile()
    prof.enable()
    for i in range(steps):
        run(i)
    prof.disable()
    torch.cuda.synchronize()
    for title, pr in (("main thread (forward, loss, optimizer)", prof), ("autograd thread (op-layer backward)", bprof)):
        print(f"===== {title}")
        st = pstats.Stats(pr)
        st.sort_stats("tottime").print_stats(25)
        st.sort_stats("cumulative").print_stats(25)


if __name__ == "__main__":
    main()
