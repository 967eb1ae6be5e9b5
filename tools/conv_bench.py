"""Microbenchmark of single bf16 conv shapes through the op layer (fwd, dgrad, wgrad), HIP events.

    python tools/conv_bench.py                      # the U-Net's heaviest shapes
    python tools/conv_bench.py 16,512,512,64,0,64,3,1,1 ...   # N,H,W,C1,C2,K,k,stride,pad
Env knobs of the library (UNETSEG_NO_HALO, UNETSEG_TN_CFG, ...) are read at first use, so compare
variants in separate processes.
"""
import os
import sys

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
for p in (REPO, os.path.join(REPO, "unet-embroidery-seg_amd")):
    sys.path.insert(0, p)

os.environ.setdefault("UNETSEG_NO_OVERLAP", "1")  # per-op timing: no wgrad/dgrad concurrency
import torch  # noqa: E402

DEFAULT = [
    "16,512,512,64,0,64,3,1,1", "16,256,256,64,128,64,3,1,1", "16,256,256,64,0,64,3,1,1",
    "16,128,128,256,256,128,3,1,1", "16,64,64,512,512,256,3,1,1", "16,32,32,1024,2048,512,3,1,1",
    "16,128,128,64,0,256,1,1,0", "16,128,128,256,0,64,1,1,0", "16,16,16,512,0,512,3,1,1",
    "16,32,32,512,0,512,3,2,1", "16,128,128,64,0,64,3,1,1",
]


def main():
    from unetseg_hip import ops
    from unetseg_hip.lib import DT_BF16
    from unetseg_hip.nn import Conv2d

    shapes = sys.argv[1:] or DEFAULT
    reps = int(os.environ.get("REPS", "10"))
    stats = bool(int(os.environ.get("STATS", "0")))  # BN partial statistics in the fwd epilogue
    accum = bool(int(os.environ.get("ACC", "0")))    # dgrad accumulates into an existing gradient
    torch.manual_seed(0)
    for sh in shapes:
        N, H, W, C1, C2, K, k, s, p = (int(v) for v in sh.split(","))
        cin = C1 + C2
        conv = Conv2d(cin, K, k, stride=s, padding=p, bias=False).cuda()
        conv.weight.grad = torch.zeros_like(conv.weight)
        pc = ops.PackedConv(conv)
        ctx = ops.Ctx(DT_BF16, True, True, torch.device("cuda"))
        pc.pack(ctx, True)
        x1 = ops.Node(torch.randn(N, H, W, C1, device="cuda").bfloat16())
        x2 = ops.Node(torch.randn(N, H, W, C2, device="cuda").bfloat16()) if C2 else None
        x1.need_grad = True
        if x2 is not None:
            x2.need_grad = True
        times = {}
        for it in range(reps + 2):
            ctx = ops.Ctx(DT_BF16, True, True, torch.device("cuda"))
            x1.grad = torch.zeros_like(x1.data) if accum else None
            if x2 is not None:
                x2.grad = None
            ops.PROBE = []
            y, _ = ops.conv(ctx, x1, pc, x2=x2, stats=stats)
            y.grad = torch.randn_like(y.data)
            ctx.backward()
            torch.cuda.synchronize()
            if it >= 2:
                for kind, fl, nl, e0, e1, desc in ops.PROBE:
                    # dgrad_padk / wgrad_padk / fwd_bnrelu_in ... under their direction
                    t = times.setdefault(desc[0].split("_")[0], [1e9, fl])
                    t[0] = min(t[0], e0.elapsed_time(e1) * 1e-3)  # best of reps
            ops.PROBE = None
        line = [f"{sh:34s}"]
        for kd in ("fwd", "dgrad", "wgrad"):
            if kd in times:
                t, fl = times[kd]
                line.append(f"{kd} {1e6 * t:8.1f} us {fl / t / 1e12:7.1f} TF/s")
        print("  ".join(line), flush=True)


if __name__ == "__main__":
    main()
