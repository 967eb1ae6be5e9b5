"""Microbenchmark of the memory-bound BN kernels at the unet_resnet50 B=16 shapes (HIP events).

    python tools/elem_bench.py
Prints per (M, C, variant): time and effective HBM GB/s (algorithmic bytes: every tensor the
kernel must read or write once) for bn_bwd_reduce, bn_bwd_finalize, bn_bwd_apply, bn_apply.
"""
import os
import sys

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
for p in (REPO, os.path.join(REPO, "unet-embroidery-seg_amd")):
    sys.path.insert(0, p)

import torch  # noqa: E402

SHAPES = [(1048576, 64), (262144, 64), (262144, 256), (65536, 128), (65536, 512), (16384, 256), (16384, 1024),
          (4096, 512), (4096, 2048)]


def timeit(fn, reps=20):
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    for _ in range(3):
        fn()
    torch.cuda.synchronize()
    e0.record()
    for _ in range(reps):
        fn()
    e1.record()
    torch.cuda.synchronize()
    return e0.elapsed_time(e1) * 1e-3 / reps


def main():
    from unetseg_hip.lib import DT_BF16, lib

    P = lambda t: 0 if t is None else t.data_ptr()  # noqa: E731
    dev = torch.device("cuda")
    st = torch.cuda.current_stream().cuda_stream
    tot = {}
    for M, C in SHAPES:
        bf = lambda: torch.randn(M, C, device=dev).bfloat16()  # noqa: E731
        dA, Y, A, Y2, out1, out2 = bf(), bf(), bf(), bf(), bf(), bf()
        mean, inv = torch.randn(C, device=dev), torch.rand(C, device=dev) + 0.5
        sc, sh = torch.rand(C, device=dev) + 0.5, torch.randn(C, device=dev)
        g = torch.ones(C, device=dev)
        dg, db = torch.zeros(C, device=dev), torch.zeros(C, device=dev)
        G = lib.reduce_tiles(DT_BF16, M, C, None, None)
        part = torch.empty(3, C, G, device=dev)
        coef = torch.empty(6, C, device=dev)
        S = M * C * 2
        mbits = torch.randint(0, 256, (M * (C // 8),), dtype=torch.uint8, device=dev)
        for var in ("plain", "amask", "amask+y2", "mbits", "mbits+y2"):
            mA = P(A) if var.startswith("amask") else P(mbits) if var.startswith("mbits") else 0
            lda = 0 if var.startswith("mbits") else C
            msc, msh = (P(sc), P(sh)) if var == "plain" else (0, 0)
            y2 = Y2 if var.endswith("+y2") else None
            nt = 2 + (var.startswith("amask")) + (y2 is not None) + (1 / 16 if var.startswith("mbits") else 0)

            def red():
                lib.bn_bwd_reduce(DT_BF16, P(dA), C, mA, lda, msc, msh, P(Y), C, P(mean), P(inv), P(y2), C,
                                  P(mean), P(inv), M, C, P(part), G, st)

            def fin():
                lib.bn_bwd_finalize(P(part), C, G, M, 2 if y2 is not None else 1, P(g), P(inv), P(dg), P(db), P(g),
                                    P(inv), P(dg), P(db), P(coef), st)

            def app():
                lib.bn_bwd_apply(DT_BF16, P(dA), C, mA, lda, msc, msh, P(Y), C, P(mean), P(inv), P(out1), C, P(y2), C,
                                 P(mean), P(inv), P(out2 if y2 is not None else None), C, P(coef), 0, 0, 0, M, C, st)

            t_r, t_f, t_a = timeit(red), timeit(fin), timeit(app)
            na = nt + 1 + (y2 is not None)
            print(f"M={M:8d} C={C:5d} {var:9s} reduce {t_r * 1e6:7.1f} us {nt * S / t_r / 1e9:6.0f} GB/s | "
                  f"finalize {t_f * 1e6:6.1f} us | apply {t_a * 1e6:7.1f} us {na * S / t_a / 1e9:6.0f} GB/s", flush=True)
            for k, t in (("reduce", t_r), ("finalize", t_f), ("apply", t_a)):
                tot[k] = tot.get(k, 0.0) + t

        def fapply():
            lib.bn_apply(DT_BF16, P(Y), C, P(sc), P(sh), P(A), C, 0, 0, 1, 1, P(out1), C, M, C, st)

        t = timeit(fapply)
        print(f"M={M:8d} C={C:5d} bn_apply(res) {t * 1e6:7.1f} us {3 * S / t / 1e9:6.0f} GB/s", flush=True)
        Gs = -(-M // 128)
        sp = torch.randn(Gs, 2, C, device=dev).abs()
        rm, rv, nbt = torch.zeros(C, device=dev), torch.ones(C, device=dev), torch.zeros(1, dtype=torch.int64, device=dev)
        o4 = [torch.empty(C, device=dev) for _ in range(4)]

        def bfin():
            lib.bn_finalize(P(sp), C, Gs, M, 128, P(g), P(sh), P(rm), P(rv), P(nbt), 0.1, 1e-5, *[P(o) for o in o4], st)

        def rows():
            lib.bn_bwd_finalize_rows(P(sp), C, Gs, M, P(g), P(inv), P(dg), P(db), P(coef), st)

        print(f"M={M:8d} C={C:5d} bn_finalize (G={Gs}) {timeit(bfin) * 1e6:6.1f} us  bwd_finalize_rows "
              f"{timeit(rows) * 1e6:6.1f} us", flush=True)
    print({k: round(v * 1e3, 3) for k, v in tot.items()}, "ms summed")


if __name__ == "__main__":
    main()
