"""Kernel-configuration introspection of recorded conv calls (no launches).

``ops.PROBE`` records every conv call of a step as (kind, flops, launches, e0, e1, desc) with
desc = (direction, N, H, W, C1, C2, K, R, S, stride, pad, ld1, ld2).  ``call_configs`` maps one
record to the kernel configurations the library dispatches for it, through the host-only
``unetseg_conv2d_*_config`` queries of the C ABI.  The parity tests use this to prove they cover
every configuration the benchmark step runs; ``tools/bench_conv_configs.py`` prints the table.
"""
from __future__ import annotations

import os

from . import lib as _lib
from .lib import DT_BF16


def _out_hw(H, W, R, S, stride, pad):
    return (H + 2 * pad - R) // stride + 1, (W + 2 * pad - S) // stride + 1


def call_configs(desc, dt=DT_BF16):
    """-> list of configuration keys (strings) one probe record launches"""
    d, N, H, W, C1, C2, K, R, S, stride, pad, ld1, ld2 = desc
    cin = C1 + C2
    if d == "stem_fwd":
        cfg, _ = _lib.stem_config(N, H, W, K)
        return [f"stem_fwd:{cfg}"]
    if d == "stem_wgrad":
        # unetseg_stem_wgrad: the wgrad_fast family (64x256 for K = 64: the LDS-DMA ring when the
        # output width is a multiple of 32, else the register-staged walk), then the split-K reduce
        Qs = (W - 1) // 2 + 1
        ring = Qs % 32 == 0 and not os.environ.get("UNETSEG_WG_NO_RING")
        tile = "wgrad64x256" if K <= 64 else "wgrad128"
        return [f"stem_wgrad:{'wgrad_ring64x256' if ring and K <= 64 else tile}", "reduce"]
    Pq, Qq = _out_hw(H, W, R, S, stride, pad)
    if d == "fwd":
        return ["fwd:" + _lib.fwd_config(dt, C1, ld1 or C1, C2, ld2 or C2, N, H, W, K, R, S, stride, pad)]
    if d == "fwd_affine":  # eval-mode BN on the accumulator: always the generic kernel
        return ["fwd_affine:generic"]
    if d == "fwd_bnrelu_in":  # 1x1 conv applying the producer's BN-ReLU on load (register-staged)
        cfg = _lib.load().unetseg_conv2d_fwd_bnrelu_in_config(dt, C1, ld1 or C1, N, H, W, K)
        return ["fwd_bnrelu_in:" + _lib.CFG_NAMES.get(cfg, str(cfg))]
    if d in ("dgrad", "dgrad_post1", "dgrad_post2", "dgrad_post3", "dgrad_post4"):
        tag = "dgrad" if d == "dgrad" else d
        return [f"{tag}:{c}" for c in _lib.dgrad_config(dt, K, N, Pq, Qq, K, cin, R, S, stride, pad, cin, H, W)]
    if d == "dgrad_padk":
        Kp = -(-K // 64) * 64
        return [f"dgrad:{c}" for c in _lib.dgrad_config(dt, Kp, N, Pq, Qq, Kp, C1, 1, 1, 1, 0, C1, H, W)]
    if d == "wgrad_bnrelu_in":
        kern, sp, red = _lib.wgrad_config(dt, C1, ld1 or C1, 0, 0, N, H, W, K, K, 1, 1, 1, 0)
        return [f"wgrad_bnrelu_in:{kern}", red]
    if d in ("wgrad", "wgrad_padk"):
        Kw = -(-K // 64) * 64 if d == "wgrad_padk" else K
        c2 = 0 if d == "wgrad_padk" else C2
        kern, sp, red = _lib.wgrad_config(dt, C1, ld1 or C1, c2, ld2 or c2, N, H, W, Kw, Kw, R, S, stride, pad)
        return [f"wgrad:{kern}", red]
    raise ValueError(f"unknown probe direction {d!r}")


def probe_table(records, dt=DT_BF16):
    """{config key: [calls, seconds]} over ops.PROBE records (event times summed per call; a
    call's whole bracket -- every parity class, the split-K reduce -- is charged to its first key,
    the reduce key only counts calls)"""
    out = {}
    for kind, flops, nl, e0, e1, desc in records:
        t = e0.elapsed_time(e1) * 1e-3
        for i, key in enumerate(call_configs(desc, dt)):
            v = out.setdefault(key, [0, 0.0])
            v[0] += 1
            if i == 0:
                v[1] += t
    return out
