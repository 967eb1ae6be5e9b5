"""GPU: every conv kernel configuration the benchmark step selects, at shapes that select it.

The library picks a kernel configuration per call from the shape (conv_fast.hip tn_config: halo /
register-staged TN tiles / LDS-DMA rings with compile-time taps; wgrad: halo / LDS-DMA ring /
register-staged tiles with split-K slabs and their reduce).  Each case below names the configuration it must
select -- asserted through the host-only ``unetseg_conv2d_*_config`` queries of the C ABI -- and
checks the launch against a float64 reference computed on the same bf16-rounded operands
(im2col + GEMM in torch float64 on the GPU: exact products, so the only error left is the
kernel's own fp32 accumulation and its single bf16 rounding).

Tolerances (stated here):
  * bf16 outputs (conv output y, data gradient dx, masked gradient d):
    |out - ref| <= 2^-8 |ref| + 1e-4 max|ref|   (one round-to-nearest bf16 rounding = half an ulp
    <= 2^-8 relative, plus fp32 accumulation noise near zero);
  * fp32 weight gradient: |dw - ref| <= 1e-3 |ref| + 2e-5 max|ref|;
  * BN partial statistics / fused backward partials: 1e-4 relative after merging the row tiles.
``test_bench_configs_covered`` runs one real training step of each BASELINE GPU configuration
(unet_resnet50 512x512 B=16, attention_unet and multitask_unet 512x512 B=8) with the probe on and
asserts every configuration it launched appears in CASES.
Shapes follow the reference layers (model/resnet_backbone.py:35-115, model/unet_resnet.py:7-42,70-78).
"""
import math

import numpy as np
import pytest
import torch
import torch.nn.functional as F

pytestmark = pytest.mark.gpu

DEV = "cuda"
RNG = 1234


@pytest.fixture(scope="module", autouse=True)
def _need_gpu():
    if not torch.cuda.is_available():
        pytest.skip("no GPU")
    from unetseg_hip import load
    load()


# id: (direction, (N, H, W, C1, C2, K, R, stride), expected configuration key(s))
#   direction: fwd_relu (bias + ReLU epilogue, decoder) | fwd_stats (BN partials, encoder) |
#              fwd_all (bias + ReLU + stats: every runtime epilogue flag of a TN tile) |
#              dgrad (plain, then accumulated onto a random gradient) | post1 | post2 | wgrad
CASES = {
    # the first 3x3 conv of unet_plain / attention_unet on the 8-channel packed image (conv_first.hip):
    # random values in all 8 channels (the kernel is exact for any 8-channel input), stats / bias + ReLU,
    # attention_unet's C4 shape
    "first3x3_stats": ("fwd_stats", (2, 64, 96, 8, 0, 64, 3, 1), ["fwd:first3x3"]),
    "first3x3_relu": ("fwd_relu", (3, 32, 32, 8, 0, 64, 3, 1), ["fwd:first3x3"]),
    "first3x3_bench": ("fwd_stats", (8, 512, 512, 8, 0, 64, 3, 1), ["fwd:first3x3"]),
    # ---- forward ----
    "fwd_halo3_relu": ("fwd_relu", (2, 64, 256, 64, 0, 64, 3, 1), ["fwd:halo3"]),           # up_conv @512^2 (rows)
    "fwd_halo3_stats": ("fwd_stats", (2, 128, 128, 64, 0, 64, 3, 1), ["fwd:halo3"]),        # layer1 conv2
    # more spatial tiles than persistent blocks, unevenly dealt (320 tiles over 256 / 128 blocks):
    # the three-stage halo pipeline's prefetch of absent tiles and its per-block tile counts
    "fwd_halo3_relu_multi": ("fwd_relu", (5, 128, 128, 64, 0, 64, 3, 1), ["fwd:halo3"]),
    "fwd_halo3_stats_multi": ("fwd_stats", (5, 128, 128, 64, 0, 64, 3, 1), ["fwd:halo3"]),
    "fwd_halo3_k128_multi": ("fwd_all", (3, 128, 128, 64, 0, 128, 3, 1), ["fwd:halo3"]),
    "fwd_ring256x128_t9": ("fwd_all", (16, 32, 32, 1024, 2048, 512, 3, 1), ["fwd:ring256x128_t9"]),  # up_concat4.conv1
    "fwd_ring256x128_t9_s2": ("fwd_stats", (16, 128, 128, 128, 0, 128, 3, 2), ["fwd:ring256x128_t9"]),  # layer2 conv2
    "fwd_ring256x128_t1": ("fwd_stats", (16, 64, 64, 512, 0, 128, 1, 1), ["fwd:ring256x128_t1"]),
    "fwd_ring128x128_5st_t9": ("fwd_stats", (8, 128, 128, 128, 0, 128, 3, 2), ["fwd:ring128x128_5st_t9"]),
    "fwd_ring128x128_5st_t1": ("fwd_stats", (16, 32, 32, 1024, 0, 256, 1, 1), ["fwd:ring128x128_5st_t1"]),
    "fwd_ring128x64_t9": ("fwd_relu", (1, 256, 256, 64, 128, 64, 3, 1), ["fwd:ring128x64_t9"]),  # up_concat1.conv1
    "fwd_ring64x128_t9": ("fwd_stats", (1, 64, 64, 256, 0, 256, 3, 2), ["fwd:ring64x128_t9"]),
    "fwd_ring64x128_t1": ("fwd_stats", (1, 16, 16, 2048, 0, 512, 1, 1), ["fwd:ring64x128_t1"]),
    "fwd_tn128x128_1st": ("fwd_all", (1, 64, 64, 128, 0, 512, 1, 1), ["fwd:tn128x128_1st"]),
    "fwd_tn128x128_1step": ("fwd_stats", (1, 128, 128, 64, 0, 256, 1, 1), ["fwd:tn128x128_1step"]),
    "fwd_tn128x64": ("fwd_stats", (1, 32, 32, 512, 0, 64, 1, 1), ["fwd:tn128x64"]),
    "fwd_tn128x64_1st": ("fwd_all", (16, 128, 128, 256, 0, 64, 1, 1), ["fwd:tn128x64_1st"]),        # layer1 conv1
    "fwd_tn128x64_1st_ragged": ("fwd_stats", (3, 15, 17, 192, 0, 40, 1, 1), ["fwd:tn128x64_1st"]),
    "fwd_tn128x64_1st_k64": ("fwd_stats", (1, 128, 128, 64, 0, 64, 1, 1), ["fwd:tn128x64_1st"]),
    "fwd_tn64x128": ("fwd_all", (1, 64, 64, 512, 0, 128, 1, 1), ["fwd:tn64x128"]),
    # batch 8 (attention_unet / multitask_unet, BASELINE C4 / C5): layer2 conv1 512 -> 128 at 64^2
    "fwd_tn128x128": ("fwd_all", (8, 64, 64, 512, 0, 128, 1, 1), ["fwd:tn128x128"]),
    # generic kernel: an 8-channel first conv whose width is not a multiple of 32 (odd input sizes;
    # the 512^2 / 128^2 configurations run first3x3, the cases above)
    "fwd_generic_cin8": ("fwd_stats", (2, 64, 72, 8, 0, 64, 3, 1), ["fwd:generic"]),
    # ---- data gradient (plain / accumulated) ----
    "dgrad_halo3": ("dgrad", (1, 128, 128, 64, 0, 64, 3, 1), ["dgrad:halo3"]),
    "dgrad_halo3_multi": ("dgrad", (5, 128, 128, 64, 0, 64, 3, 1), ["dgrad:halo3"]),
    "dgrad_ring256x128_t9": ("dgrad", (16, 64, 64, 128, 0, 128, 3, 1), ["dgrad:ring256x128_t9"]),
    "dgrad_ring256x128_t9_cat": ("dgrad", (16, 32, 32, 1024, 2048, 512, 3, 1), ["dgrad:ring256x128_t9"]),
    "dgrad_ring256x128_t1": ("dgrad", (16, 64, 64, 128, 0, 512, 1, 1), ["dgrad:ring256x128_t1"]),
    "dgrad_ring128x128_5st_t9": ("dgrad", (8, 64, 64, 128, 0, 128, 3, 1), ["dgrad:ring128x128_5st_t9"]),
    "dgrad_ring128x128_5st_t1": ("dgrad", (16, 32, 32, 256, 0, 1024, 1, 1), ["dgrad:ring128x128_5st_t1"]),
    "dgrad_ring128x64_t9": ("dgrad", (1, 256, 256, 64, 0, 128, 3, 1), ["dgrad:ring128x64_t9"]),  # attention down1
    "dgrad_ring64x128_t9": ("dgrad", (1, 32, 32, 256, 0, 256, 3, 1), ["dgrad:ring64x128_t9"]),
    "dgrad_ring64x128_t1": ("dgrad", (1, 16, 16, 512, 0, 2048, 1, 1), ["dgrad:ring64x128_t1"]),
    "dgrad_tn128x128_1st": ("dgrad", (1, 64, 64, 512, 0, 128, 1, 1), ["dgrad:tn128x128_1st"]),
    "dgrad_tn128x128_1st_bench": ("dgrad", (16, 128, 128, 256, 0, 128, 1, 1), ["dgrad:tn128x128_1st"]),  # layer2 conv1
    "dgrad_tn128x128_s2": ("dgrad", (2, 64, 64, 256, 0, 512, 1, 2),
                           ["dgrad:tn64x128", "dgrad:tn128x128", "dgrad:tn128x128", "dgrad:tn128x128"]),
    "dgrad_tn128x128_1step": ("dgrad", (1, 128, 128, 256, 0, 64, 1, 1), ["dgrad:tn128x128_1step"]),
    "dgrad_tn128x64": ("dgrad", (1, 32, 32, 64, 0, 512, 1, 1), ["dgrad:tn128x64"]),
    "dgrad_tn128x64_1st_k64": ("dgrad", (1, 128, 128, 64, 0, 64, 1, 1), ["dgrad:tn128x64_1st"]),
    "dgrad_tn128x64_1st": ("dgrad", (16, 128, 128, 64, 0, 256, 1, 1), ["dgrad:tn128x64_1st"]),
    "dgrad_tn128x128_1st_ragged": ("dgrad", (3, 15, 17, 136, 0, 192, 1, 1), ["dgrad:tn128x128_1st"]),
    # ---- data gradient with the producer's ReLU (post 1) / BN-ReLU (post 2) backward fused ----
    "post1_halo3": ("post1", (2, 64, 256, 64, 0, 64, 3, 1), ["dgrad_post1:halo3"]),
    "post1_ring256x128_t9": ("post1", (16, 32, 32, 512, 0, 512, 3, 1), ["dgrad_post1:ring256x128_t9"]),
    "post1_ring128x128_5st_t9": ("post1", (8, 64, 64, 128, 0, 128, 3, 1), ["dgrad_post1:ring128x128_5st_t9"]),
    "post2_halo3": ("post2", (1, 128, 128, 64, 0, 64, 3, 1), ["dgrad_post2:halo3"]),
    "post1_halo3_multi": ("post1", (5, 128, 128, 64, 0, 64, 3, 1), ["dgrad_post1:halo3"]),
    "post2_halo3_multi": ("post2", (5, 128, 128, 64, 0, 64, 3, 1), ["dgrad_post2:halo3"]),
    "post2_tn128x128_1st": ("post2", (1, 64, 64, 512, 0, 128, 1, 1), ["dgrad_post2:tn128x128_1st"]),
    # batch 8: layer2 conv3 (128 -> 512 at 64^2), its data gradient with bn2-ReLU's backward fused
    "post2_tn128x128": ("post2", (8, 64, 64, 128, 0, 512, 1, 1), ["dgrad_post2:tn128x128"]),
    "post2_tn64x128": ("post2", (1, 64, 64, 128, 0, 512, 1, 1), ["dgrad_post2:tn64x128"]),
    "post2_tn128x64": ("post2", (1, 32, 32, 64, 0, 512, 1, 1), ["dgrad_post2:tn128x64"]),
    "post2_tn128x64_1st_k64": ("post2", (1, 128, 128, 64, 0, 64, 1, 1), ["dgrad_post2:tn128x64_1st"]),
    "post2_tn128x64_1st": ("post2", (16, 128, 128, 64, 0, 256, 1, 1), ["dgrad_post2:tn128x64_1st"]),  # layer1 conv3
    "post2_ring128x128_5st_t9": ("post2", (8, 64, 64, 128, 0, 128, 3, 1), ["dgrad_post2:ring128x128_5st_t9"]),
    "post2_ring128x128_5st_t1": ("post2", (16, 32, 32, 256, 0, 1024, 1, 1), ["dgrad_post2:ring128x128_5st_t1"]),
    # stride-2 3x3: the four parity classes have 4 / 2 / 2 / 1 taps -> generic ring, ring_t1, ...
    "post2_ring256x128_s2": ("post2", (16, 128, 128, 128, 0, 128, 3, 2), ["dgrad_post2:multi128x128"] * 4),
    "post2_ring256x128_t9": ("post2", (16, 64, 64, 128, 0, 128, 3, 1), ["dgrad_post2:ring256x128_t9"]),
    "post2_ring256x128_t1": ("post2", (16, 64, 64, 128, 0, 512, 1, 1), ["dgrad_post2:ring256x128_t1"]),
    "post2_ring64x128_s2": ("post2", (1, 32, 32, 512, 0, 512, 3, 2), ["dgrad_post2:multi64x128"] * 4),
    # stride-2 3x3 data gradients: the four parity classes in one launch (launch_tn_multi)
    "dgrad_multi128x128_s2": ("dgrad", (16, 64, 64, 256, 0, 256, 3, 2), ["dgrad:multi128x128"] * 4),
    "dgrad_multi64x128_s2": ("dgrad", (16, 32, 32, 512, 0, 512, 3, 2), ["dgrad:multi64x128"] * 4),
    "dgrad_multi_ragged_s2": ("dgrad", (2, 17, 23, 128, 0, 192, 3, 2), None),
    "post2_multi_ragged_s2": ("post2", (2, 17, 23, 128, 0, 192, 3, 2), None),
    "post2_ring64x128_t9": ("post2", (1, 32, 32, 256, 0, 256, 3, 1), ["dgrad_post2:ring64x128_t9"]),
    "post2_ring64x128_t1": ("post2", (1, 16, 16, 512, 0, 2048, 1, 1), ["dgrad_post2:ring64x128_t1"]),
    # ---- weight gradient (+ split-K reduce) ----
    "wgrad_halo3": ("wgrad", (2, 64, 256, 64, 0, 64, 3, 1), ["wgrad:halo3_wgrad", None]),
    "wgrad_halo3_cat": ("wgrad", (16, 32, 32, 1024, 2048, 512, 3, 1), ["wgrad:halo3_wgrad", None]),
    "wgrad_ring128_r16": ("wgrad", (16, 128, 128, 64, 0, 256, 1, 1), ["wgrad:wgrad_ring128", "reduce"]),
    "wgrad_ring128_r4": ("wgrad", (1, 64, 64, 128, 0, 512, 1, 1), ["wgrad:wgrad_ring128", "reduce"]),
    "wgrad_ring128_r1": ("wgrad", (1, 32, 32, 256, 0, 1024, 1, 1), ["wgrad:wgrad_ring128", "reduce"]),
    "wgrad_ring128_s2": ("wgrad", (16, 32, 32, 512, 0, 512, 3, 2), ["wgrad:wgrad_ring128", None]),
    "wgrad_ring128_1x1s2": ("wgrad", (2, 32, 32, 256, 0, 512, 1, 2), ["wgrad:wgrad_ring128", None]),
    # 8-wide rows (4 rows per K step), a partial column tile (Ng = 576), padding taps
    "wgrad_ring128_q8": ("wgrad", (2, 8, 8, 64, 0, 128, 3, 1), ["wgrad:wgrad_ring128", None]),
    "wgrad_ring128_16x16": ("wgrad", (16, 16, 16, 2048, 0, 512, 1, 1), ["wgrad:wgrad_ring128", None]),
    # register-staged kernels: K steps that straddle rows (ragged grids), a concat source
    "wgrad128_ragged": ("wgrad", (1, 15, 17, 64, 0, 256, 1, 1), ["wgrad:wgrad128", None]),
    "wgrad64x256_ragged": ("wgrad", (1, 15, 17, 256, 0, 64, 1, 1), ["wgrad:wgrad64x256", None]),
    "wgrad128_row_cat": ("wgrad", (2, 64, 64, 64, 64, 256, 1, 1), ["wgrad:wgrad128_row", None]),
    "wgrad_ring64x256": ("wgrad", (16, 128, 128, 256, 0, 64, 1, 1), ["wgrad:wgrad_ring64x256", "reduce"]),
    # bottleneck conv3 reading bn2-ReLU on load (ops.bn(lazy=True), unetseg_conv2d_*_bnrelu_in)
    "bnin_tn128x128_1step": ("fwd_bnrelu_in", (16, 128, 128, 64, 0, 256, 1, 1), ["fwd_bnrelu_in:tn128x128_1step"]),
    "bnin_tn128x128_1st": ("fwd_bnrelu_in", (16, 64, 64, 128, 0, 512, 1, 1), ["fwd_bnrelu_in:tn128x128_1st"]),
    "bnin_tn128x128_1st_k256": ("fwd_bnrelu_in", (16, 32, 32, 256, 0, 1024, 1, 1), ["fwd_bnrelu_in:tn128x128_1st"]),
    "bnin_tn256x128": ("fwd_bnrelu_in", (16, 16, 16, 512, 0, 2048, 1, 1), ["fwd_bnrelu_in:tn256x128"]),
    "bnin_tn64x128": ("fwd_bnrelu_in", (1, 16, 16, 512, 0, 2048, 1, 1), ["fwd_bnrelu_in:tn64x128"]),
    # batch 8: layer4 conv3 (512 -> 2048 at 16^2) reading bn2-ReLU on load
    "bnin_tn128x128": ("fwd_bnrelu_in", (8, 16, 16, 512, 0, 2048, 1, 1), ["fwd_bnrelu_in:tn128x128"]),
    "bnin_ragged": ("fwd_bnrelu_in", (1, 15, 17, 64, 0, 256, 1, 1), None),
    "bnin_wgrad_ring_r16": ("wgrad_bnrelu_in", (16, 128, 128, 64, 0, 256, 1, 1), ["wgrad_bnrelu_in:wgrad_ring128", "reduce"]),
    "bnin_wgrad_ring_r4": ("wgrad_bnrelu_in", (1, 64, 64, 128, 0, 512, 1, 1), ["wgrad_bnrelu_in:wgrad_ring128", "reduce"]),
    "bnin_wgrad_ring64x256": ("wgrad_bnrelu_in", (2, 32, 32, 256, 0, 64, 1, 1), ["wgrad_bnrelu_in:wgrad_ring64x256", None]),
    "bnin_wgrad_ring_16x16": ("wgrad_bnrelu_in", (16, 16, 16, 512, 0, 2048, 1, 1), ["wgrad_bnrelu_in:wgrad_ring128", None]),
    "bnin_wgrad_ragged": ("wgrad_bnrelu_in", (1, 15, 17, 64, 0, 256, 1, 1), ["wgrad_bnrelu_in:wgrad128", None]),
}


def _bf(t):
    return t.to(torch.bfloat16)


def _nhwc(t):
    return t.permute(0, 2, 3, 1).contiguous()


def _nchw(t):
    return t.permute(0, 3, 1, 2).double()


def _out_hw(H, W, R, stride):
    pad = R // 2
    return (H + 2 * pad - R) // stride + 1, (W + 2 * pad - R) // stride + 1


def _ref_fwd(x, w, stride, pad):
    """float64 conv via im2col (x [N,C,H,W] f64, w [K,C,R,S] f64)"""
    N = x.shape[0]
    K, C, R, S = w.shape
    cols = F.unfold(x, (R, S), padding=pad, stride=stride)
    P, Q = (x.shape[2] + 2 * pad - R) // stride + 1, (x.shape[3] + 2 * pad - S) // stride + 1
    return (w.reshape(K, -1) @ cols).reshape(N, K, P, Q)


def _ref_dgrad(dy, w, H, W, stride, pad):
    N, K, P, Q = dy.shape
    _, C, R, S = w.shape
    cols = w.reshape(K, -1).t() @ dy.reshape(N, K, P * Q)
    return F.fold(cols, (H, W), (R, S), padding=pad, stride=stride)


def _ref_wgrad(x, dy, R, stride, pad):
    N, K, P, Q = dy.shape
    cols = F.unfold(x, (R, R), padding=pad, stride=stride)  # [N, C*R*R, L]
    return torch.einsum("nkl,ncl->kc", dy.reshape(N, K, P * Q), cols).reshape(K, x.shape[1], R, R)


def _check_bf16(out, ref, what):
    out, ref = out.double(), ref.double()
    m = ref.abs().max().item()
    err = (out - ref).abs()
    bound = 2.0 ** -8 * ref.abs() + 1e-4 * m
    bad = (err > bound).sum().item()
    assert bad == 0, f"{what}: {bad} elements outside 2^-8|ref| + 1e-4 max|ref| (max err {err.max().item():.3e}, max|ref| {m:.3e})"


def _key_list(direction, shape):
    from unetseg_hip import introspect
    N, H, W, C1, C2, K, R, s = shape
    d = {"fwd_relu": "fwd", "fwd_stats": "fwd", "fwd_all": "fwd", "dgrad": "dgrad", "post1": "dgrad_post1",
         "post2": "dgrad_post2", "wgrad": "wgrad", "fwd_bnrelu_in": "fwd_bnrelu_in",
         "wgrad_bnrelu_in": "wgrad_bnrelu_in"}[direction]
    return introspect.call_configs((d, N, H, W, C1, C2, K, R, R, s, R // 2, C1, C2))


# residual post-op data gradients (dgrad_post3): the configurations tests/test_gpu_post_res.py drives
# (N, H, W, K, C) of its SHAPES with a fixed configuration
POST3_SHAPES = [(16, 128, 128, 64, 256), (4, 64, 64, 128, 512), (16, 32, 32, 256, 1024), (16, 16, 16, 512, 2048),
                (16, 128, 128, 128, 256), (16, 64, 64, 256, 512), (16, 32, 32, 512, 1024)]


RELU_BITS_SHAPES = [(16, 512, 512), (2, 64, 96)]


def covered_keys():
    import os
    from unetseg_hip import introspect
    keys = set()
    for N, H, W, K, C in POST3_SHAPES:
        keys.update(introspect.call_configs(("dgrad_post3", N, H, W, C, 0, K, 1, 1, 1, 0, C, 0)))
    # ReLU-bit data gradients (dgrad_post4): tests/test_gpu_relu_bits.py's shapes
    for N, H, W in RELU_BITS_SHAPES:
        keys.update(introspect.call_configs(("dgrad_post4", N, H, W, 64, 0, 64, 3, 3, 1, 1, 64, 0)))
    for env in HALO_MODES.values():
        saved = {k: os.environ.get(k) for k in env}
        os.environ.update(env)
        try:
            for direction, shape, _ in HALO_CASES.values():
                keys.update(_key_list(direction, shape))
        finally:
            for k, v in saved.items():
                if v is None:
                    del os.environ[k]
                else:
                    os.environ[k] = v
    for direction, shape, expect in CASES.values():
        if not _gather_ring(expect):
            keys.update(_key_list(direction, shape))
            continue
        old = os.environ.get("UNETSEG_TN_NO_HALO_RING")
        os.environ["UNETSEG_TN_NO_HALO_RING"] = "1"
        try:
            keys.update(_key_list(direction, shape))
        finally:
            if old is None:
                del os.environ["UNETSEG_TN_NO_HALO_RING"]
            else:
                os.environ["UNETSEG_TN_NO_HALO_RING"] = old
    return keys


class _Op:
    """operands of one case: bf16-rounded x (cat of x1, x2), w, dy on the device"""

    def __init__(self, shape, seed):
        N, H, W, C1, C2, K, R, s = shape
        g = torch.Generator(device=DEV).manual_seed(seed)
        self.shape = shape
        cin = C1 + C2
        self.pad = R // 2
        self.P, self.Q = _out_hw(H, W, R, s)
        self.x = _bf(torch.randn(N, cin, H, W, generator=g, device=DEV))
        self.w32 = _bf(torch.randn(K, cin, R, R, generator=g, device=DEV) / math.sqrt(cin * R * R)).float()
        self.dy = _bf(torch.randn(N, K, self.P, self.Q, generator=g, device=DEV))
        self.bias = torch.randn(K, generator=g, device=DEV) * 0.1
        self.gen = g

    def x_parts(self):
        N, H, W, C1, C2, K, R, s = self.shape
        x1 = _nhwc(self.x[:, :C1])
        x2 = _nhwc(self.x[:, C1:]) if C2 else None
        return x1, x2

    def packed(self):
        from unetseg_hip.lib import DT_BF16, lib
        K, C, R, S = self.w32.shape
        wk = torch.empty(K, R, S, C, dtype=torch.bfloat16, device=DEV)
        wt = torch.empty(C, R, S, K, dtype=torch.bfloat16, device=DEV)
        lib.pack_conv_weight(DT_BF16, self.w32.data_ptr(), K, C, R, S, C, wk.data_ptr(), wt.data_ptr(), _st())
        return wk, wt


def _st():
    return torch.cuda.current_stream().cuda_stream


def _P(t):
    return 0 if t is None else t.data_ptr()


# the halo-A ring (configuration 21: 3x3 stride-1 convs on 8 x 32 spatial tiles, A operand from a
# per-chunk halo in LDS) takes the 256x128 gather ring's place where it applies (the default); the
# gather-ring cases of those shapes run with UNETSEG_TN_NO_HALO_RING=1 (read per call)
HALO_CASES = {
    "hring_fwd_cat": ("fwd_all", (16, 32, 32, 1024, 2048, 512, 3, 1), ["fwd:ring256x128_halo"]),  # up_concat4.conv1
    "hring_fwd_cat_c1_128": ("fwd_all", (16, 64, 64, 128, 64, 256, 3, 1), ["fwd:ring256x128_halo"]),
    "hring_fwd_stats": ("fwd_stats", (16, 64, 64, 256, 0, 256, 3, 1), ["fwd:ring256x128_halo"]),
    "hring_fwd_ng192": ("fwd_all", (16, 64, 64, 128, 0, 192, 3, 1), ["fwd:ring256x128_halo"]),
    "hring_dgrad": ("dgrad", (16, 64, 64, 256, 0, 256, 3, 1), ["dgrad:ring256x128_halo"]),
    "hring_dgrad_cat": ("dgrad", (16, 128, 128, 256, 256, 128, 3, 1), ["dgrad:ring256x128_halo"]),  # up_concat2.conv1
    "hring_post1": ("post1", (16, 32, 32, 512, 0, 512, 3, 1), ["dgrad_post1:ring256x128_halo"]),
    "hring_post2": ("post2", (16, 64, 64, 128, 0, 128, 3, 1), ["dgrad_post2:ring256x128_halo"]),
    # <= 64 output channels: 256x64 tiles (up_concat1.conv1 192 -> 64 at 256^2, here at 64^2)
    "hring64_fwd_cat": ("fwd_all", (2, 64, 64, 64, 128, 64, 3, 1), ["fwd:ring256x64_halo"]),
    "hring64_fwd_stats_k40": ("fwd_stats", (2, 64, 96, 192, 0, 40, 3, 1), ["fwd:ring256x64_halo"]),
    "hring64_dgrad": ("dgrad", (2, 64, 64, 64, 0, 128, 3, 1), ["dgrad:ring256x64_halo"]),
    "hring64_post1": ("post1", (2, 32, 64, 64, 0, 128, 3, 1), ["dgrad_post1:ring256x64_halo"]),
    # one or two 128x128 tiles per CU: 4 x 32 tiles (layer3 conv2 256 -> 256 at 32^2)
    "hring128_fwd_stats": ("fwd_stats", (16, 32, 32, 256, 0, 256, 3, 1), ["fwd:ring128x128_halo"]),
    "hring128_post2": ("post2", (16, 32, 32, 256, 0, 256, 3, 1), ["dgrad_post2:ring128x128_halo"]),
    "hring128_dgrad_ng192": ("dgrad", (8, 32, 64, 384, 0, 192, 3, 1), ["dgrad:ring128x128_halo"]),
    "hring128_post1": ("post1", (8, 32, 32, 512, 0, 512, 3, 1), ["dgrad_post1:ring128x128_halo"]),  # B=8 up_concat4.conv2
}


def _gather_ring(expect):
    """a case written for the 256x128 gather ring on a shape the halo-A ring now takes"""
    return bool(expect) and any(k is not None and k.endswith(("ring256x128_t9", "ring128x64_t9", "ring128x128_5st_t9"))
                                for k in expect)


def _persist_keys(expect):
    """the keys of a halo-A ring case under the persistent kernel (configurations 24 / 25)"""
    return [k.replace("ring256x128_halo", "ring256x128_hp").replace("ring256x64_halo", "ring256x64_hp")
            if k is not None else None for k in expect]


#: halo-A ring modes: the one-tile-per-block kernel (UNETSEG_TN_PERSIST=0) and the persistent kernel
#: (tn_halo_persist_kernel) at a fixed 3 tiles per block -- every case then pipelines across tile
#: boundaries (the next tile's halo and weight stages in flight through the epilogue), and the last
#: block of most shapes gets a ragged share
HALO_MODES = {"plain": {"UNETSEG_TN_PERSIST": "0"}, "persist3": {"UNETSEG_TN_PERSIST_T": "3"}}


@pytest.mark.parametrize("mode", list(HALO_MODES))
@pytest.mark.parametrize("cid", list(HALO_CASES))
def test_halo_ring_case(cid, mode, monkeypatch):
    for k, v in HALO_MODES[mode].items():
        monkeypatch.setenv(k, v)
    direction, shape, expect = HALO_CASES[cid]
    _run_case(cid, direction, shape, _persist_keys(expect) if mode == "persist3" else expect)


@pytest.mark.parametrize("cid", list(CASES))
def test_config_case(cid, monkeypatch):
    if _gather_ring(CASES[cid][2]):
        monkeypatch.setenv("UNETSEG_TN_NO_HALO_RING", "1")
    _run_case(cid, *CASES[cid])


def _run_case(cid, direction, shape, expect):
    from unetseg_hip.lib import DT_BF16, lib
    keys = _key_list(direction, shape)
    if expect is not None:
        got = [k for k in keys if k is not None]
        want = [k for k in expect if k is not None]
        assert got[:len(want)] == want, f"{cid}: selects {keys}, expected {expect}"
    N, H, W, C1, C2, K, R, s = shape
    cin = C1 + C2
    op = _Op(shape, RNG + sum(map(ord, cid)))
    pad, P, Q = op.pad, op.P, op.Q
    x64, w64, dy64 = op.x.double(), op.w32.double(), op.dy.double()
    wk, wt = op.packed()
    st = _st()
    if direction.endswith("bnrelu_in"):
        _bnrelu_in_case(cid, direction, shape, op, wk, lib, st)
        return
    if direction.startswith("fwd"):
        x1, x2 = op.x_parts()
        relu = direction in ("fwd_relu", "fwd_all")
        stats = direction in ("fwd_stats", "fwd_all")
        bias = op.bias if relu else None
        M = N * P * Q
        tile = lib.conv2d_fwd_tile_m(DT_BF16, C1, C1, C2, C2, N, H, W, K, R, R, s, pad)
        G = -(-M // tile)
        stt = torch.empty(G, 2, K, dtype=torch.float32, device=DEV) if stats else None
        y = torch.empty(N, P, Q, K, dtype=torch.bfloat16, device=DEV)
        lib.conv2d_fwd(DT_BF16, _P(x1), C1, C1, _P(x2), C2, C2, N, H, W, _P(wk), K, R, R, s, pad, _P(bias), int(relu),
                       _P(y), K, _P(stt), st)
        ref = _ref_fwd(x64, w64, s, pad)
        if relu:
            ref = torch.relu(ref + op.bias.double().view(1, -1, 1, 1))
        out = _nchw(y)
        _check_bf16(out, ref, f"{cid} y")
        if stats:
            # merge the per-row-tile (sum, M2) partials and compare with the stored outputs' stats
            st_ = stt.double()
            cnt = torch.tensor([min(tile, M - g_ * tile) for g_ in range(G)], dtype=torch.float64, device=DEV)
            tot = st_[:, 0].sum(0)
            mean = tot / M
            m2 = (st_[:, 1] + cnt[:, None] * (st_[:, 0] / cnt[:, None] - mean) ** 2).sum(0)
            o = out.permute(1, 0, 2, 3).reshape(K, -1)
            torch.testing.assert_close(tot, o.sum(1), rtol=1e-4, atol=1e-4 * o.abs().sum(1).max().item() / M * 10)
            torch.testing.assert_close(m2 / M, o.var(1, unbiased=False), rtol=1e-4, atol=1e-6)
        return
    if direction in ("dgrad", "post1", "post2"):
        dyh = _nhwc(op.dy)
        ref = _ref_dgrad(dy64, w64, H, W, s, pad)
        dx = torch.empty(N, H, W, cin, dtype=torch.bfloat16, device=DEV)
        if direction == "dgrad":
            lib.conv2d_dgrad(DT_BF16, _P(dyh), K, N, P, Q, _P(wt), K, cin, R, R, s, pad, _P(dx), cin, H, W, 0, st)
            _check_bf16(_nchw(dx), ref, f"{cid} dx")
            # accumulate onto an existing gradient: dx' = bf16(float(dx0) + float(bf16 dgrad))
            g0 = _bf(torch.randn(N, H, W, cin, generator=op.gen, device=DEV))
            dx.copy_(g0)
            lib.conv2d_dgrad(DT_BF16, _P(dyh), K, N, P, Q, _P(wt), K, cin, R, R, s, pad, _P(dx), cin, H, W, 1, st)
            # either rounding order (the TN epilogue rounds the dgrad first, halo adds the fp32
            # value): within half an ulp of the dgrad plus half an ulp of the sum
            acc_ref = _nchw(g0) + ref
            err = (_nchw(dx) - acc_ref).abs()
            bound = 2.0 ** -8 * (ref.abs() + acc_ref.abs()) + 1e-4 * ref.abs().max().item()
            assert int((err > bound).sum()) == 0, f"{cid} dx accumulated: max err {err.max().item():.3e}"
            return
        post = 1 if direction == "post1" else 2
        # aux: the producer's output (post 1: ReLU output >= 0 with zeros; post 2: BN input z)
        z = _bf(torch.randn(N, H, W, cin, generator=op.gen, device=DEV))
        aux = torch.relu(z) if post == 1 else z
        sc = (1 + 0.3 * torch.randn(cin, generator=op.gen, device=DEV)).float()
        sh = (0.3 * torch.randn(cin, generator=op.gen, device=DEV)).float()
        mu = (0.1 * torch.randn(cin, generator=op.gen, device=DEV)).float()
        inv = (1 + 0.2 * torch.rand(cin, generator=op.gen, device=DEV)).float()
        coeffs = [_P(sc), _P(sh), _P(mu), _P(inv)] if post == 2 else [0, 0, 0, 0]
        args = [DT_BF16, _P(dyh), K, N, P, Q, _P(wt), K, cin, R, R, s, pad]
        rows = lib.conv2d_dgrad_post(*args, 0, cin, H, W, post, _P(aux), cin, *coeffs, 0, 0, st)
        assert rows > 0, f"{cid}: shape has no fused path"
        part = torch.empty(rows, 2, cin, dtype=torch.float32, device=DEV)
        rc = lib.conv2d_dgrad_post(*args, _P(dx), cin, H, W, post, _P(aux), cin, *coeffs, _P(part), rows, st)
        assert rc == 0
        a64 = _nchw(aux)
        if post == 1:
            mask = a64 > 0
        else:  # sign of fmaf(z, sc, sh): exact in float64 (24x24-bit product)
            mask = (a64 * sc.double().view(1, -1, 1, 1) + sh.double().view(1, -1, 1, 1)) > 0
        d = _nchw(dx)
        _check_bf16(d, torch.where(mask, ref, torch.zeros_like(ref)), f"{cid} d")
        assert (d[~mask] == 0).all()
        # fused reduction over the stored (rounded, masked) d
        q0 = d.sum((0, 2, 3))
        torch.testing.assert_close(part[:, 0].double().sum(0), q0, rtol=1e-4, atol=1e-4 * d.abs().sum((0, 2, 3)).max().item() / d[:, 0].numel())
        if post == 2:
            xhat = (a64 - mu.double().view(1, -1, 1, 1)) * inv.double().view(1, -1, 1, 1)
            q1 = (d * xhat).sum((0, 2, 3))
            scale = (d * xhat).abs().sum((0, 2, 3)).max().item() / d[:, 0].numel()
            torch.testing.assert_close(part[:, 1].double().sum(0), q1, rtol=1e-4, atol=1e-4 * scale)
        return
    # weight gradient
    x1, x2 = op.x_parts()
    dyh = _nhwc(op.dy)
    ws_bytes = lib.conv2d_wgrad_workspace(DT_BF16, N, P, Q, K, cin, R, R)
    ws = torch.empty(max(ws_bytes, 1) // 4 + 1, dtype=torch.float32, device=DEV)
    dw = torch.empty(K, cin, R, R, dtype=torch.float32, device=DEV)
    lib.conv2d_wgrad(DT_BF16, _P(x1), C1, C1, _P(x2), C2, C2, N, H, W, _P(dyh), K, K, R, R, s, pad, _P(ws), ws_bytes,
                     _P(dw), cin, 0, st)
    ref = _ref_wgrad(x64, dy64, R, s, pad)
    m = ref.abs().max().item()
    err = (dw.double() - ref).abs()
    bad = (err > 1e-3 * ref.abs() + 2e-5 * m).sum().item()
    assert bad == 0, f"{cid}: {bad} dw elements out of tolerance (max err {err.max().item():.3e}, max|ref| {m:.3e})"
    # accumulate (deterministic split-K order: the second pass adds exactly the same values)
    dw1 = dw.clone()
    lib.conv2d_wgrad(DT_BF16, _P(x1), C1, C1, _P(x2), C2, C2, N, H, W, _P(dyh), K, K, R, R, s, pad, _P(ws), ws_bytes,
                     _P(dw), cin, 1, st)
    assert torch.equal(dw, dw1 + dw1), f"{cid}: accumulated wgrad is not 2x the first (non-deterministic reduce?)"


def _bnrelu_in_case(cid, direction, shape, op, wk, lib, st):
    """x1 = z (the producer's BN input); the conv must read a = bf16(relu(fmaf(z, sc, sh))), as the
    bn_apply pass would have stored it.  fwd: output and BN partials vs the float64 conv of a;
    wgrad: dW vs the float64 reference and bit-equal to the plain wgrad of the materialised a."""
    from unetseg_hip.lib import DT_BF16
    N, H, W, C1, C2, K, R, s = shape
    z = _nhwc(op.x)
    sc = (1 + 0.3 * torch.randn(C1, generator=op.gen, device=DEV)).float()
    sh = (0.3 * torch.randn(C1, generator=op.gen, device=DEV)).float()
    # fmaf(z, sc, sh) = the exact value rounded once to fp32 (exact in float64: 8 x 24-bit product)
    a = torch.relu((z.double() * sc.double() + sh.double()).float()).to(torch.bfloat16)
    a64 = _nchw(a)
    if direction == "fwd_bnrelu_in":
        M = N * H * W
        tile = lib.conv2d_fwd_tile_m(DT_BF16, C1, C1, 0, 0, N, H, W, K, 1, 1, 1, 0)
        G = -(-M // tile)
        stt = torch.empty(G, 2, K, dtype=torch.float32, device=DEV)
        y = torch.empty(N, H, W, K, dtype=torch.bfloat16, device=DEV)
        lib.conv2d_fwd_bnrelu_in(DT_BF16, _P(z), C1, C1, N, H, W, _P(wk), K, _P(sc), _P(sh), 0, 0, _P(y), K, _P(stt),
                                 st)
        ref = _ref_fwd(a64, op.w32.double(), 1, 0)
        out = _nchw(y)
        _check_bf16(out, ref, f"{cid} y")
        # same values as the unfused conv of the stored activation
        y2 = torch.empty_like(y)
        st2 = torch.empty_like(stt)
        lib.conv2d_fwd(DT_BF16, _P(a), C1, C1, 0, 0, 0, N, H, W, _P(wk), K, 1, 1, 1, 0, 0, 0, _P(y2), K, _P(st2), st)
        torch.testing.assert_close(y.float(), y2.float(), rtol=0, atol=0)
        torch.testing.assert_close(stt, st2, rtol=1e-6, atol=1e-5)
        return
    dyh = _nhwc(op.dy)
    ws_bytes = lib.conv2d_wgrad_workspace(DT_BF16, N, H, W, K, C1, 1, 1)
    ws = torch.empty(max(ws_bytes, 1) // 4 + 1, dtype=torch.float32, device=DEV)
    dw = torch.empty(K, C1, 1, 1, dtype=torch.float32, device=DEV)
    lib.conv2d_wgrad_bnrelu_in(DT_BF16, _P(z), C1, C1, N, H, W, _P(dyh), K, K, _P(sc), _P(sh), _P(ws), ws_bytes, _P(dw),
                               C1, 0, st)
    ref = _ref_wgrad(a64, op.dy.double(), 1, 1, 0)
    m = ref.abs().max().item()
    err = (dw.double() - ref).abs()
    assert int((err > 1e-3 * ref.abs() + 2e-5 * m).sum()) == 0, f"{cid}: max err {err.max().item():.3e}"
    dw2 = torch.empty_like(dw)
    lib.conv2d_wgrad(DT_BF16, _P(a), C1, C1, 0, 0, 0, N, H, W, _P(dyh), K, K, 1, 1, 1, 0, _P(ws), ws_bytes, _P(dw2), C1,
                     0, st)
    assert torch.equal(dw, dw2), f"{cid}: fused wgrad differs from the wgrad of the stored activation"


@pytest.mark.parametrize("N,H,tn,expect", [(16, 512, False, "stem_halo"), (16, 512, True, "tn128x64"),
                                           (2, 200, False, "tn128x64"), (3, 256, False, "stem_halo")])
def test_stem_bench_size(N, H, tn, expect, monkeypatch):
    """ResNet stem at the benchmark size (model/resnet_backbone.py:126-131): 7x7/s2/p3 3->64 on the
    width-packed fast kernels (stem_fwd: the persistent-halo stem kernel when the output tiles into
    16 x 32 pixels, else -- or with UNETSEG_STEM_TN=1 -- the TN 128x64 tile; stem_wgrad: 64x256 split-K
    ring + reduce); y and the BN statistics' inputs against float64."""
    from unetseg_hip import ops
    from unetseg_hip.lib import DT_BF16, stem_config
    from unetseg_hip.nn import Conv2d
    if tn:
        monkeypatch.setenv("UNETSEG_STEM_TN", "1")
    cfg, splits = stem_config(N, H, H, 64)
    assert cfg == expect and splits >= 16, (cfg, splits)
    g = torch.Generator(device=DEV).manual_seed(N + H)
    conv = Conv2d(3, 64, 7, stride=2, padding=3, bias=False).to(DEV)
    with torch.no_grad():
        conv.weight.copy_(_bf(torch.randn(64, 3, 7, 7, generator=g, device=DEV) / math.sqrt(147)).float())
    conv.weight.grad = torch.zeros_like(conv.weight)
    x = torch.rand(N, 3, H, H, generator=g, device=DEV)
    ctx = ops.Ctx(DT_BF16, True, True, torch.device(DEV))
    y, (stt, tile) = ops.stem_conv(ctx, x, conv)
    xr = _bf(x).double()
    ref = _ref_fwd(xr, conv.weight.detach().double(), 2, 3)
    _check_bf16(_nchw(y.data), ref, "stem y")
    # the BN partials (sum, M2 about the tile mean per row tile) merge to the stored output's statistics
    M = y.data.shape[0] * y.data.shape[1] * y.data.shape[2]
    G = stt.shape[0]
    st_ = stt.double()
    cnt = torch.tensor([min(tile, M - g_ * tile) for g_ in range(G)], dtype=torch.float64, device=DEV)
    tot = st_[:, 0].sum(0)
    mean = tot / M
    m2 = (st_[:, 1] + cnt[:, None] * (st_[:, 0] / cnt[:, None] - mean) ** 2).sum(0)
    o = y.data.reshape(M, -1).double().t()
    torch.testing.assert_close(tot, o.sum(1), rtol=1e-4, atol=1e-4 * o.abs().sum(1).max().item() / M * 10)
    torch.testing.assert_close(m2 / M, o.var(1, unbiased=False), rtol=1e-4, atol=1e-6)
    dy = _bf(torch.randn(ref.shape, generator=g, device=DEV))
    y.grad = _nhwc(dy)
    ctx.backward()
    torch.cuda.synchronize()
    dref = _ref_wgrad(xr, dy.double(), 7, 2, 3)
    err = (conv.weight.grad.double() - dref).abs()
    m = dref.abs().max().item()
    assert (err <= 1e-3 * dref.abs() + 2e-5 * m).all(), err.max().item()


@pytest.mark.parametrize("model_name,batch", [("unet_resnet50", 16), ("attention_unet", 8), ("multitask_unet", 8)])
def test_bench_configs_covered(model_name, batch):
    """One real training step of each BASELINE GPU configuration (C2/C3: unet_resnet50 512x512 B=16,
    Lovasz + Adam; C4: attention_unet 512x512 B=8; C5: multitask_unet 512x512 B=8, BCE + CE) with the
    probe on: every kernel configuration it launches must be exercised by a case above."""
    import contextlib
    import io

    from model.model_factory import create_model
    from unetseg_hip import introspect, ops
    from unetseg_hip.arena import FusedAdam
    from unetseg_hip.losses import binary_segmentation_loss, multitask_loss
    from utils.synthetic import make_batch
    multitask = model_name == "multitask_unet"
    with contextlib.redirect_stdout(io.StringIO()):
        model = create_model(model_name, num_classes=1 if multitask else 2, weights="").to(DEV).train()
    model.compute_dtype = "bf16"
    opt = FusedAdam(model, lr=1e-4)
    x, y, c = make_batch(batch, 512, seed=7, with_cls=True)
    x, y, c = x.to(DEV), y.to(DEV), c.to(DEV)
    ops.PROBE = []
    try:
        opt.zero_grad()
        if multitask:
            seg, cls = model(x)
            loss = multitask_loss(seg, cls, y, c, 1.0, "bce")[0]
        else:
            loss = binary_segmentation_loss(model(x), y, "lovasz_hinge")
        loss.backward()
        opt.step()
        torch.cuda.synchronize()
        used = set()
        for rec in ops.PROBE:
            used.update(introspect.call_configs(rec[5]))
    finally:
        ops.PROBE = None
    del model, opt
    torch.cuda.empty_cache()
    assert np.isfinite(loss.item())
    used.discard(None)
    stem = {"stem_fwd:tn128x64", "stem_fwd:stem_halo", "stem_wgrad:wgrad_ring64x256"}  # test_stem_bench_size
    missing = sorted(used - covered_keys() - stem)
    assert not missing, f"{model_name} B={batch}: configurations without a parity case: {missing}"


@pytest.mark.parametrize("cid", [c for c in CASES if "halo3" in c and not c.startswith("wgrad")])
def test_halo3_case_hs(cid, monkeypatch):
    """the halo3 cases again on the half-tile pipeline (UNETSEG_HALO_HS=1, read per launch; the
    default since round 5 is the whole-tile double buffer)"""
    monkeypatch.setenv("UNETSEG_HALO_HS", "1")
    _run_case(cid, *CASES[cid])


@pytest.mark.parametrize("hs", ["0", "1"])
@pytest.mark.parametrize("direction", ["fwd_relu", "fwd_stats", "post1", "dgrad"])
def test_halo3_hs_repeat_bit_identical(direction, hs, monkeypatch):
    """the halo3 half-tile pipeline's waits are hand-counted vmcnt values (conv_halo.hip
    hs_wait); a count too high would let a tap read a half stage before its DMA landed -- a silent LDS
    race.  The same 512^2 launch, three times in one process (and at 128^2 with several tiles per
    block), must give bit-identical outputs -- on the half-tile pipeline and on the double buffer."""
    from unetseg_hip.lib import DT_BF16, lib
    monkeypatch.setenv("UNETSEG_HALO_HS", hs)
    for shape in ((4, 512, 512, 64, 0, 64, 3, 1), (5, 128, 128, 64, 0, 64, 3, 1)):
        N, H, W, C1, C2, K, R, s = shape
        op = _Op(shape, RNG + 77)
        wk, wt = op.packed()
        st = _st()
        x1, _ = op.x_parts()
        dyh = _nhwc(op.dy)
        z = _bf(torch.randn(N, H, W, C1, generator=op.gen, device=DEV))
        aux = torch.relu(z)
        outs = []
        for _ in range(3):
            if direction.startswith("fwd"):
                y = torch.empty(N, H, W, K, dtype=torch.bfloat16, device=DEV)
                stats = direction == "fwd_stats"
                tile = lib.conv2d_fwd_tile_m(DT_BF16, C1, C1, 0, 0, N, H, W, K, R, R, s, 1)
                stt = torch.empty(-(-N * H * W // tile), 2, K, dtype=torch.float32, device=DEV) if stats else None
                lib.conv2d_fwd(DT_BF16, _P(x1), C1, C1, 0, 0, 0, N, H, W, _P(wk), K, R, R, s, 1,
                               0 if stats else _P(op.bias), int(not stats), _P(y), K, _P(stt), st)
                outs.append((y,) + ((stt,) if stats else ()))
            elif direction == "dgrad":
                dx = torch.empty(N, H, W, C1, dtype=torch.bfloat16, device=DEV)
                lib.conv2d_dgrad(DT_BF16, _P(dyh), K, N, H, W, _P(wt), K, C1, R, R, s, 1, _P(dx), C1, H, W, 0, st)
                outs.append((dx,))
            else:
                args = [DT_BF16, _P(dyh), K, N, H, W, _P(wt), K, C1, R, R, s, 1]
                rows = lib.conv2d_dgrad_post(*args, 0, C1, H, W, 1, _P(aux), C1, 0, 0, 0, 0, 0, 0, st)
                assert rows > 0
                dx = torch.empty(N, H, W, C1, dtype=torch.bfloat16, device=DEV)
                part = torch.empty(rows, 2, C1, dtype=torch.float32, device=DEV)
                lib.conv2d_dgrad_post(*args, _P(dx), C1, H, W, 1, _P(aux), C1, 0, 0, 0, 0, _P(part), rows, st)
                outs.append((dx, part))
        torch.cuda.synchronize()
        for o in outs[1:]:
            for a_, b_ in zip(outs[0], o):
                assert torch.equal(a_.view(torch.int16) if a_.dtype == torch.bfloat16 else a_,
                                   b_.view(torch.int16) if b_.dtype == torch.bfloat16 else b_), (direction, shape)
