"""GPU: producer/consumer fusions of the decoder, each against its unfused kernels.

Head: the model's 1x1 head fused into the epilogue of the decoder's last 3x3 conv
(unetseg_conv2d_fwd_head; reference model/unet_resnet.py:77-79 up_conv[3..4] -> final, and the
multitask seg_head).

* the activation y it stores is bit-identical to the plain conv (unetseg_conv2d_fwd);
* its logits equal a float64 head applied to that stored bf16 y (fp32 sums in another order than the
  separate head kernel: 1e-5 of max|logit|), for 1 and 2 logits, at the bench's 512x512 rows and a
  multi-image case;
* unet_resnet50 / multitask_unet bf16 forward: logits with the fusion equal those without within the
  same bound, and the training step's gradients agree to 1 % in norm (the backward is the same
  kernels; only bf16 roundings of the loss gradient can flip).

Upsample backward + ReLU backward (unetseg_upsample2x_bwd_relu; unetUp conv2 -> ReLU -> the next
block's UpsamplingBilinear2d, model/unet_resnet.py:25-33): the stored gradient is bit-identical to
upsample2x_bwd followed by relu_bwd_bias, the bias partials sum to the same column sums (fp32
summation order: 1e-5 relative), at every decoder shape of the 512x512 bench.
"""
import math

import os

import pytest
import torch

pytestmark = pytest.mark.gpu
DEV = "cuda"


@pytest.fixture(scope="module", autouse=True)
def _need_gpu():
    if not torch.cuda.is_available():
        pytest.skip("no GPU")
    from unetseg_hip import load
    load()


def _st():
    return torch.cuda.current_stream().cuda_stream


@pytest.mark.parametrize("N,H,W,Kh", [(2, 64, 256, 2), (2, 64, 256, 1), (3, 32, 64, 2), (1, 512, 512, 2)])
def test_conv_fwd_head(N, H, W, Kh):
    from unetseg_hip.lib import DT_BF16, lib
    g = torch.Generator(device=DEV).manual_seed(N * 1000 + H + Kh)
    C = 64
    x = torch.randn(N, H, W, C, generator=g, device=DEV).to(torch.bfloat16)
    w = (torch.randn(C, C, 3, 3, generator=g, device=DEV) / math.sqrt(9 * C)).contiguous()
    b = torch.randn(C, generator=g, device=DEV) * 0.1
    hw = torch.randn(Kh, C, 1, 1, generator=g, device=DEV) / 8.0
    hb = torch.randn(Kh, generator=g, device=DEV)
    wk = torch.empty(C, 3, 3, C, dtype=torch.bfloat16, device=DEV)
    wt = torch.empty(C, 3, 3, C, dtype=torch.bfloat16, device=DEV)
    lib.pack_conv_weight(DT_BF16, w.data_ptr(), C, C, 3, 3, C, wk.data_ptr(), wt.data_ptr(), _st())
    assert lib.conv2d_fwd_head_ok(DT_BF16, C, N, H, W, C, Kh) == 1
    assert lib.conv2d_fwd_head_ok(DT_BF16, C, N, H, W, C, 3) == 0
    y_ref = torch.empty(N, H, W, C, dtype=torch.bfloat16, device=DEV)
    lib.conv2d_fwd(DT_BF16, x.data_ptr(), C, C, 0, 0, 0, N, H, W, wk.data_ptr(), C, 3, 3, 1, 1, b.data_ptr(), 1,
                   y_ref.data_ptr(), C, 0, _st())
    y = torch.full((N, H, W, C), float("nan"), dtype=torch.bfloat16, device=DEV)
    logits = torch.full((N, Kh, H, W), float("nan"), device=DEV)
    lib.conv2d_fwd_head(DT_BF16, x.data_ptr(), C, N, H, W, wk.data_ptr(), b.data_ptr(), y.data_ptr(), C, Kh,
                        hw.data_ptr(), hb.data_ptr(), logits.data_ptr(), _st())
    torch.cuda.synchronize()
    assert torch.equal(y.view(torch.int16), y_ref.view(torch.int16)), "stored activation differs from the plain conv"
    ref = torch.einsum("nhwc,kc->nkhw", y.double(), hw.view(Kh, C).double()) + hb.double().view(1, Kh, 1, 1)
    err = (logits.double() - ref).abs().max().item()
    assert err <= 1e-5 * ref.abs().max().item() + 1e-6, err


@pytest.mark.parametrize("name", ["unet_resnet50", "multitask_unet"])
def test_model_head_fusion_unchanged(name):
    from model.model_factory import build_model
    from unetseg_hip import ops
    from unetseg_hip.losses import binary_segmentation_loss
    from utils.synthetic import make_batch

    torch.manual_seed(0)
    kw = dict(num_classes=1) if name == "multitask_unet" else dict(num_classes=2)
    m = build_model(name, **kw).cuda().train()
    m.compute_dtype = "bf16"
    x, y = make_batch(2, 64, seed=7)
    x, y = x.cuda(), y.cuda()
    outs = []
    for fuse in (False, True):
        ops.FUSE_HEAD = fuse
        try:
            m.zero_grad(set_to_none=False)
            with torch.autocast("cuda", dtype=torch.bfloat16):
                out = m(x)
            seg = out[0] if isinstance(out, tuple) else out
            if seg.shape[1] == 2:
                loss = binary_segmentation_loss(seg, y, "bce")
            else:
                loss = torch.nn.functional.binary_cross_entropy_with_logits(seg[:, 0], y.float())
            loss.backward()
            torch.cuda.synchronize()
            outs.append((seg.detach().clone(), [p.grad.detach().clone() for p in m.parameters()]))
        finally:
            ops.FUSE_HEAD = True
    (s0, g0), (s1, g1) = outs
    assert (s0 - s1).abs().max().item() <= 1e-5 * s0.abs().max().item() + 1e-6
    # the backward runs the same kernels; the logits differ by fp32 summation order only, which can
    # flip a bf16 rounding of the gradient here and there: relative norm, not elementwise
    for a, b in zip(g0, g1):
        assert (a - b).norm().item() <= 1e-2 * a.norm().item() + 1e-8


# heights that are multiples of 8 run the row-streaming kernel (16 rows per block at 16 x 256^2 x 64, else 8;
# half-pixel and align_corners weights), the others the row-blocked one
@pytest.mark.parametrize("N,H,W,C,align", [(16, 256, 256, 64, 1), (16, 128, 128, 128, 1), (16, 32, 32, 512, 1),
                                           (2, 24, 40, 64, 0), (3, 5, 7, 256, 1), (4, 7, 9, 64, 1), (2, 9, 33, 128, 0),
                                           (5, 3, 2, 64, 1), (8, 64, 64, 256, 1), (3, 16, 72, 64, 0), (2, 8, 8, 512, 1)])
def test_upsample_bwd_relu(N, H, W, C, align):
    from unetseg_hip.lib import DT_BF16, lib
    g = torch.Generator(device=DEV).manual_seed(N * 7 + H + C)
    dy = torch.randn(N, 2 * H, 2 * W, C, generator=g, device=DEV).to(torch.bfloat16)
    a = torch.relu(torch.randn(N, H, W, C, generator=g, device=DEV)).to(torch.bfloat16)
    # reference: the unfused kernels (the row-blocked adjoint: read per call, UNETSEG_UP_STREAM=0)
    da = torch.empty(N, H, W, C, dtype=torch.bfloat16, device=DEV)
    os.environ["UNETSEG_UP_STREAM"] = "0"
    try:
        lib.upsample2x_bwd(DT_BF16, dy.data_ptr(), C, N, H, W, C, align, da.data_ptr(), C, 0, _st())
    finally:
        os.environ.pop("UNETSEG_UP_STREAM", None)
    M = N * H * W
    Gr = lib.reduce_tiles(DT_BF16, M, C, None, None)
    pref = torch.zeros(C, Gr, device=DEV)
    dref = torch.empty_like(da)
    lib.relu_bwd_bias(DT_BF16, da.data_ptr(), C, a.data_ptr(), C, dref.data_ptr(), C, M, C, pref.data_ptr(), Gr,
                      _st())
    rows = lib.upsample2x_bwd_tiles(DT_BF16, N, H, W, C)
    part = torch.full((rows, 2, C), float("nan"), device=DEV)
    dx = torch.full((N, H, W, C), float("nan"), dtype=torch.bfloat16, device=DEV)
    lib.upsample2x_bwd_relu(DT_BF16, dy.data_ptr(), C, N, H, W, C, align, a.data_ptr(), C, dx.data_ptr(), C,
                            part.data_ptr(), rows, _st())
    torch.cuda.synchronize()
    assert torch.equal(dx.view(torch.int16), dref.view(torch.int16)), "masked gradient differs"
    got = part[:, 0, :].double().sum(0)
    ref = pref.double().sum(1)
    assert (got - ref).abs().max().item() <= 1e-5 * ref.abs().max().item() + 1e-5
    assert torch.allclose(got, dx.double().sum((0, 1, 2)), rtol=1e-5, atol=1e-4)


@pytest.mark.parametrize("N,H,W,C,align", [(8, 256, 256, 64, 0), (8, 32, 32, 512, 0), (16, 128, 128, 128, 1),
                                           (2, 24, 40, 64, 0), (3, 16, 72, 64, 1), (4, 7, 9, 64, 0)])
def test_upsample_bwd_stream(N, H, W, C, align):
    """the plain upsample adjoint (unetseg_upsample2x_bwd: the attention U-Net decoder's Upsample,
    model/unet_attention.py) on the row-streaming kernel, bit-identical to the row-blocked one, stored and
    accumulated (heights that are not a multiple of 8 take the row-blocked kernel in both runs)"""
    from unetseg_hip.lib import DT_BF16, lib
    g = torch.Generator(device=DEV).manual_seed(N * 11 + H + C)
    dy = torch.randn(N, 2 * H, 2 * W, C, generator=g, device=DEV).to(torch.bfloat16)
    base = torch.randn(N, H, W, C, generator=g, device=DEV).to(torch.bfloat16)
    outs = []
    for stream in ("0", "1"):
        os.environ["UNETSEG_UP_STREAM"] = stream
        try:
            o = []
            for acc in (0, 1):
                dx = base.clone() if acc else torch.full_like(base, float("nan"))
                lib.upsample2x_bwd(DT_BF16, dy.data_ptr(), C, N, H, W, C, align, dx.data_ptr(), C, acc, _st())
                o.append(dx)
            torch.cuda.synchronize()
        finally:
            os.environ.pop("UNETSEG_UP_STREAM", None)
        outs.append(o)
    for a, b in zip(*outs):
        assert torch.equal(a.view(torch.int16), b.view(torch.int16))


@pytest.mark.parametrize("M,C,mode", [(16 * 128 * 128, 256, 1), (16 * 32 * 32, 1024, 2), (3 * 15 * 17, 64, 1)])
def test_bn_mask_bits(M, C, mode):
    """unetseg_bn_apply_mask (the residual BN-add-ReLU of the bottleneck, model/resnet_backbone.py:66-76):
    the activation is bit-identical to unetseg_bn_apply, the packed bits are (out > 0), and the BN backward
    reading the bits (lda = 0) is bit-identical to reading the activation"""
    from unetseg_hip.lib import DT_BF16, lib
    g = torch.Generator(device=DEV).manual_seed(M + C)
    bf = torch.bfloat16
    y = torch.randn(M, C, generator=g, device=DEV).to(bf)
    r = torch.randn(M, C, generator=g, device=DEV).to(bf)
    sc, sh = torch.rand(C, generator=g, device=DEV) + 0.5, torch.randn(C, generator=g, device=DEV) * 0.2
    sc2, sh2 = torch.rand(C, generator=g, device=DEV) + 0.5, torch.randn(C, generator=g, device=DEV) * 0.2
    m2 = (sc2.data_ptr(), sh2.data_ptr()) if mode == 2 else (0, 0)
    a_ref = torch.empty(M, C, dtype=bf, device=DEV)
    lib.bn_apply(DT_BF16, y.data_ptr(), C, sc.data_ptr(), sh.data_ptr(), r.data_ptr(), C, *m2, mode, 1,
                 a_ref.data_ptr(), C, M, C, _st())
    a = torch.empty_like(a_ref)
    bits = torch.empty(M * C // 8, dtype=torch.uint8, device=DEV)
    lib.bn_apply_mask(DT_BF16, y.data_ptr(), C, sc.data_ptr(), sh.data_ptr(), r.data_ptr(), C, *m2, mode,
                      a.data_ptr(), C, M, C, bits.data_ptr(), _st())
    torch.cuda.synchronize()
    assert torch.equal(a.view(torch.int16), a_ref.view(torch.int16))
    want = (a.float() > 0).view(M, C // 8, 8).to(torch.int32)
    want = (want << torch.arange(8, device=DEV, dtype=torch.int32)).sum(-1).to(torch.uint8).view(-1)
    assert torch.equal(bits, want)
    # backward through the same BN with the mask from the activation vs from the bits
    dA = torch.randn(M, C, generator=g, device=DEV).to(bf)
    mean, inv = torch.randn(C, generator=g, device=DEV) * 0.1, torch.rand(C, generator=g, device=DEV) + 0.5
    Gr = lib.reduce_tiles(DT_BF16, M, C, None, None)
    outs = []
    for src, lda in ((a, C), (bits, 0)):
        part = torch.empty(3, C, Gr, device=DEV)
        y2 = (r.data_ptr(), C, mean.data_ptr(), inv.data_ptr()) if mode == 2 else (0, 0, 0, 0)
        lib.bn_bwd_reduce(DT_BF16, dA.data_ptr(), C, src.data_ptr(), lda, 0, 0, y.data_ptr(), C, mean.data_ptr(),
                          inv.data_ptr(), *y2, M, C, part.data_ptr(), Gr, _st())
        coef = torch.randn(6, C, generator=torch.Generator(device=DEV).manual_seed(1), device=DEV)
        dy1 = torch.empty(M, C, dtype=bf, device=DEV)
        dy2 = torch.empty(M, C, dtype=bf, device=DEV)
        dz = torch.empty(M, C, dtype=bf, device=DEV)
        yb = (r.data_ptr(), C, mean.data_ptr(), inv.data_ptr(), dy2.data_ptr(), C) if mode == 2 else (0, 0, 0, 0, 0, 0)
        lib.bn_bwd_apply(DT_BF16, dA.data_ptr(), C, src.data_ptr(), lda, 0, 0, y.data_ptr(), C, mean.data_ptr(),
                         inv.data_ptr(), dy1.data_ptr(), C, *yb, coef.data_ptr(), dz.data_ptr(), C, 0, M, C, _st())
        torch.cuda.synchronize()
        outs.append((part.clone(), dy1.clone(), dy2.clone() if mode == 2 else None, dz.clone()))
    (p0, d0, e0, z0), (p1, d1, e1, z1) = outs
    nq = 3 if mode == 2 else 2
    assert torch.equal(p0[:nq], p1[:nq])
    assert torch.equal(d0.view(torch.int16), d1.view(torch.int16))
    assert torch.equal(z0.view(torch.int16), z1.view(torch.int16))
    if mode == 2:
        assert torch.equal(e0.view(torch.int16), e1.view(torch.int16))


@pytest.mark.parametrize("M,C,lda0", [(16 * 256 * 256, 64, 1), (16 * 64 * 64, 512, 0), (3 * 15 * 17, 64, 0),
                                      (4096, 2048, 1), (5 * 7 * 9, 256, 1)])
def test_bn_bwd_block_counts(M, C, lda0, monkeypatch):
    """BN backward under other block counts (the reduction's ~1024 and the apply pass's own ~4096,
    elem.hip unetseg_reduce_tiles / apply_tiles): the apply pass is bit-identical whatever its
    geometry; the reduction's per-channel totals (model/train.py's BatchNorm2d backward: sum dz,
    sum dz * xhat) match a float64 reference under every block count"""
    from unetseg_hip.lib import DT_BF16, lib
    g = torch.Generator(device=DEV).manual_seed(M + C + lda0)
    bf = torch.bfloat16
    y = torch.randn(M, C, generator=g, device=DEV).to(bf)
    a = torch.relu(torch.randn(M, C, generator=g, device=DEV)).to(bf)
    dA = torch.randn(M, C, generator=g, device=DEV).to(bf)
    mean, inv = torch.randn(C, generator=g, device=DEV) * 0.1, torch.rand(C, generator=g, device=DEV) + 0.5
    if lda0:  # the packed ReLU mask (lda = 0) instead of the activation
        w = (a.float() > 0).view(M, C // 8, 8).to(torch.int32)
        src = (w << torch.arange(8, device=DEV, dtype=torch.int32)).sum(-1).to(torch.uint8).view(-1)
        lda = 0
    else:
        src, lda = a, C
    coef = torch.randn(3, C, generator=g, device=DEV)
    dz = torch.where(a.double() > 0, dA.double(), torch.zeros((), dtype=torch.float64, device=DEV))
    xhat = (y.double() - mean.double()) * inv.double()
    want = torch.stack([dz.sum(0), (dz * xhat).sum(0)])
    scale = torch.stack([dz.abs().sum(0), (dz * xhat).abs().sum(0)])
    applies = []
    for red, app in ((None, None), ("512", "64"), ("4096", "100000"), ("64", "1")):
        for k, v in (("UNETSEG_RED_TARGET", red), ("UNETSEG_APPLY_TARGET", app)):
            if v is None:
                monkeypatch.delenv(k, raising=False)
            else:
                monkeypatch.setenv(k, v)
        Gr = lib.reduce_tiles(DT_BF16, M, C, None, None)
        part = torch.full((2, C, Gr), float("nan"), device=DEV)
        lib.bn_bwd_reduce(DT_BF16, dA.data_ptr(), C, src.data_ptr(), lda, 0, 0, y.data_ptr(), C, mean.data_ptr(),
                          inv.data_ptr(), 0, 0, 0, 0, M, C, part.data_ptr(), Gr, _st())
        dy1 = torch.full((M, C), float("nan"), dtype=bf, device=DEV)
        dzo = torch.full((M, C), float("nan"), dtype=bf, device=DEV)
        lib.bn_bwd_apply(DT_BF16, dA.data_ptr(), C, src.data_ptr(), lda, 0, 0, y.data_ptr(), C, mean.data_ptr(),
                         inv.data_ptr(), dy1.data_ptr(), C, 0, 0, 0, 0, 0, 0, coef.data_ptr(), dzo.data_ptr(), C, 0,
                         M, C, _st())
        torch.cuda.synchronize()
        got = part.double().sum(2)
        assert ((got - want).abs() <= 1e-5 * scale + 1e-6).all(), (red, (got - want).abs().max().item())
        applies.append((dy1.view(torch.int16).clone(), dzo.view(torch.int16).clone()))
    for d, z in applies[1:]:
        assert torch.equal(d, applies[0][0]) and torch.equal(z, applies[0][1])
    assert torch.equal(applies[0][1], dz.to(bf).view(torch.int16))
