"""GPU: every HIP kernel against a plain-PyTorch fp32 CPU reference of the same op.

fp32 mode is expected to match to ~1e-5 relative (exact-f32 MFMA, different summation order);
bf16 mode rounds operands/outputs to bf16, compared at 2e-2 of the output scale.
"""
import math

import numpy as np
import pytest
import torch
import torch.nn.functional as F

pytestmark = pytest.mark.gpu

DEV = "cuda"


@pytest.fixture(scope="module", autouse=True)
def _need_gpu():
    if not torch.cuda.is_available():
        pytest.skip("no GPU")
    from unetseg_hip import load
    load()


def _ops():
    from unetseg_hip import ops
    from unetseg_hip.lib import DT_BF16, DT_F32
    return ops, DT_BF16, DT_F32


def _ctx(dt, training=True, record=True):
    ops, _, _ = _ops()
    return ops.Ctx(dt, training, record, torch.device(DEV))


def _node(x_nchw, dt, need_grad=True):
    """NCHW fp32 CPU -> NHWC device Node"""
    ops, DT_BF16, _ = _ops()
    t = x_nchw.permute(0, 2, 3, 1).contiguous().to(DEV)
    t = t.to(torch.bfloat16 if dt == DT_BF16 else torch.float32)
    return ops.Node(t, need_grad)


def _nchw(t):
    return t.float().permute(0, 3, 1, 2).cpu()


def _rel(a, b):
    a, b = a.double(), b.double()
    return float((a - b).abs().max() / (b.abs().max() + 1e-12))


def _round(t, dt):
    _, DT_BF16, _ = _ops()
    return t.to(torch.bfloat16).float() if dt == DT_BF16 else t


CONV_CASES = [
    # N, H, W, C1, C2, K, k, stride, pad, bias, relu
    (2, 17, 19, 64, 0, 96, 3, 1, 1, True, True),
    (2, 16, 16, 128, 0, 64, 1, 2, 0, False, False),
    (2, 33, 31, 3, 0, 64, 7, 2, 3, False, False),
    (1, 9, 12, 64, 128, 64, 3, 1, 1, True, True),
    (2, 15, 15, 256, 0, 256, 3, 2, 1, False, False),
    (2, 8, 8, 512, 0, 2048, 1, 1, 0, False, False),
    # fast-path shapes (bf16: channels % 64, Q % 32 for wgrad)
    (2, 32, 32, 64, 0, 64, 3, 1, 1, True, True),
    (1, 32, 64, 128, 64, 128, 3, 1, 1, True, True),
    (2, 64, 64, 128, 0, 128, 3, 2, 1, False, False),
    (2, 64, 64, 256, 0, 512, 1, 2, 0, False, False),
    (1, 96, 32, 64, 128, 64, 3, 1, 1, True, True),
    (3, 33, 64, 192, 0, 32, 1, 1, 0, False, False),
    # narrow 1x1 output (K % 64 != 0): gradients through dY zero-padded to 64 channels
    (2, 21, 23, 128, 0, 40, 1, 1, 0, False, False),
    # 3x3 halo kernel (64 input channels, H % 8 == 0, W % 32 == 0): fwd 64->192, dgrad 192<-64
    (2, 16, 64, 64, 0, 192, 3, 1, 1, True, True),
    (1, 24, 32, 192, 0, 64, 3, 1, 1, False, False),
    # one K step (64 input channels, 1x1): single-stage 128x128 TN configuration
    (2, 16, 24, 64, 0, 256, 1, 1, 0, False, False),
    # small M, long K: 64-row tiles
    (1, 8, 8, 320, 0, 256, 3, 1, 1, True, True),
]


@pytest.mark.parametrize("case", CONV_CASES)
@pytest.mark.parametrize("dtname", ["fp32", "bf16"])
def test_conv_fwd_dgrad_wgrad(case, dtname):
    ops, DT_BF16, DT_F32 = _ops()
    dt = DT_BF16 if dtname == "bf16" else DT_F32
    from unetseg_hip.nn import Conv2d
    N, H, W, C1, C2, K, k, s, p, bias, relu = case
    g = torch.Generator().manual_seed(hash(case) & 0xFFFF)
    cin = C1 + C2
    conv = Conv2d(cin, K, k, stride=s, padding=p, bias=bias)
    with torch.no_grad():
        conv.weight.copy_(torch.randn(conv.weight.shape, generator=g) / math.sqrt(cin * k * k))
        if bias:
            conv.bias.copy_(torch.randn(K, generator=g) * 0.1)
    conv = conv.to(DEV)
    conv.weight.grad = torch.zeros_like(conv.weight)
    if bias:
        conv.bias.grad = torch.zeros_like(conv.bias)
    cpad = 8 if cin < 8 else None
    pc = ops.PackedConv(conv, cpad)
    ctx = _ctx(dt)
    pc.pack(ctx, need_t=True)
    x1 = torch.randn(N, C1, H, W, generator=g)
    x2 = torch.randn(N, C2, H, W, generator=g) if C2 else None
    if cin < 8:
        x1p = torch.cat([x1, torch.zeros(N, 8 - cin, H, W)], 1)
        n1 = _node(x1p, dt)
    else:
        n1 = _node(x1, dt)
    n2 = _node(x2, dt) if C2 else None
    y, _ = ops.conv(ctx, n1, pc, x2=n2, relu=relu)
    # reference on the (rounded) operands
    xr = _round(torch.cat([x1, x2], 1) if C2 else x1, dt).requires_grad_(True)
    wr = _round(conv.weight.detach().cpu(), dt).requires_grad_(True)
    br = conv.bias.detach().cpu().requires_grad_(True) if bias else None
    ref = F.conv2d(xr, wr, br, s, p)
    if relu:
        ref = F.relu(ref)
    out = _nchw(y.data)
    tol = 2e-2 if dt == DT_BF16 else 2e-5
    assert _rel(out, ref.detach()) < tol
    # backward
    dy = torch.randn(ref.shape, generator=g)
    dy_r = _round(dy, dt)
    y.grad = _node(dy_r, dt).data
    if cin < 8:
        n1.need_grad = False
    ctx.backward()
    ref.backward(dy_r)
    tolg = 3e-2 if dt == DT_BF16 else 1e-4
    if relu:  # mask from the device output; compare with the device's own mask
        pass
    wgrad = conv.weight.grad.cpu()
    assert _rel(wgrad, wr.grad) < tolg, _rel(wgrad, wr.grad)
    if bias:
        assert _rel(conv.bias.grad.cpu(), br.grad) < tolg
    if cin >= 8:
        dx = _nchw(n1.grad)
        if C2:
            dx = torch.cat([dx, _nchw(n2.grad)], 1)
        assert _rel(dx, xr.grad) < tolg, _rel(dx, xr.grad)


@pytest.mark.parametrize("N,H,W", [(2, 64, 64), (1, 37, 50), (3, 32, 96)])
def test_stem_conv_fast(N, H, W):
    """ResNet stem (7x7/s2/p3, 3->64) on the width-packed fast path (ops.stem_conv) against
    F.conv2d on the bf16-rounded operands: output, BN partial stats (column sums) and wgrad."""
    ops, DT_BF16, _ = _ops()
    from unetseg_hip.nn import Conv2d
    g = torch.Generator().manual_seed(N * 1000 + H * 10 + W)
    conv = Conv2d(3, 64, 7, stride=2, padding=3, bias=False)
    with torch.no_grad():
        conv.weight.copy_(torch.randn(conv.weight.shape, generator=g) / math.sqrt(147))
    conv = conv.to(DEV)
    conv.weight.grad = torch.zeros_like(conv.weight)
    x = torch.rand(N, 3, H, W, generator=g)
    ctx = _ctx(DT_BF16)
    y, (st, tile) = ops.stem_conv(ctx, x.to(DEV), conv)
    xr = _round(x, DT_BF16)
    wr = _round(conv.weight.detach().cpu(), DT_BF16).requires_grad_(True)
    ref = F.conv2d(xr, wr, None, 2, 3)
    out = _nchw(y.data)
    assert out.shape == ref.shape
    assert _rel(out, ref.detach()) < 2e-2
    # partial stats: column sums over all row tiles == per-channel sum of the stored outputs
    colsum = st[:, 0, :].sum(0).cpu().double()
    assert torch.allclose(colsum, out.double().sum((0, 2, 3)), rtol=1e-3, atol=1e-2)
    dy = _round(torch.randn(ref.shape, generator=g), DT_BF16)
    y.grad = _node(dy, DT_BF16).data
    ctx.backward()
    torch.cuda.synchronize()
    ref.backward(dy)
    assert _rel(conv.weight.grad.cpu(), wr.grad) < 3e-2, _rel(conv.weight.grad.cpu(), wr.grad)


@pytest.mark.parametrize("dtname", ["fp32", "bf16"])
@pytest.mark.parametrize("mode", ["plain", "res", "res_bn"])
def test_bn_train_fwd_bwd(dtname, mode):
    ops, DT_BF16, DT_F32 = _ops()
    dt = DT_BF16 if dtname == "bf16" else DT_F32
    from unetseg_hip.nn import BatchNorm2d, Conv2d
    g = torch.Generator().manual_seed(5)
    N, C, H, W = 3, 64, 11, 13
    conv = Conv2d(32, C, 1, bias=False)
    conv2 = Conv2d(32, C, 1, bias=False)
    with torch.no_grad():
        conv.weight.copy_(torch.randn(conv.weight.shape, generator=g) * 0.3)
        conv2.weight.copy_(torch.randn(conv2.weight.shape, generator=g) * 0.3)
    bnm, bnm2 = BatchNorm2d(C), BatchNorm2d(C)
    with torch.no_grad():
        for b in (bnm, bnm2):
            b.weight.copy_(1 + 0.2 * torch.randn(C, generator=g))
            b.bias.copy_(0.2 * torch.randn(C, generator=g))
    mods = [conv.to(DEV), conv2.to(DEV), bnm.to(DEV), bnm2.to(DEV)]
    for m in mods:
        for prm in m.parameters():
            prm.grad = torch.zeros_like(prm)
    ctx = _ctx(dt)
    pc, pc2 = ops.PackedConv(conv), ops.PackedConv(conv2)
    pc.pack(ctx, True)
    pc2.pack(ctx, True)
    x = torch.randn(N, 32, H, W, generator=g) + 0.5
    xn = _node(x, dt)
    y, st = ops.conv(ctx, xn, pc, stats=True)
    r = torch.randn(N, C, H, W, generator=g)
    rn = _node(r, dt)
    if mode == "plain":
        a = ops.bn(ctx, y, st, bnm, relu=True)
    elif mode == "res":
        a = ops.bn(ctx, y, st, bnm, relu=True, res=rn)
    else:
        y2, st2 = ops.conv(ctx, xn, pc2, stats=True)
        a = ops.bn(ctx, y2 if False else y, st, bnm, relu=True, res_bn=(y2, st2, bnm2))
    # reference: BN on the device's own conv outputs (isolates the BN kernels)
    yr = _nchw(y.data).requires_grad_(True)
    rb = torch.nn.BatchNorm2d(C).train()
    with torch.no_grad():
        rb.weight.copy_(bnm.weight.cpu())
        rb.bias.copy_(bnm.bias.cpu())
    ref = rb(yr)
    if mode == "res":
        rr = _round(r, dt).requires_grad_(True)
        ref = ref + rr
    if mode == "res_bn":
        y2r = _nchw(y2.data).requires_grad_(True)
        rb2 = torch.nn.BatchNorm2d(C).train()
        with torch.no_grad():
            rb2.weight.copy_(bnm2.weight.cpu())
            rb2.bias.copy_(bnm2.bias.cpu())
        ref = ref + rb2(y2r)
    ref = F.relu(ref)
    tol = 2e-2 if dt == DT_BF16 else 1e-5
    assert _rel(_nchw(a.data), ref.detach()) < tol
    torch.testing.assert_close(bnm.running_mean.cpu(), rb.running_mean, rtol=1e-4, atol=1e-5)
    torch.testing.assert_close(bnm.running_var.cpu(), rb.running_var, rtol=1e-4, atol=1e-5)
    assert int(bnm.num_batches_tracked) == 1
    dA = _round(torch.randn(ref.shape, generator=g), dt)
    a.grad = _node(dA, dt).data
    # stop at the BN input (conv grads are tested separately)
    ctx.tape = ctx.tape[-1:]
    ctx.backward()
    ref.backward(dA)
    tolg = 3e-2 if dt == DT_BF16 else 1e-4
    assert _rel(_nchw(y.grad), yr.grad) < tolg
    assert _rel(bnm.weight.grad.cpu(), rb.weight.grad) < tolg
    assert _rel(bnm.bias.grad.cpu(), rb.bias.grad) < tolg
    if mode == "res":
        assert _rel(_nchw(rn.grad), rr.grad) < tolg
    if mode == "res_bn":
        assert _rel(_nchw(y2.grad), y2r.grad) < tolg
        assert _rel(bnm2.weight.grad.cpu(), rb2.weight.grad) < tolg


@pytest.mark.parametrize("dtname", ["fp32", "bf16"])
@pytest.mark.parametrize("k,s,ceil,H", [(3, 2, True, 256 // 8), (3, 2, True, 31), (2, 2, False, 16), (2, 2, False, 9)])
def test_maxpool(dtname, k, s, ceil, H):
    ops, DT_BF16, DT_F32 = _ops()
    dt = DT_BF16 if dtname == "bf16" else DT_F32
    g = torch.Generator().manual_seed(9)
    x = _round(torch.randn(2, 16, H, H + 1, generator=g), dt)
    x[0, 0, :3, :3] = 0.5  # ties
    ctx = _ctx(dt)
    xn = _node(x, dt)
    y = ops.maxpool(ctx, xn, k, s, ceil)
    xr = x.clone().requires_grad_(True)
    ref = F.max_pool2d(xr, k, s, 0, ceil_mode=ceil)
    assert tuple(_nchw(y.data).shape) == tuple(ref.shape)
    torch.testing.assert_close(_nchw(y.data), ref.detach(), rtol=0, atol=0)
    dy = _round(torch.randn(ref.shape, generator=g), dt)
    y.grad = _node(dy, dt).data
    ctx.backward()
    ref.backward(dy)
    tol = 1e-2 if dt == DT_BF16 else 1e-6
    assert _rel(_nchw(xn.grad), xr.grad) < tol


@pytest.mark.parametrize("dtname", ["fp32", "bf16"])
@pytest.mark.parametrize("align", [True, False])
@pytest.mark.parametrize("H,W", [(8, 8), (5, 7), (16, 16), (1, 3)])
def test_upsample(dtname, align, H, W):
    ops, DT_BF16, DT_F32 = _ops()
    dt = DT_BF16 if dtname == "bf16" else DT_F32
    g = torch.Generator().manual_seed(11)
    x = _round(torch.randn(2, 24, H, W, generator=g), dt)
    ctx = _ctx(dt)
    xn = _node(x, dt)
    y = ops.upsample2x(ctx, xn, align)
    xr = x.clone().requires_grad_(True)
    ref = F.interpolate(xr, scale_factor=2, mode="bilinear", align_corners=align)
    tol = 1e-2 if dt == DT_BF16 else 1e-6
    assert _rel(_nchw(y.data), ref.detach()) < tol
    dy = _round(torch.randn(ref.shape, generator=g), dt)
    y.grad = _node(dy, dt).data
    ctx.backward()
    ref.backward(dy)
    assert _rel(_nchw(xn.grad), xr.grad) < tol


@pytest.mark.parametrize("dtname", ["fp32", "bf16"])
@pytest.mark.parametrize("align", [True, False])
@pytest.mark.parametrize("N,H,W", [(1, 5, 7), (1, 3, 3), (3, 7, 2)])
def test_upsample_fwd_partial_rows(dtname, align, N, H, W):
    """output row counts N * 2H that leave a partial last row block of upsample_fwd_kernel (2 of its 4
    rows; the model tests' N = 2 never do)"""
    ops, DT_BF16, DT_F32 = _ops()
    dt = DT_BF16 if dtname == "bf16" else DT_F32
    g = torch.Generator().manual_seed(13 + H)
    x = _round(torch.randn(N, 16, H, W, generator=g), dt)
    y = ops.upsample2x(_ctx(dt), _node(x, dt), align)
    ref = F.interpolate(x, scale_factor=2, mode="bilinear", align_corners=align)
    assert _rel(_nchw(y.data), ref) < (1e-2 if dt == DT_BF16 else 1e-6)


@pytest.mark.parametrize("dtname", ["fp32", "bf16"])
@pytest.mark.parametrize("align", [True, False])
@pytest.mark.parametrize("H,C", [(4, 1024), (16, 256), (32, 64)])
def test_upsample_strided_grad(dtname, align, H, C):
    """model-shaped upsample whose gradient arrives as a channel slice of a concat gradient
    (ld > C), accumulated onto an existing gradient"""
    ops, DT_BF16, DT_F32 = _ops()
    dt = DT_BF16 if dtname == "bf16" else DT_F32
    g = torch.Generator().manual_seed(5)
    x = _round(torch.randn(2, C, H, H, generator=g), dt)
    ctx = _ctx(dt)
    xn = _node(x, dt)
    y = ops.upsample2x(ctx, xn, align)
    xr = x.clone().requires_grad_(True)
    ref = F.interpolate(xr, scale_factor=2, mode="bilinear", align_corners=align)
    tol = 1e-2 if dt == DT_BF16 else 1e-6
    assert _rel(_nchw(y.data), ref.detach()) < tol
    dy = _round(torch.randn(2, C + 32, 2 * H, 2 * H, generator=g), dt)
    full = _node(dy, dt).data
    y.grad = full[..., 32:]
    g0 = _round(torch.randn(x.shape, generator=g), dt)
    xn.grad = _node(g0, dt).data.clone()
    ctx.backward()
    ref.backward(dy[:, 32:])
    assert _rel(_nchw(xn.grad), xr.grad + g0) < tol


@pytest.mark.parametrize("dtname", ["fp32", "bf16"])
@pytest.mark.parametrize("K", [1, 2])
@pytest.mark.parametrize("N,H,W", [(2, 37, 50), (1, 64, 64), (3, 5, 7)])
def test_pw_head(dtname, K, N, H, W):
    """1x1 head conv (64 -> K, bias) to fp32 NCHW logits, forward and backward"""
    ops, DT_BF16, DT_F32 = _ops()
    from unetseg_hip.nn import Conv2d
    dt = DT_BF16 if dtname == "bf16" else DT_F32
    g = torch.Generator().manual_seed(13)
    conv = Conv2d(64, K, 1).to(DEV)
    conv.weight.grad = torch.zeros_like(conv.weight)
    conv.bias.grad = torch.zeros_like(conv.bias)
    x = _round(torch.randn(N, 64, H, W, generator=g), dt)
    ctx = _ctx(dt)
    xn = _node(x, dt)
    y, holder = ops.pw_head(ctx, xn, conv)
    xr = x.clone().requires_grad_(True)
    wr = conv.weight.detach().cpu().clone().requires_grad_(True)
    br = conv.bias.detach().cpu().clone().requires_grad_(True)
    ref = F.conv2d(xr, wr, br)
    tol = 2e-2 if dt == DT_BF16 else 1e-5
    assert _rel(y.cpu(), ref.detach()) < tol
    dy = torch.randn(ref.shape, generator=g)
    holder["grad"] = dy.to(DEV)
    ctx.backward()
    ref.backward(dy)
    assert _rel(_nchw(xn.grad), xr.grad) < tol
    assert _rel(conv.weight.grad.cpu(), wr.grad) < 1e-4
    assert _rel(conv.bias.grad.cpu(), br.grad) < 1e-4


@pytest.mark.parametrize("B,H,W", [(3, 40, 48), (2, 64, 64), (1, 7, 5)])
def test_lovasz_matches_oracle(B, H, W):
    from oracle import ref_cpu
    from unetseg_hip import losses
    g = torch.Generator().manual_seed(B * 100 + H)
    out = torch.randn(B, 2, H, W, generator=g) * 2
    tgt = (torch.rand(B, H, W, generator=g) < 0.35).long()
    o = out.clone().requires_grad_(True)
    ref = ref_cpu.binary_segmentation_loss(o, tgt, "lovasz_hinge")
    ref.backward()
    od = out.to(DEV).requires_grad_(True)
    loss = losses.binary_segmentation_loss(od, tgt.to(DEV), "lovasz_hinge")
    loss.backward()
    assert abs(loss.item() - ref.item()) < 1e-5 * max(1, abs(ref.item()))
    assert _rel(od.grad.cpu(), o.grad) < 1e-5


def test_lovasz_golden(golden_dir):
    """against the reference's own Lovasz values (tests/golden/losses.npz), incl. heavy ties"""
    import os
    from unetseg_hip import losses
    d = np.load(os.path.join(golden_dir, "losses.npz"))
    lg = torch.from_numpy(d["logits"])
    lab = torch.from_numpy(d["labels"]).long()
    two = torch.stack([torch.zeros_like(lg), lg], 1).to(DEV).requires_grad_(True)
    loss = losses.binary_segmentation_loss(two, lab.to(DEV), "lovasz_hinge")
    loss.backward()
    np.testing.assert_allclose(loss.item(), d["lovasz"][0], rtol=1e-5)
    np.testing.assert_allclose(two.grad[:, 1].cpu().numpy(), d["lovasz_grad"], rtol=1e-4, atol=1e-8)
    tied = torch.from_numpy(d["tied"])
    two_t = torch.stack([torch.zeros_like(tied), tied], 1).to(DEV)
    lt = losses.binary_segmentation_loss(two_t, lab.to(DEV), "lovasz_hinge")
    np.testing.assert_allclose(lt.item(), d["lovasz_tied"][0], rtol=1e-5)


def test_bce_golden(golden_dir):
    import os
    from unetseg_hip import losses
    d = np.load(os.path.join(golden_dir, "losses.npz"))
    two = torch.from_numpy(d["two"]).to(DEV).requires_grad_(True)
    b = losses.binary_segmentation_loss(two, torch.from_numpy(d["tgt"]).to(DEV), "bce",
                                        pos_weight=torch.tensor([1.7], device=DEV))
    b.backward()
    np.testing.assert_allclose(b.item(), d["bce_pw"][0], rtol=1e-5)
    np.testing.assert_allclose(two.grad.cpu().numpy(), d["bce_grad"], rtol=1e-4, atol=1e-9)


def test_confusion_golden(golden_dir):
    import os
    from unetseg_hip import losses
    d = np.load(os.path.join(golden_dir, "metrics.npz"))
    conf = losses.binary_confusion(torch.from_numpy(d["outs"]).to(DEV), torch.from_numpy(d["tg"]).to(DEV))
    assert conf.cpu().tolist() == d["conf"].tolist()


def test_adam_matches_torch():
    from unetseg_hip.lib import lib
    g = torch.Generator().manual_seed(1)
    n = 10007
    p = torch.randn(n, generator=g)
    pt = p.clone().requires_grad_(True)
    opt = torch.optim.Adam([pt], lr=1e-3, betas=(0.9, 0.999), weight_decay=1e-4)
    pd, m, v = p.to(DEV), torch.zeros(n, device=DEV), torch.zeros(n, device=DEV)
    for step in range(1, 4):
        gr = torch.randn(n, generator=g)
        pt.grad = gr.clone()
        opt.step()
        gd = gr.to(DEV)
        lib.adam(pd.data_ptr(), gd.data_ptr(), m.data_ptr(), v.data_ptr(), n, 1e-3, 0.9, 0.999, 1e-8, 1e-4, step, 0,
                 torch.cuda.current_stream().cuda_stream)
    torch.testing.assert_close(pd.cpu(), pt.detach(), rtol=1e-6, atol=1e-7)


@pytest.mark.parametrize("dtname", ["fp32", "bf16"])
def test_pack_conv_weights_batched(dtname):
    """unetseg_pack_conv_weights (one launch for every conv) == torch permutes of the fp32 weights:
    wk [K][R][S][Cpad] (zero channels C..Cpad-1) and wt [C][R][S][K] (bf16 narrow 1x1 convs: rows padded
    to 64 with zero columns, the padded-K dgrad's operand); ragged K/C tiles, tap chunks of a 7x7, K not a
    multiple of 8 (scalar store path), bit-exact conversion."""
    ops, DT_BF16, DT_F32 = _ops()
    dt = DT_BF16 if dtname == "bf16" else DT_F32
    tdt = torch.bfloat16 if dtname == "bf16" else torch.float32
    g = torch.Generator().manual_seed(7)
    shapes = [(64, 64, 3, 3, None, True), (64, 3, 7, 7, 8, False), (40, 24, 3, 3, None, True),
              (512, 2048, 1, 1, None, True), (36, 20, 3, 3, None, True), (96, 136, 1, 1, None, True),
              (128, 192, 3, 3, None, True), (32, 64, 1, 1, None, True)]
    convs, pcs, need_t = [], [], []
    for K, C, R, S, cpad, nt in shapes:
        conv = torch.nn.Conv2d(C, K, (R, S), bias=False)
        conv.weight.data = torch.randn(K, C, R, S, generator=g).to(DEV)
        convs.append(conv)
        pcs.append(ops.PackedConv(conv, cpad))
        need_t.append(nt)
    ctx = _ctx(dt)
    table = ops.PackTable()
    table.run(ctx, pcs, need_t)
    torch.cuda.synchronize()
    for (K, C, R, S, cpad, nt), conv, pc in zip(shapes, convs, pcs):
        w = conv.weight.data.cpu()
        cp = cpad or C
        ref_k = torch.zeros(K, R, S, cp)
        ref_k[..., :C] = w.permute(0, 2, 3, 1)
        assert torch.equal(pc.wk.cpu(), ref_k.to(tdt)), (K, C, R, S)
        if nt:
            # narrow 1x1 convs in bf16 (PAD_K): wt rows are 64-padded, the pad columns zero (PackedConv.kld)
            wt = pc.wt.cpu()
            assert wt.shape[-1] == pc.kld and (pc.kld == K or (dtname == "bf16" and R == S == 1 and pc.kld % 64 == 0))
            assert torch.equal(wt[..., :K], w.permute(1, 2, 3, 0).contiguous().to(tdt)), (K, C, R, S)
            assert not wt[..., K:].any(), (K, C, R, S)




@pytest.mark.parametrize("dtname", ["fp32", "bf16"])
@pytest.mark.parametrize("N,H,Cs,Cg,Ci", [(2, 16, 64, 128, 32), (1, 24, 128, 256, 64), (2, 8, 512, 1024, 256)])
def test_attention_gate_op(dtname, N, H, Cs, Cg, Ci):
    """AttentionGate (model/unet_attention.py:7-35 of the reference) as one op: theta/phi 1x1 convs
    + BN, ReLU of the sum, psi 1x1 conv + BN + sigmoid, skip * alpha -- forward, input gradients and
    every parameter gradient against torch fp32 functional code in training mode.  inter = 32 takes
    the zero-padded narrow-gradient path in bf16."""
    from model.unet_attention import AttentionGate
    ops, DT_BF16, DT_F32 = _ops()
    dt = DT_BF16 if dtname == "bf16" else DT_F32
    g = torch.Generator().manual_seed(13)
    gm = AttentionGate(Cg, Cs, Ci)
    for p in gm.parameters():
        p.data = torch.randn(p.shape, generator=g) * (0.3 if p.dim() > 1 else 0.2)
    for bnm in (gm.theta[1], gm.phi[1], gm.psi[1]):
        bnm.weight.data += 1.0
    ref_params = {n: _round(p.data.clone(), dt) if p.dim() > 1 else p.data.clone() for n, p in gm.named_parameters()}
    gm = gm.to(DEV)
    for p in gm.parameters():
        p.grad = torch.zeros_like(p)
    ctx = _ctx(dt)
    for conv in (gm.theta[0], gm.phi[0]):
        conv._pc = ops.PackedConv(conv)
        conv._pc.pack(ctx, True)
    skip = _round(torch.randn(N, Cs, H, H, generator=g), dt)
    gate = _round(torch.randn(N, Cg, H, H, generator=g), dt)
    sn, gn = _node(skip, dt), _node(gate, dt)
    out = ops.attention_gate(ctx, sn, gn, gm, gm.theta[0]._pc, gm.phi[0]._pc)
    dout = _round(torch.randn(N, Cs, H, H, generator=g), dt)
    out.grad = _node(dout, dt).data
    ctx.backward()
    torch.cuda.synchronize()

    rp = {n: v.clone().requires_grad_(True) for n, v in ref_params.items()}
    sr, gr = skip.clone().requires_grad_(True), gate.clone().requires_grad_(True)

    def bn(x, pre):
        return F.batch_norm(x, None, None, rp[pre + ".weight"], rp[pre + ".bias"], training=True, eps=1e-5)

    th = bn(F.conv2d(sr, rp["theta.0.weight"]), "theta.1")
    ph = bn(F.conv2d(gr, rp["phi.0.weight"]), "phi.1")
    f = torch.relu(th + ph)
    psi = bn(F.conv2d(f, rp["psi.0.weight"], rp["psi.0.bias"]), "psi.1")
    ref = sr * torch.sigmoid(psi)
    ref.backward(dout)
    tol = 5e-2 if dt == DT_BF16 else 1e-4
    # fp32 is the parity check; bf16 a sanity bound: th/ph/f and the gradients between the three
    # BNs are stored in bf16 (deterministically 0.16 on the 512-pixel case, same with the generic
    # narrow-gradient kernels and without the weight-gradient stream)
    gtol = 2.5e-1 if dt == DT_BF16 else 1e-4
    assert _rel(_nchw(out.data), ref.detach()) < tol
    assert _rel(_nchw(sn.grad), sr.grad) < gtol
    assert _rel(_nchw(gn.grad), gr.grad) < gtol
    for n, p in gm.named_parameters():
        if n == "psi.0.bias":  # a bias in front of a batch-stat BN has an exactly zero gradient
            assert p.grad.abs().max().item() < (1e-3 if dt == DT_BF16 else 1e-4)
            continue
        assert _rel(p.grad.cpu(), rp[n].grad) < (1e-1 if dt == DT_BF16 else 1e-3), n
