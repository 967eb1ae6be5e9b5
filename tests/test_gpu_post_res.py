"""Residual BN-add-ReLU backward pass 1 in the next block's conv1 data gradient
(unetseg_conv2d_dgrad_post_res; reference: model/resnet_backbone.py:88 conv1, :110-113 bn3 + residual add +
ReLU).

Kernel level: the fused call must store exactly mask * (the accumulated bf16 data gradient the plain
unetseg_conv2d_dgrad(accumulate=1) produces) -- the same tile computes the same GEMM and rounds the sum the
same way -- and its row partials must merge to the float64 sums of d and d * xhat over the pixels
(tolerance 1e-4 of the sum of |terms|).  Shapes: the bench's conv1 data gradients at the three tile
configurations the fused epilogue exists for (1 K step: 128x128 single stage; 2-4 steps: the short-K
single-stage tile; 8 steps at 16x16: the 256x128 ring with one tap), with and without the downsample
branch, and each layer's block-0 conv1, whose dx is a channel slice of the decoder's skip-concat gradient
(pixel stride = the concat width; the other channels must stay untouched).  Model level: a bf16 unet_resnet50 train step with the fusion on and off gives the same forward,
bit-identical gradients for every parameter the backward reaches before the first fused block, and
elsewhere gradients as close to the fp32 HIP step as the unfused bf16 step's (median and mean of the
per-tensor relative L2 within 10 %), while the on/off difference stays below bf16's own deviation from
fp32: the fused partials are summed in another order, a one-ulp change of a BN coefficient flips bf16
roundings, and the encoder backward (Lovasz at B=4) amplifies them, so a fixed tolerance would test noise.
"""
import numpy as np
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


def _P(t):
    return 0 if t is None else t.data_ptr()


# (N, H, W, K (conv1 output = reduction), C (block channels = dgrad output), second branch, expected config,
# pixel stride of dx: C, or the decoder's skip-concat width when the gradient is a channel slice of it)
SHAPES = [
    (16, 128, 128, 64, 256, False, "tn128x128_1step", 256),   # layer1 blocks 1-2
    (4, 64, 64, 128, 512, True, "tn128x128_1st", 512),        # layer2 block 1 (block 0 below it has a downsample)
    (16, 32, 32, 256, 1024, False, "tn128x128_1st", 1024),    # layer3
    (16, 16, 16, 512, 2048, True, "ring256x128_t1", 2048),    # layer4
    (1, 15, 17, 64, 256, False, None, 256),                   # ragged rows
    # fewer than 65 rows in the last (only) tile: its second row-wave is empty and the epilogue's
    # unconditional loads must stay inside the tensor (the 2x2 layer4 maps of a 64^2 input, M = 8)
    (2, 2, 2, 512, 2048, True, None, 2048),
    (1, 5, 5, 64, 256, False, None, 256),
    # a layer's block 0 conv1, fusing the previous layer's last block (its output is also the decoder's
    # skip input, up_concat2/3/4 in = 512 / 1024 / 3072 channels: dx is the first C channels of that
    # gradient, after the downsample branch accumulated onto it)
    (16, 128, 128, 128, 256, False, "fused", 512),            # layer2.0 conv1 <- layer1.2
    (16, 64, 64, 256, 512, False, "fused", 1024),             # layer3.0 conv1 <- layer2.3
    (16, 32, 32, 512, 1024, False, "fused", 3072),            # layer4.0 conv1 <- layer3.5
]


@pytest.mark.parametrize("N,H,W,K,C,two,cfg,ldx", SHAPES)
def test_dgrad_post_res_kernel(N, H, W, K, C, two, cfg, ldx):
    from unetseg_hip import introspect
    from unetseg_hip.lib import DT_BF16, lib

    if cfg is not None and cfg != "fused":
        keys = introspect.call_configs(("dgrad", N, H, W, C, 0, K, 1, 1, 1, 0, C, 0))
        assert keys == [f"dgrad:{cfg}"], keys
    g = torch.Generator(device=DEV).manual_seed(N * 7 + K)
    M = N * H * W
    dy = torch.randn(N, H, W, K, generator=g, device=DEV).bfloat16()
    w = (torch.randn(K, C, generator=g, device=DEV) / K ** 0.5).bfloat16()
    wt = w.t().contiguous()  # [C][K]: the dgrad B operand image (wt [C][R][S][K] with R = S = 1)
    wide = torch.randn(N, H, W, ldx, generator=g, device=DEV).bfloat16()
    old = wide[..., :C].contiguous()
    y1 = torch.randn(N, H, W, C, generator=g, device=DEV).bfloat16()
    mean1 = 0.1 * torch.randn(C, generator=g, device=DEV)
    inv1 = 0.5 + torch.rand(C, generator=g, device=DEV)
    y2 = torch.randn(N, H, W, C, generator=g, device=DEV).bfloat16() if two else None
    mean2 = 0.1 * torch.randn(C, generator=g, device=DEV) if two else None
    inv2 = 0.5 + torch.rand(C, generator=g, device=DEV) if two else None
    mbits = torch.randint(0, 256, (M * (C // 8),), generator=g, device=DEV, dtype=torch.uint8)
    st = _st()
    rows = lib.conv2d_dgrad_post_res(DT_BF16, _P(dy), K, N, H, W, _P(wt), K, C, 0, ldx, _P(y1), C, 0, 0, 0, 0, 0, 0,
                                     0, 0, 0, st)
    if cfg is None and rows == 0:
        pytest.skip("no fused kernel for this shape (the op layer falls back)")
    assert rows > 0
    # reference: the plain accumulating data gradient, then the mask
    ref = old.clone()
    lib.conv2d_dgrad(DT_BF16, _P(dy), K, N, H, W, _P(wt), K, C, 1, 1, 1, 0, _P(ref), C, H, W, 1, st)
    bits = torch.stack([(mbits >> e) & 1 for e in range(8)], dim=1).reshape(M, C).bool()
    dref = torch.where(bits, ref.reshape(M, C).float(), torch.zeros(()).to(DEV))
    nq = 3 if two else 2
    part = torch.full((rows, nq, C), float("nan"), device=DEV)
    buf = wide.clone()
    dx = buf[..., :C]
    lib.conv2d_dgrad_post_res(DT_BF16, _P(dy), K, N, H, W, _P(wt), K, C, _P(dx), ldx, _P(y1), C, _P(mean1), _P(inv1),
                              _P(mbits), _P(y2), C, _P(mean2), _P(inv2), _P(part), rows, st)
    torch.cuda.synchronize()
    assert torch.equal(buf[..., C:], wide[..., C:]), "channels past C were written"
    assert torch.equal(dx.reshape(M, C).float(), dref), (dx.reshape(M, C).float() - dref).abs().max().item()
    d64 = dref.double()
    terms = [d64, d64 * ((y1.reshape(M, C).double() - mean1.double()) * inv1.double())]
    if two:
        terms.append(d64 * ((y2.reshape(M, C).double() - mean2.double()) * inv2.double()))
    got = part.double().sum(0)
    for k, t in enumerate(terms):
        bound = 1e-4 * t.abs().sum(0) + 1e-6
        err = (got[k] - t.sum(0)).abs()
        assert bool((err <= bound).all()), f"quantity {k}: max err {err.max().item():.3e}"


def test_train_step_post_res_matches_unfused(monkeypatch):
    """unet_resnet50 bf16 train step (Lovasz): fused residual backward vs the separate reduce pass, both
    against the fp32 HIP step of the same weights and batch."""
    from model.model_factory import build_model
    from oracle import ref_cpu
    from oracle.weights import make_torch_state
    from unetseg_hip import ops
    from unetseg_hip.losses import binary_segmentation_loss
    from utils.synthetic import make_batch

    state = make_torch_state(ref_cpu.model_spec("unet_resnet50", num_classes=2))
    x, y = make_batch(4, 128, seed=9)
    runs = {}
    for tag, on, dt in (("on", True, "bf16"), ("off", False, "bf16"), ("f32", False, "fp32")):
        monkeypatch.setattr(ops, "FUSE_RES", on)
        m = build_model("unet_resnet50", num_classes=2)
        m.load_state_dict(state)
        m = m.to(DEV).train()
        m.compute_dtype = dt
        o = m(x.to(DEV))
        loss = binary_segmentation_loss(o, y.to(DEV), "lovasz_hinge")
        loss.backward()
        torch.cuda.synchronize()
        runs[tag] = (o.detach().float().cpu(), loss.item(),
                     {n: p.grad.detach().double().cpu().clone() for n, p in m.named_parameters()})
    (o1, l1, g1), (o2, l2, g2), (_, _, g3) = runs["on"], runs["off"], runs["f32"]
    assert torch.equal(o1, o2) and l1 == l2

    def rel(a, b):
        den = b.norm().item()
        return (a - b).norm().item() / den if den > 0 else (a - b).norm().item()

    # the decoder and layer4's last block run before the first fused block (layer4.2's conv1 fuses
    # layer4.1's bn3): their gradients do not depend on the fusion
    before = [n for n in g1 if not n.startswith("resnet.") or n.startswith("resnet.layer4.2.")]
    for n in before:
        assert torch.equal(g1[n], g2[n]), n
    names = list(g1)
    r_onoff = np.array([rel(g1[n], g2[n]) for n in names])
    e_on = np.array([rel(g1[n], g3[n]) for n in names])
    e_off = np.array([rel(g2[n], g3[n]) for n in names])
    print(f"post_res on/off relative L2: median {np.median(r_onoff):.3e} max {r_onoff.max():.3e}; vs fp32: "
          f"on median {np.median(e_on):.3e} mean {e_on.mean():.3e}, off median {np.median(e_off):.3e} "
          f"mean {e_off.mean():.3e}")
    assert np.median(e_on) <= 1.1 * np.median(e_off) + 1e-6
    assert e_on.mean() <= 1.1 * e_off.mean() + 1e-6
    assert np.median(r_onoff) <= np.median(e_off)
