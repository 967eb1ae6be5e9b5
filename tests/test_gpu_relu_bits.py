"""ReLU mask bits between the decoder's 512^2 convs (reference model/unet_resnet.py:90-97 up_conv:
Conv2d(64, 64, 3) -> ReLU -> Conv2d(64, 64, 3) -> ReLU).

unetseg_conv2d_fwd_mask stores y exactly as unetseg_conv2d_fwd (bias + ReLU) and, besides, the packed
mask mbits[pixel][8] with bit e of byte b = (y[pixel][8b + e] > 0).  The consumer's data gradient with
post 4 (mask from those bits) must equal post 1 (mask from y itself) bit for bit: the same dx and the
same bias-gradient partials -- both read the same predicate, only from 1/16 of the bytes.  Shapes: the
bench's 16 x 512^2 and a small multi-image case.  Model level: a bf16 unet_resnet50 train step with
the bits on and off gives bit-identical logits, loss and parameter gradients.
"""
import math

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


@pytest.mark.parametrize("N,H,W", [(16, 512, 512), (2, 64, 96)])
def test_fwd_mask_and_post4(N, H, W):
    from unetseg_hip import introspect
    from unetseg_hip.lib import DT_BF16, lib
    g = torch.Generator(device=DEV).manual_seed(N * 131 + H + W)
    C = 64
    M = N * H * W
    x = torch.randn(N, H, W, C, generator=g, device=DEV).to(torch.bfloat16)
    w = (torch.randn(C, C, 3, 3, generator=g, device=DEV) / math.sqrt(9 * C)).contiguous()
    b = torch.randn(C, generator=g, device=DEV) * 0.1
    wk = torch.empty(C, 3, 3, C, dtype=torch.bfloat16, device=DEV)
    wt = torch.empty(C, 3, 3, C, dtype=torch.bfloat16, device=DEV)
    lib.pack_conv_weight(DT_BF16, w.data_ptr(), C, C, 3, 3, C, wk.data_ptr(), wt.data_ptr(), _st())
    assert lib.conv2d_fwd_mask(DT_BF16, 0, C, N, H, W, 0, 0, 0, C, 0, 0) == 1
    assert lib.conv2d_fwd_mask(DT_BF16, 0, C, N, H, W + 8, 0, 0, 0, C, 0, 0) == 0  # not on the halo path
    y_ref = torch.empty(N, H, W, C, dtype=torch.bfloat16, device=DEV)
    lib.conv2d_fwd(DT_BF16, x.data_ptr(), C, C, 0, 0, 0, N, H, W, wk.data_ptr(), C, 3, 3, 1, 1, b.data_ptr(), 1,
                   y_ref.data_ptr(), C, 0, _st())
    y = torch.full((N, H, W, C), float("nan"), dtype=torch.bfloat16, device=DEV)
    mbits = torch.full((M * 8,), 0xA5, dtype=torch.uint8, device=DEV)
    assert lib.conv2d_fwd_mask(DT_BF16, x.data_ptr(), C, N, H, W, wk.data_ptr(), b.data_ptr(), y.data_ptr(), C,
                               mbits.data_ptr(), _st()) == 0
    torch.cuda.synchronize()
    assert torch.equal(y.view(torch.int16), y_ref.view(torch.int16)), "stored activation differs from the plain conv"
    on = (y.reshape(M, 8, 8).float() > 0).to(torch.int32)
    packed = (on << torch.arange(8, device=DEV, dtype=torch.int32)).sum(-1).to(torch.uint8).reshape(-1)
    assert torch.equal(mbits, packed), f"{int((mbits != packed).sum())} mask bytes differ"
    frac = on.float().mean().item()
    assert 0.2 < frac < 0.8, frac  # both branches of the mask are exercised

    # consumer data gradient: post 4 (bits) == post 1 (activation), dx and partials bit for bit
    assert introspect.call_configs(("dgrad_post4", N, H, W, C, 0, C, 3, 3, 1, 1, C, 0)) == ["dgrad_post4:halo3"]
    dy = torch.randn(N, H, W, C, generator=g, device=DEV).to(torch.bfloat16)
    args = [DT_BF16, dy.data_ptr(), C, N, H, W, wt.data_ptr(), C, C, 3, 3, 1, 1]
    rows1 = lib.conv2d_dgrad_post(*args, 0, C, H, W, 1, y.data_ptr(), C, 0, 0, 0, 0, 0, 0, _st())
    rows4 = lib.conv2d_dgrad_post(*args, 0, C, H, W, 4, mbits.data_ptr(), 0, 0, 0, 0, 0, 0, 0, _st())
    assert rows1 == rows4 and rows4 > 0
    out = {}
    for post, aux, ld in ((1, y, C), (4, mbits, 0)):
        dx = torch.full((N, H, W, C), float("nan"), dtype=torch.bfloat16, device=DEV)
        part = torch.full((rows4, 2, C), float("nan"), device=DEV)
        assert lib.conv2d_dgrad_post(*args, dx.data_ptr(), C, H, W, post, aux.data_ptr(), ld, 0, 0, 0, 0,
                                     part.data_ptr(), rows4, _st()) == 0
        out[post] = (dx, part)
    torch.cuda.synchronize()
    assert torch.equal(out[1][0].view(torch.int16), out[4][0].view(torch.int16)), "dx differs"
    assert torch.equal(out[1][1][:, 0], out[4][1][:, 0]), "bias partials differ"
    # a 1x1 or strided consumer has no post-4 kernel: the op layer falls back to post 1
    assert lib.conv2d_dgrad_post(DT_BF16, dy.data_ptr(), C, N, H, W, wt.data_ptr(), C, C, 1, 1, 1, 0, 0, C, H, W, 4,
                                 mbits.data_ptr(), 0, 0, 0, 0, 0, 0, 0, _st()) == -1


def test_train_step_relu_bits_bit_identical(monkeypatch):
    from model.model_factory import build_model
    from oracle import ref_cpu
    from oracle.weights import make_torch_state
    from unetseg_hip import ops
    from unetseg_hip.losses import binary_segmentation_loss
    from utils.synthetic import make_batch

    state = make_torch_state(ref_cpu.model_spec("unet_resnet50", num_classes=2))
    x, y = make_batch(2, 128, seed=4)
    runs = {}
    for on in (True, False):
        monkeypatch.setattr(ops, "RELU_BITS", on)
        m = build_model("unet_resnet50", num_classes=2)
        m.load_state_dict(state)
        m = m.to(DEV).train()
        m.compute_dtype = "bf16"
        o = m(x.to(DEV))
        loss = binary_segmentation_loss(o, y.to(DEV), "lovasz_hinge")
        loss.backward()
        torch.cuda.synchronize()
        runs[on] = (o.detach().float().cpu(), loss.item(),
                    {n: p.grad.detach().cpu().clone() for n, p in m.named_parameters()})
    (o1, l1, g1), (o0, l0, g0) = runs[True], runs[False]
    assert torch.equal(o1, o0) and l1 == l0
    for n in g1:
        assert torch.equal(g1[n], g0[n]), n
