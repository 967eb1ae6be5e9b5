"""The head's input gradient synthesised instead of stored (reference model/unet_resnet.py:77-79:
up_conv[3] Conv2d(64, 64, 3) -> ReLU -> final Conv2d(64, k, 1); the same head in
model/unet_multitask.py's seg head).

With the head fused into the producer conv's epilogue, the backward of `final` through the ReLU is
dY[pix][c] = bf16(y[pix][c] > 0 ? sum_k dlogit[k][pix] * W_final[k][c] : 0) (pw_small_bwd_relu's dx).
unetseg_conv2d_fwd_head_mask stores y's ReLU bits; unetseg_pw_small_bwd_relu with dx == NULL then
writes only the head's weight / bias partials and the producer's bias partials, and the producer's
data gradient (unetseg_conv2d_dgrad_post_syn, post 4) and weight gradient (unetseg_conv2d_wgrad_syn)
rebuild dY from the logit gradient, the head weights and the bits inside their halo tiles.  Every
output must equal the stored-dY path bit for bit: the forward (y, logits) of the plain fused head,
the mask bytes, the three partial buffers, dx + its bias partials, and dW.  Shapes: the bench's
16 x 512^2 (k = 2), C5's 8 x 512^2 (k = 1) and a small multi-image case.  Model level: a bf16
unet_resnet50 train step with the synthesis on and off gives bit-identical logits, loss and
parameter gradients.
"""
import math

import pytest
import torch

pytestmark = pytest.mark.gpu
DEV = "cuda"

#: (N, H, W, k) -- tests/test_gpu_configs.py covered_keys() lists these shapes' configurations
HEAD_SYN_SHAPES = [(16, 512, 512, 2), (8, 512, 512, 1), (2, 64, 96, 2)]


@pytest.fixture(scope="module", autouse=True)
def _need_gpu():
    if not torch.cuda.is_available():
        pytest.skip("no GPU")
    from unetseg_hip import load
    load()


def _st():
    return torch.cuda.current_stream().cuda_stream


def _bits(t16):
    return t16.view(torch.int16)


@pytest.mark.parametrize("N,H,W,K", HEAD_SYN_SHAPES)
def test_head_syn_bit_identical(N, H, W, K):
    from unetseg_hip import introspect
    from unetseg_hip.lib import DT_BF16, lib
    g = torch.Generator(device=DEV).manual_seed(N * 977 + H + W + K)
    C = 64
    M = N * H * W
    st = _st()

    def packed(w):
        wk = torch.empty(C, 3, 3, C, dtype=torch.bfloat16, device=DEV)
        wt = torch.empty(C, 3, 3, C, dtype=torch.bfloat16, device=DEV)
        lib.pack_conv_weight(DT_BF16, w.data_ptr(), C, C, 3, 3, C, wk.data_ptr(), wt.data_ptr(), st)
        return wk, wt

    x0 = torch.randn(N, H, W, C, generator=g, device=DEV).to(torch.bfloat16)
    w1 = (torch.randn(C, C, 3, 3, generator=g, device=DEV) / math.sqrt(9 * C)).contiguous()
    w2 = (torch.randn(C, C, 3, 3, generator=g, device=DEV) / math.sqrt(9 * C)).contiguous()
    b1 = torch.randn(C, generator=g, device=DEV) * 0.1
    b2 = torch.randn(C, generator=g, device=DEV) * 0.1
    hw = torch.randn(K, C, generator=g, device=DEV) / 8
    hb = torch.randn(K, generator=g, device=DEV) * 0.1
    wk1, wt1 = packed(w1)
    wk2, wt2 = packed(w2)
    # conv1 (+ its bits: the post-4 mask of conv2's data gradient)
    c1 = torch.empty(N, H, W, C, dtype=torch.bfloat16, device=DEV)
    mb1 = torch.empty(M * 8, dtype=torch.uint8, device=DEV)
    assert lib.conv2d_fwd_mask(DT_BF16, x0.data_ptr(), C, N, H, W, wk1.data_ptr(), b1.data_ptr(), c1.data_ptr(), C,
                               mb1.data_ptr(), st) == 0
    # conv2 + fused head: plain and with the bits
    y_ref = torch.empty(N, H, W, C, dtype=torch.bfloat16, device=DEV)
    lg_ref = torch.empty(N, K, H, W, device=DEV)
    lib.conv2d_fwd_head(DT_BF16, c1.data_ptr(), C, N, H, W, wk2.data_ptr(), b2.data_ptr(), y_ref.data_ptr(), C, K,
                        hw.data_ptr(), hb.data_ptr(), lg_ref.data_ptr(), st)
    y = torch.full((N, H, W, C), float("nan"), dtype=torch.bfloat16, device=DEV)
    lg = torch.full((N, K, H, W), float("nan"), device=DEV)
    mb2 = torch.full((M * 8,), 0x5A, dtype=torch.uint8, device=DEV)
    lib.conv2d_fwd_head_mask(DT_BF16, c1.data_ptr(), C, N, H, W, wk2.data_ptr(), b2.data_ptr(), y.data_ptr(), C, K,
                             hw.data_ptr(), hb.data_ptr(), lg.data_ptr(), mb2.data_ptr(), st)
    torch.cuda.synchronize()
    assert torch.equal(_bits(y), _bits(y_ref)), "stored activation differs from the plain fused head"
    assert torch.equal(lg, lg_ref), "logits differ from the plain fused head"
    on = (y.reshape(M, 8, 8).float() > 0).to(torch.int32)
    want = (on << torch.arange(8, device=DEV, dtype=torch.int32)).sum(-1).to(torch.uint8).reshape(-1)
    assert torch.equal(mb2, want), f"{int((mb2 != want).sum())} mask bytes differ"
    assert 0.2 < on.float().mean().item() < 0.8

    # head backward: stored dx vs partials only
    dl = torch.randn(N, K, H, W, generator=g, device=DEV)
    G = lib.pw_small_tiles(M)
    bufs = {}
    for tag in ("ref", "syn"):
        bufs[tag] = [torch.full(s, float("nan"), device=DEV) for s in ((K, C, G), (K, G), (G, 2, C))]
    dx_ref = torch.full((N, H, W, C), float("nan"), dtype=torch.bfloat16, device=DEV)
    pw, pb, pd = bufs["ref"]
    lib.pw_small_bwd_relu(DT_BF16, dl.data_ptr(), y.data_ptr(), C, M, H * W, C, K, hw.data_ptr(), dx_ref.data_ptr(), C,
                          pw.data_ptr(), pb.data_ptr(), pd.data_ptr(), st)
    pw, pb, pd = bufs["syn"]
    lib.pw_small_bwd_relu(DT_BF16, dl.data_ptr(), y.data_ptr(), C, M, H * W, C, K, hw.data_ptr(), 0, 0,
                          pw.data_ptr(), pb.data_ptr(), pd.data_ptr(), st)
    torch.cuda.synchronize()
    assert torch.equal(bufs["ref"][0], bufs["syn"][0]), "head weight partials differ"
    assert torch.equal(bufs["ref"][1], bufs["syn"][1]), "head bias partials differ"
    assert torch.equal(bufs["ref"][2][:, 0], bufs["syn"][2][:, 0]), "producer bias partials differ"  # slot 0 only

    # conv2 data gradient (post 4 with conv1's bits): stored dY vs synthesised
    assert introspect.call_configs(("dgrad_syn", N, H, W, C, 0, C, 3, 3, 1, 1, C, 0)) == ["dgrad_syn:halo3"]
    args = [DT_BF16, dx_ref.data_ptr(), C, N, H, W, wt2.data_ptr(), C, C, 3, 3, 1, 1]
    rows = lib.conv2d_dgrad_post(*args, 0, C, H, W, 4, mb1.data_ptr(), 0, 0, 0, 0, 0, 0, 0, st)
    assert rows > 0
    assert lib.conv2d_dgrad_post_syn(DT_BF16, 0, K, 0, 0, N, H, W, 0, 0, C, 0, 0, 0, st) == rows
    gx_ref = torch.full((N, H, W, C), float("nan"), dtype=torch.bfloat16, device=DEV)
    pr_ref = torch.full((rows, 2, C), float("nan"), device=DEV)
    assert lib.conv2d_dgrad_post(*args, gx_ref.data_ptr(), C, H, W, 4, mb1.data_ptr(), 0, 0, 0, 0, 0,
                                 pr_ref.data_ptr(), rows, st) == 0
    gx = torch.full((N, H, W, C), float("nan"), dtype=torch.bfloat16, device=DEV)
    pr = torch.full((rows, 2, C), float("nan"), device=DEV)
    assert lib.conv2d_dgrad_post_syn(DT_BF16, dl.data_ptr(), K, hw.data_ptr(), mb2.data_ptr(), N, H, W,
                                     wt2.data_ptr(), gx.data_ptr(), C, mb1.data_ptr(), pr.data_ptr(), rows, st) == 0
    torch.cuda.synchronize()
    assert torch.equal(_bits(gx), _bits(gx_ref)), f"{int((_bits(gx) != _bits(gx_ref)).sum())} dx values differ"
    assert torch.equal(pr[:, 0], pr_ref[:, 0]), "conv1 bias partials differ"

    # conv2 weight gradient: stored dY vs synthesised
    ws_bytes = lib.conv2d_wgrad_workspace(DT_BF16, N, H, W, C, C, 3, 3)
    ws = torch.empty(ws_bytes // 4 + 1, device=DEV)
    dw_ref = torch.full((C, C, 3, 3), float("nan"), device=DEV)
    lib.conv2d_wgrad(DT_BF16, c1.data_ptr(), C, C, 0, 0, 0, N, H, W, dx_ref.data_ptr(), C, C, 3, 3, 1, 1,
                     ws.data_ptr(), ws_bytes, dw_ref.data_ptr(), C, 0, st)
    torch.cuda.synchronize()
    dw = torch.full((C, C, 3, 3), float("nan"), device=DEV)
    lib.conv2d_wgrad_syn(DT_BF16, c1.data_ptr(), C, N, H, W, dl.data_ptr(), K, hw.data_ptr(), mb2.data_ptr(),
                         ws.data_ptr(), ws_bytes, dw.data_ptr(), 0, st)
    torch.cuda.synchronize()
    assert torch.equal(dw, dw_ref), f"dW differs: max {float((dw - dw_ref).abs().max())}"


def test_train_step_head_syn_bit_identical(monkeypatch):
    from model.model_factory import build_model
    from oracle import ref_cpu
    from oracle.weights import make_torch_state
    from unetseg_hip import ops
    from unetseg_hip.losses import binary_segmentation_loss
    from utils.synthetic import make_batch

    state = make_torch_state(ref_cpu.model_spec("unet_resnet50", num_classes=2))
    x, y = make_batch(2, 128, seed=5)
    runs = {}
    calls = []
    real = ops.lib.conv2d_dgrad_post_syn

    def spy(*a):
        if a[12]:  # a launching call (part != NULL)
            calls.append(a[5:8])
        return real(*a)

    for on in (True, False):
        monkeypatch.setattr(ops, "SYN_HEAD", on)
        calls.clear()
        m = build_model("unet_resnet50", num_classes=2)
        m.load_state_dict(state)
        m = m.to(DEV).train()
        m.compute_dtype = "bf16"
        o = m(x.to(DEV))
        loss = binary_segmentation_loss(o, y.to(DEV), "lovasz_hinge")
        with monkeypatch.context() as mp:
            mp.setattr(ops.lib, "conv2d_dgrad_post_syn", spy, raising=False)
            loss.backward()
        torch.cuda.synchronize()
        assert bool(calls) == on, calls  # the synthesised path ran exactly when enabled
        runs[on] = (o.detach().float().cpu(), loss.item(),
                    {n: p.grad.detach().cpu().clone() for n, p in m.named_parameters()})
    (o1, l1, g1), (o0, l0, g0) = runs[True], runs[False]
    assert torch.equal(o1, o0) and l1 == l0
    for n in g1:
        assert torch.equal(g1[n], g0[n]), n
