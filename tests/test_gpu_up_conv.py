"""The decoder's last upsample blended inside its consumer conv (reference model/unet_resnet.py:21,90-97:
up_conv = UpsamplingBilinear2d(2) -> Conv2d(64, 64, 3) -> ReLU -> ...).

unetseg_conv2d_fwd_up_mask / unetseg_conv2d_wgrad_up take the half-resolution source and blend each
halo tile of the upsampled input in the conv (the four-tap arithmetic of unetseg_upsample2x_fwd), so the
full-resolution tensor is never stored.  They must equal unetseg_upsample2x_fwd followed by
unetseg_conv2d_fwd_mask / unetseg_conv2d_wgrad bit for bit: y, the ReLU bits and dW.  Shapes: the
bench's 16 x 512^2, a small multi-image case, both align_corners modes.
"""
import math

import pytest
import torch

pytestmark = pytest.mark.gpu
DEV = "cuda"

#: (N, H, W, align) -- H, W of the conv (upsampled) grid
UP_SHAPES = [(16, 512, 512, 1), (2, 64, 96, 1), (3, 32, 64, 0)]


@pytest.fixture(scope="module", autouse=True)
def _need_gpu():
    if not torch.cuda.is_available():
        pytest.skip("no GPU")
    from unetseg_hip import load
    load()


def _st():
    return torch.cuda.current_stream().cuda_stream


@pytest.mark.parametrize("N,H,W,align", UP_SHAPES)
def test_up_conv_bit_identical(N, H, W, align):
    from unetseg_hip.lib import DT_BF16, lib
    g = torch.Generator(device=DEV).manual_seed(N * 31 + H + W + align)
    C = 64
    M = N * H * W
    st = _st()
    src = torch.randn(N, H // 2, W // 2, C, generator=g, device=DEV).to(torch.bfloat16)
    w = (torch.randn(C, C, 3, 3, generator=g, device=DEV) / math.sqrt(9 * C)).contiguous()
    b = torch.randn(C, generator=g, device=DEV) * 0.1
    wk = torch.empty(C, 3, 3, C, dtype=torch.bfloat16, device=DEV)
    wt = torch.empty(C, 3, 3, C, dtype=torch.bfloat16, device=DEV)
    lib.pack_conv_weight(DT_BF16, w.data_ptr(), C, C, 3, 3, C, wk.data_ptr(), wt.data_ptr(), st)
    assert lib.conv2d_fwd_up_mask(DT_BF16, 0, C, N, H, W, align, 0, 0, 0, C, 0, 0) == 1
    assert lib.conv2d_fwd_up_mask(DT_BF16, 0, C, N, H, W + 2, align, 0, 0, 0, C, 0, 0) == 0  # no halo path

    # reference: the stored upsample, then the conv with bits
    up = torch.empty(N, H, W, C, dtype=torch.bfloat16, device=DEV)
    lib.upsample2x_fwd(DT_BF16, src.data_ptr(), C, N, H // 2, W // 2, C, align, up.data_ptr(), C, st)
    torch.cuda.synchronize()
    ref = torch.nn.functional.interpolate(src.permute(0, 3, 1, 2).float(), scale_factor=2, mode="bilinear",
                                          align_corners=bool(align)).permute(0, 2, 3, 1)
    assert (up.float() - ref).abs().max().item() <= 2 ** -7 * ref.abs().max().item()  # the upsample itself
    y_ref = torch.empty(N, H, W, C, dtype=torch.bfloat16, device=DEV)
    mb_ref = torch.empty(M * 8, dtype=torch.uint8, device=DEV)
    assert lib.conv2d_fwd_mask(DT_BF16, up.data_ptr(), C, N, H, W, wk.data_ptr(), b.data_ptr(), y_ref.data_ptr(), C,
                               mb_ref.data_ptr(), st) == 0
    y = torch.full((N, H, W, C), float("nan"), dtype=torch.bfloat16, device=DEV)
    mb = torch.full((M * 8,), 0x3C, dtype=torch.uint8, device=DEV)
    assert lib.conv2d_fwd_up_mask(DT_BF16, src.data_ptr(), C, N, H, W, align, wk.data_ptr(), b.data_ptr(),
                                  y.data_ptr(), C, mb.data_ptr(), st) == 0
    torch.cuda.synchronize()
    bad = int((y.view(torch.int16) != y_ref.view(torch.int16)).sum())
    assert bad == 0, f"{bad} outputs differ from upsample + conv"
    assert torch.equal(mb, mb_ref)

    # weight gradient
    dy = torch.randn(N, H, W, C, generator=g, device=DEV).to(torch.bfloat16)
    ws_bytes = lib.conv2d_wgrad_workspace(DT_BF16, N, H, W, C, C, 3, 3)
    ws = torch.empty(ws_bytes // 4 + 1, device=DEV)
    dw_ref = torch.full((C, C, 3, 3), float("nan"), device=DEV)
    lib.conv2d_wgrad(DT_BF16, up.data_ptr(), C, C, 0, 0, 0, N, H, W, dy.data_ptr(), C, C, 3, 3, 1, 1, ws.data_ptr(),
                     ws_bytes, dw_ref.data_ptr(), C, 0, st)
    torch.cuda.synchronize()
    dw = torch.full((C, C, 3, 3), float("nan"), device=DEV)
    lib.conv2d_wgrad_up(DT_BF16, src.data_ptr(), C, N, H, W, align, dy.data_ptr(), C, C, ws.data_ptr(), ws_bytes,
                        dw.data_ptr(), 0, st)
    torch.cuda.synchronize()
    assert torch.equal(dw, dw_ref), f"dW differs: max {float((dw - dw_ref).abs().max())}"

    if N == 16:  # kernel times at the bench shape (information for DESIGN; no bound)
        def timed(fn, reps=5):
            fn()
            e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
            e0.record()
            for _ in range(reps):
                fn()
            e1.record()
            torch.cuda.synchronize()
            return e0.elapsed_time(e1) / reps * 1e3

        t_up = timed(lambda: lib.upsample2x_fwd(DT_BF16, src.data_ptr(), C, N, H // 2, W // 2, C, align, up.data_ptr(),
                                                C, st))
        t_fwd = timed(lambda: lib.conv2d_fwd_mask(DT_BF16, up.data_ptr(), C, N, H, W, wk.data_ptr(), b.data_ptr(),
                                                  y_ref.data_ptr(), C, mb_ref.data_ptr(), st))
        t_fused = timed(lambda: lib.conv2d_fwd_up_mask(DT_BF16, src.data_ptr(), C, N, H, W, align, wk.data_ptr(),
                                                       b.data_ptr(), y.data_ptr(), C, mb.data_ptr(), st))
        t_wg = timed(lambda: lib.conv2d_wgrad(DT_BF16, up.data_ptr(), C, C, 0, 0, 0, N, H, W, dy.data_ptr(), C, C, 3,
                                              3, 1, 1, ws.data_ptr(), ws_bytes, dw_ref.data_ptr(), C, 0, st))
        t_wgu = timed(lambda: lib.conv2d_wgrad_up(DT_BF16, src.data_ptr(), C, N, H, W, align, dy.data_ptr(), C, C,
                                                  ws.data_ptr(), ws_bytes, dw.data_ptr(), 0, st))
        print(f"\nup+conv {t_up:.1f}+{t_fwd:.1f} us -> fused {t_fused:.1f} us; wgrad {t_wg:.1f} -> from source "
              f"{t_wgu:.1f} us")
