"""The stem pool's specialised kernels (3x3, stride 2, ceil mode; reference model/resnet_backbone.py:135
nn.MaxPool2d(kernel_size=3, stride=2, padding=0, ceil_mode=True)) against the generic pooling kernels
(UNETSEG_MAXPOOL_GENERIC=1, read per call), which test_gpu_ops.py::test_maxpool checks against
torch.nn.functional.max_pool2d: the pooled values, the argmax bytes and the input gradient (plain and
accumulated) must be bit-identical -- same comparisons, same summation order.  Shapes: the bench's
16 x 256^2 x 64 stem output, odd sizes (partial last windows in both directions), fp32 and bf16,
with ties and NaNs in the input.
"""
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


def _run(lib, dt, x, dy, acc0, generic, k=3, ceil=1):
    N, H, W, C = x.shape
    st = torch.cuda.current_stream().cuda_stream
    P, Q = dy.shape[1], dy.shape[2]
    y = torch.full((N, P, Q, C), float("nan"), dtype=x.dtype, device=DEV)
    idx = torch.full((N * P * Q * C,), 0xEE, dtype=torch.uint8, device=DEV)
    dx = acc0.clone() if acc0 is not None else torch.full_like(x, float("nan"))
    if generic:
        os.environ["UNETSEG_MAXPOOL_GENERIC"] = "1"
    try:
        assert lib.maxpool_fwd(dt, x.data_ptr(), C, N, H, W, C, k, 2, ceil, y.data_ptr(), C, idx.data_ptr(), None,
                               None, st) == 0
        assert lib.maxpool_bwd(dt, dy.data_ptr(), C, idx.data_ptr(), N, H, W, C, k, 2, P, Q, dx.data_ptr(), C,
                               int(acc0 is not None), st) == 0
        torch.cuda.synchronize()
    finally:
        os.environ.pop("UNETSEG_MAXPOOL_GENERIC", None)
    return y, idx, dx


@pytest.mark.parametrize("dtname", ["bf16", "fp32"])
@pytest.mark.parametrize("N,H,W,C", [(16, 256, 256, 64), (2, 17, 23, 16), (1, 6, 9, 8), (3, 3, 4, 24)])
def test_maxpool_k3s2_matches_generic(dtname, N, H, W, C):
    from unetseg_hip.lib import DT_BF16, DT_F32, lib
    dt = DT_BF16 if dtname == "bf16" else DT_F32
    tdt = torch.bfloat16 if dt == DT_BF16 else torch.float32
    if C % (8 if dt == DT_BF16 else 4):
        pytest.skip("vector width")
    g = torch.Generator(device=DEV).manual_seed(H * 31 + W)
    x = torch.randn(N, H, W, C, generator=g, device=DEV).to(tdt)
    x[0, :3, :3, :] = 0.5  # ties inside one window
    x[-1, H // 2, W // 2, 1] = float("nan")
    P = (H - 3 + 1) // 2 + 1
    Q = (W - 3 + 1) // 2 + 1
    if (P - 1) * 2 >= H:
        P -= 1
    if (Q - 1) * 2 >= W:
        Q -= 1
    dy = torch.randn(N, P, Q, C, generator=g, device=DEV).to(tdt)
    acc0 = torch.randn(N, H, W, C, generator=g, device=DEV).to(tdt)
    for acc in (None, acc0):
        ref = _run(lib, dt, x, dy, acc, True)
        got = _run(lib, dt, x, dy, acc, False)
        for name, a, b in zip(("y", "idx", "dx"), got, ref):
            a = a.view(torch.int16 if a.dtype == torch.bfloat16 else torch.int32 if a.dtype == torch.float32 else a.dtype)
            b = b.view(a.dtype)
            assert torch.equal(a, b), f"{name} differs (accumulate={acc is not None}): {int((a != b).sum())} elements"


@pytest.mark.parametrize("dtname", ["bf16", "fp32"])
@pytest.mark.parametrize("N,H,W,C", [(8, 512, 512, 64), (8, 64, 64, 512), (2, 18, 22, 16), (1, 7, 9, 8)])
def test_maxpool_k2s2_matches_generic(dtname, N, H, W, C):
    """The 2x2 / stride-2 pool of unet_plain / attention_unet (model/unet_plain.py:25; floor mode): the
    exact-tiling kernels against the generic ones (odd sizes take the generic path in both runs)."""
    from unetseg_hip.lib import DT_BF16, DT_F32, lib
    dt = DT_BF16 if dtname == "bf16" else DT_F32
    tdt = torch.bfloat16 if dt == DT_BF16 else torch.float32
    if C % (8 if dt == DT_BF16 else 4):
        pytest.skip("vector width")
    g = torch.Generator(device=DEV).manual_seed(H * 37 + W)
    x = torch.randn(N, H, W, C, generator=g, device=DEV).to(tdt)
    x[0, :2, :2, :] = 0.5  # ties inside one window
    x[-1, H // 2, W // 2, 1] = float("nan")
    P, Q = H // 2, W // 2
    dy = torch.randn(N, P, Q, C, generator=g, device=DEV).to(tdt)
    dy[0, 0, 0, 0] = -0.0
    acc0 = torch.randn(N, H, W, C, generator=g, device=DEV).to(tdt)
    for acc in (None, acc0):
        ref = _run(lib, dt, x, dy, acc, True, k=2, ceil=0)
        got = _run(lib, dt, x, dy, acc, False, k=2, ceil=0)
        for name, a, b in zip(("y", "idx", "dx"), got, ref):
            a = a.view(torch.int16 if a.dtype == torch.bfloat16 else torch.int32 if a.dtype == torch.float32 else a.dtype)
            b = b.view(a.dtype)
            assert torch.equal(a, b), f"{name} differs (accumulate={acc is not None}): {int((a != b).sum())} elements"
