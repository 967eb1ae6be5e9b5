"""Isolated upsample x2 timings at the unet_resnet50 512x512 batch-16 decoder shapes (bf16,
align_corners=True): forward, and backward with the fused ReLU mask.  Library: UNETSEG_LIB_PATH."""
import os
import sys

import torch

sys.path.insert(0, os.path.join(os.path.dirname(os.path.abspath(__file__)), "..", "unet-embroidery-seg_amd"))
from unetseg_hip.lib import DT_BF16, lib  # noqa: E402

DEV = "cuda"
st = torch.cuda.current_stream().cuda_stream


def timeit(fn, it=20):
    for _ in range(3):
        fn()
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    torch.cuda.synchronize()
    e0.record()
    for _ in range(it):
        fn()
    e1.record()
    torch.cuda.synchronize()
    return e0.elapsed_time(e1) / it * 1e3


for (H, C) in [(256, 64), (128, 128), (64, 256), (32, 512)]:
    N = 16
    x = torch.randn(N, H, H, C, device=DEV).to(torch.bfloat16)
    y = torch.empty(N, 2 * H, 2 * H, C, device=DEV, dtype=torch.bfloat16)
    tf = timeit(lambda: lib.upsample2x_fwd(DT_BF16, x.data_ptr(), C, N, H, H, C, 1, y.data_ptr(), C, st))
    rows = lib.upsample2x_bwd_tiles(DT_BF16, N, H, H, C)
    part = torch.empty(rows, 2, C, device=DEV)
    dx = torch.empty_like(x)
    tb = timeit(lambda: lib.upsample2x_bwd_relu(DT_BF16, y.data_ptr(), C, N, H, H, C, 1, x.data_ptr(), C,
                                                dx.data_ptr(), C, part.data_ptr(), rows, st))
    out = torch.zeros(C, device=DEV)
    tc = timeit(lambda: lib.colsum_rows(part.data_ptr(), C, rows, 0, out.data_ptr(), 1, st))
    fb = (x.numel() + y.numel()) * 2
    bb = (y.numel() + 2 * x.numel()) * 2
    print(f"H={H:4d} C={C:4d}  fwd {tf:7.1f} us {fb / tf / 1e3:5.2f} GB/s   bwd_relu {tb:7.1f} us {bb / tb / 1e3:5.2f} GB/s"
          f"   colsum_rows (G={rows}) {tc:6.1f} us")
