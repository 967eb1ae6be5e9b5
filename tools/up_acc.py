"""fp32 upsample fwd/bwd error vs an fp64 torch reference (align_corners False/True)."""
import os
import sys

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
for p in (REPO, os.path.join(REPO, "unet-embroidery-seg_amd")):
    sys.path.insert(0, p)
import torch  # noqa: E402
import torch.nn.functional as F  # noqa: E402
from unetseg_hip import ops  # noqa: E402
from unetseg_hip.lib import DT_F32  # noqa: E402

g = torch.Generator().manual_seed(1)
for align in (False, True):
    for (N, C, H) in ((2, 512, 4), (2, 256, 8), (2, 64, 32)):
        x = torch.randn(N, C, H, H, generator=g)
        ctx = ops.Ctx(DT_F32, True, True, torch.device("cuda"))
        xn = ops.Node(x.permute(0, 2, 3, 1).contiguous().cuda())
        y = ops.upsample2x(ctx, xn, align)
        ref = F.interpolate(x.double(), scale_factor=2, mode="bilinear", align_corners=align)
        ef = (y.data.permute(0, 3, 1, 2).cpu().double() - ref).abs().max().item()
        dy = torch.randn(ref.shape, generator=g)
        y.grad = dy.permute(0, 2, 3, 1).contiguous().cuda()
        ctx.backward()
        xr = x.double().requires_grad_(True)
        F.interpolate(xr, scale_factor=2, mode="bilinear", align_corners=align).backward(dy.double())
        eb = (xn.grad.permute(0, 3, 1, 2).cpu().double() - xr.grad).abs().max().item()
        print(f"align={align} N={N} C={C} H={H}: fwd err {ef:.3e}  bwd err {eb:.3e}")
