"""Bring-up diagnostic of the persistent halo-A ring's post-op partials: one dgrad_post call, the
per-row-tile partial sums (sum d) compared with torch on the stored d; prints which (row tile,
channel) entries differ.  python tools/diag_persist_post.py N H W K C post"""
import os
import sys

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
for p in (REPO, os.path.join(REPO, "unet-embroidery-seg_amd")):
    sys.path.insert(0, p)
import torch  # noqa: E402

from unetseg_hip.lib import DT_BF16, lib, load  # noqa: E402

load()
N, H, W, K, C, post = map(int, sys.argv[1:7])
dev = "cuda"
g = torch.Generator(device=dev).manual_seed(5)
dy = torch.randn(N, H, W, K, generator=g, device=dev).to(torch.bfloat16)
w = (torch.randn(K, C, 3, 3, generator=g, device=dev) / (C * 9) ** 0.5).float()
wk = torch.empty(K, 3, 3, C, dtype=torch.bfloat16, device=dev)
wt = torch.empty(C, 3, 3, K, dtype=torch.bfloat16, device=dev)
st = torch.cuda.current_stream().cuda_stream
lib.pack_conv_weight(DT_BF16, w.data_ptr(), K, C, 3, 3, C, wk.data_ptr(), wt.data_ptr(), st)
z = torch.randn(N, H, W, C, generator=g, device=dev).to(torch.bfloat16)
aux = torch.relu(z) if post == 1 else z
sc = torch.ones(C, device=dev)
sh = torch.zeros(C, device=dev)
mu = torch.zeros(C, device=dev)
inv = torch.ones(C, device=dev)
coeffs = [sc.data_ptr(), sh.data_ptr(), mu.data_ptr(), inv.data_ptr()] if post == 2 else [0, 0, 0, 0]
args = [DT_BF16, dy.data_ptr(), K, N, H, W, wt.data_ptr(), K, C, 3, 3, 1, 1]
rows = lib.conv2d_dgrad_post(*args, 0, C, H, W, post, aux.data_ptr(), C, *coeffs, 0, 0, st)
dx = torch.empty(N, H, W, C, dtype=torch.bfloat16, device=dev)
part = torch.full((rows, 2, C), float("nan"), dtype=torch.float32, device=dev)
lib.conv2d_dgrad_post(*args, dx.data_ptr(), C, H, W, post, aux.data_ptr(), C, *coeffs, part.data_ptr(), rows, st)
torch.cuda.synchronize()
# row tile m = 8 x 32 spatial block (rest = m // (W/32): image rows rest*8..+8 of the stacked rows)
d = dx.float().reshape(N * H // 8, 8, W // 32, 32, C).permute(0, 2, 1, 3, 4).reshape(rows, 256, C)
ref = d.double().sum(1)
got = part[:, 0].double()
bad = ~torch.isclose(got, ref, rtol=1e-3, atol=1e-2)
print("rows", rows, "bad entries", int(bad.sum()), "of", bad.numel(), "nan", int(torch.isnan(got).sum()))
if bad.any():
    idx = bad.nonzero()[:12].tolist()
    for r, c in idx:
        print(f"  tile {r} ch {c}: got {got[r, c].item():.4f} ref {ref[r, c].item():.4f}")
    print("bad per row tile:", bad.sum(1)[:16].tolist())
    print("bad per channel block of 16:", bad.sum(0).reshape(-1, 16).sum(1).tolist())
