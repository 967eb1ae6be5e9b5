"""debug: attention gate fp32 at the C4 512^2 shape -- where does the skip gradient differ?"""
import os, sys
REPO = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path[:0] = [REPO, os.path.join(REPO, "unet-embroidery-seg_amd"), os.path.join(REPO, "tests")]
import torch
import test_gpu_c4c5 as T
from unetseg_hip import load
load()
N, H, Cs, Cg, Ci = [int(v) for v in sys.argv[1:6]]
from model.unet_attention import AttentionGate
from unetseg_hip import ops
from unetseg_hip.lib import DT_F32
DEV = "cuda"
g = torch.Generator(device=DEV).manual_seed(N * H + Cs)
gm = AttentionGate(Cg, Cs, Ci)
for p in gm.parameters():
    p.data = torch.randn(p.shape, generator=torch.Generator().manual_seed(p.numel())) * (0.3 if p.dim() > 1 else 0.2)
for bnm in (gm.theta[1], gm.phi[1], gm.psi[1]):
    bnm.weight.data += 1.0
gm = gm.to(DEV)
for p in gm.parameters():
    p.grad = torch.zeros_like(p)
ctx = ops.Ctx(DT_F32, True, True, torch.device(DEV))
for conv in (gm.theta[0], gm.phi[0]):
    conv._pc = ops.PackedConv(conv)
    conv._pc.pack(ctx, True)
skip = torch.randn(N, H, H, Cs, generator=g, device=DEV)
gate = torch.randn(N, H, H, Cg, generator=g, device=DEV)
sn, gn = ops.Node(skip.clone()), ops.Node(gate.clone())
out = ops.attention_gate(ctx, sn, gn, gm, gm.theta[0]._pc, gm.phi[0]._pc)
dout = torch.randn(N, H, H, Cs, generator=g, device=DEV)
out.grad = dout.clone()
ctx.backward()
torch.cuda.synchronize()
for dt in (torch.float64, torch.float32):
    rp = {n: p.data.to(dt).clone().requires_grad_(True) for n, p in gm.named_parameters()}
    sr, gr = skip.to(dt).requires_grad_(True), gate.to(dt).requires_grad_(True)
    def conv1x1(x, wname, bname=None):
        y = x @ rp[wname].reshape(rp[wname].shape[0], -1).t()
        return y + rp[bname] if bname else y
    def bn(x, pre):
        m = x.mean((0, 1, 2)); v = x.var((0, 1, 2), unbiased=False)
        return (x - m) / torch.sqrt(v + 1e-5) * rp[pre + ".weight"] + rp[pre + ".bias"]
    th = conv1x1(sr, "theta.0.weight"); th.retain_grad()
    f = torch.relu(bn(th, "theta.1") + bn(conv1x1(gr, "phi.0.weight"), "phi.1")); f.retain_grad()
    psi = bn(conv1x1(f, "psi.0.weight", "psi.0.bias"), "psi.1")
    ref = sr * torch.sigmoid(psi)
    ref.backward(dout.to(dt))
    if dt == torch.float64:
        r64 = (sr.grad.detach(), th.grad.detach(), f.grad.detach(), {n: v.grad.detach() for n, v in rp.items()})
        e = (sn.grad.double() - sr.grad).abs()
        print("skip grad: max err", e.max().item(), "max ref", sr.grad.abs().max().item())
        pix = e.amax(-1).reshape(-1)
        idx = torch.nonzero(pix > 1e-3 * sr.grad.abs().max()).reshape(-1)
        print("bad pixels", idx.numel(), "of", pix.numel(), "first", idx[:10].tolist(), "last", idx[-10:].tolist())
        ch = e.reshape(-1, Cs).amax(0)
        print("per-channel max err", [round(v, 4) for v in ch.tolist()][:16])
        print("dskip direct part (dout*alpha) vs total: ", (dout.double()).abs().max().item())
    else:
        e32 = (sr.grad.double() - r64[0]).abs()
        print("torch fp32 vs f64 skip grad max err", e32.max().item())
        print("torch fp32 param grads rel:", {n: round(float((v.grad.double() - r64[3][n]).abs().max() / r64[3][n].abs().max()), 6) for n, v in rp.items()})
print("hip param grads rel:", {n: round(float((p.grad.double() - r64[3][n]).abs().max() / r64[3][n].abs().max()), 6) for n, p in gm.named_parameters()})
