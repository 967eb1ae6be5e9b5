"""Diagnostic: per-parameter gradient error of the HIP path vs the CPU oracle (fp32 / bf16)."""
import sys, os
sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path.insert(0, os.path.join(os.path.dirname(os.path.dirname(os.path.abspath(__file__))), "unet-embroidery-seg_amd"))
import torch
from model.model_factory import build_model
from oracle import ref_cpu
from oracle.weights import make_torch_state
from unetseg_hip import losses
from utils.synthetic import make_batch

torch.set_num_threads(16)
names = sys.argv[1].split(",") if len(sys.argv) > 1 else ["unet_plain"]
dtn = sys.argv[2] if len(sys.argv) > 2 else "fp32"
for name in names:
    kw = dict(num_classes=1) if name == "multitask_unet" else dict(num_classes=2)
    state = make_torch_state(ref_cpu.model_spec(name, **kw))
    m = build_model(name, **kw); m.load_state_dict(state); m = m.cuda().train(); m.compute_dtype = dtn
    x, y, c = make_batch(2, 64, seed=21, with_cls=True)
    params, buffers = ref_cpu.split_state(state)
    if name == "multitask_unet":
        mask = (torch.rand(2, 512, generator=torch.Generator().manual_seed(3)) >= 0.5).float()
        m.dropout_mask = mask
        seg, cls = m(x.cuda()); loss, _, _ = losses.multitask_loss(seg, cls, y.cuda(), c.cuda(), 1.0, "bce")
        rseg, rcls = ref_cpu.forward(name, params, buffers, x, train=True, dropout_mask=mask)
        rloss, _, _ = ref_cpu.multitask_loss(rseg, rcls, y, c)
        out, rout = seg, rseg
    else:
        out = m(x.cuda()); loss = losses.binary_segmentation_loss(out, y.cuda(), "lovasz_hinge")
        rout = ref_cpu.forward(name, params, buffers, x, train=True); rloss = ref_cpu.binary_segmentation_loss(rout, y, "lovasz_hinge")
    print(name, dtn, "logit err", (out.detach().cpu() - rout.detach()).abs().max().item(), "scale", rout.abs().max().item(),
          "loss", loss.item(), rloss.item())
    loss.backward(); rloss.backward()
    sd = dict(m.named_parameters())
    rows = []
    for k, p in params.items():
        a, b = sd[k].grad.cpu().double(), p.grad.double()
        rows.append(((a - b).norm().item() / (b.norm().item() + 1e-30), k, b.norm().item(), a.norm().item()))
    rows.sort(reverse=True)
    for r in rows[:12]:
        print("  %.3e %-45s ref|g|=%.3e hip|g|=%.3e" % r)
