"""How far does the oracle's own fp32 gradient sit from its fp64 gradient?  (conditioning check)"""
import sys, os
sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path.insert(0, os.path.join(os.path.dirname(os.path.dirname(os.path.abspath(__file__))), "unet-embroidery-seg_amd"))
import torch
from oracle import ref_cpu
from oracle.weights import make_torch_state
from utils.synthetic import make_batch
torch.set_num_threads(8)
for name in sys.argv[1].split(","):
    kw = dict(num_classes=1) if name == "multitask_unet" else dict(num_classes=2)
    state = make_torch_state(ref_cpu.model_spec(name, **kw))
    B, S = int(os.environ.get("B", 2)), int(os.environ.get("S", 64))
    x, y, c = make_batch(B, S, seed=21, with_cls=True)
    res = {}
    for dt in (torch.float32, torch.float64):
        p, b = ref_cpu.split_state(state)
        p = {k: v.detach().to(dt).requires_grad_(True) for k, v in p.items()}
        b = {k: (v.to(dt) if v.is_floating_point() else v) for k, v in b.items()}
        xx = x.to(dt)
        if name == "multitask_unet":
            mask = (torch.rand(B, 512, generator=torch.Generator().manual_seed(3)) >= 0.5).to(dt)
            s, cl = ref_cpu.forward(name, p, b, xx, True, mask)
            loss, _, _ = ref_cpu.multitask_loss(s, cl, y, c)
        else:
            out = ref_cpu.forward(name, p, b, xx, True)
            loss = ref_cpu.binary_segmentation_loss(out, y, sys.argv[2] if len(sys.argv) > 2 else "lovasz_hinge")
        loss.backward()
        res[dt] = {k: v.grad.double() for k, v in p.items()}
    rows = sorted((((res[torch.float32][k] - res[torch.float64][k]).norm() / (res[torch.float64][k].norm() + 1e-30)).item(), k)
                  for k in res[torch.float64])
    print(name, "median", rows[len(rows)//2][0], "worst", rows[-3:])
