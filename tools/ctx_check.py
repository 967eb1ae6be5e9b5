"""Does the fp32 parity check of one model depend on what ran before it in the process?
Runs the body of tests/test_gpu_models.py::test_model_fp32_parity, then the mIoU test's workload,
then the body again, printing (med_h, med_c) and the max gradient difference between the two runs."""
import os
import sys

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
for p in (REPO, os.path.join(REPO, "unet-embroidery-seg_amd"), os.path.join(REPO, "tests")):
    sys.path.insert(0, p)

import numpy as np  # noqa: E402
import torch  # noqa: E402

import test_gpu_models as T  # noqa: E402


def body(name):
    torch.set_num_threads(16)
    m, state, params, buffers, x, y, c = T._setup(name, 64, 2, seed=21)
    m.compute_dtype = "fp32"
    mask = (torch.rand(2, 512, generator=torch.Generator().manual_seed(3)) >= 0.5).float()
    out, loss, g = T._run_hip(m, name, x, y, c, mask)
    o32, l32, g32, b32 = T._oracle_grads(name, state, x, y, c, mask, torch.float32)
    o64, l64, g64, _ = T._oracle_grads(name, state, x, y, c, mask, torch.float64)
    scale = float(np.median([v.norm().item() for v in g64.values()]))
    e_hip, e_cpu = T._grad_errors(g, g64, scale), T._grad_errors(g32, g64, scale)
    print("med_h %.6e med_c %.6e  logit err %.3e" % (np.median(list(e_hip.values())), np.median(list(e_cpu.values())),
                                                     (out - o32).abs().max().item()), flush=True)
    return out, g, g32, g64


def miou_workload():
    from model.model_factory import build_model
    from oracle import ref_cpu
    from oracle.weights import make_torch_state
    from unetseg_hip import losses
    from utils.synthetic import make_batch
    state = make_torch_state(ref_cpu.model_spec("unet_resnet50", num_classes=2))
    params, buffers = ref_cpu.split_state(state)
    m = build_model("unet_resnet50", num_classes=2)
    m.load_state_dict(state)
    m = m.to("cuda").eval()
    m.compute_dtype = "fp32"
    conf = torch.zeros(4, dtype=torch.int64, device="cuda")
    for i in range(int(os.environ.get("NB", "2"))):
        x, y = make_batch(8, 512, seed=50_000 + i)
        with torch.no_grad():
            o = m(x.to("cuda"))
            losses.binary_confusion(o, y.to("cuda"), conf)
            if os.environ.get("CPU", "1") == "1":
                ref_cpu.forward("unet_resnet50", params, buffers, x, train=False)
    torch.cuda.synchronize()


if __name__ == "__main__":
    name = sys.argv[1] if len(sys.argv) > 1 else "unet_plain"
    a = body(name)
    miou_workload()
    b = body(name)
    for lbl, i in (("hip out", 0), ("hip grads", 1), ("oracle32", 2), ("oracle64", 3)):
        if i == 0:
            d = (a[0] - b[0]).abs().max().item()
        else:
            d = max((a[i][k] - b[i][k]).abs().max().item() for k in a[i])
        print(f"{lbl}: max diff between runs {d:.3e}")
