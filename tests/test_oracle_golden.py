"""CPU: pin the oracle (oracle/ref_cpu.py) against the reference's golden vectors.

The fixtures were produced by oracle/gen_golden.py from the reference itself
(/root/reference, imported read-only in the build container)."""
import os

import numpy as np
import pytest
import torch

from oracle import ref_cpu
from oracle.weights import make_torch_state

MODELS = ["unet_plain", "unet_resnet50", "attention_unet", "multitask_unet"]


def _load(golden_dir, name):
    return np.load(os.path.join(golden_dir, f"model_{name}.npz"))


@pytest.mark.parametrize("name", MODELS)
def test_spec_matches_reference_state_dict(golden_dir, name):
    d = _load(golden_dir, name)
    kw = dict(num_classes=1) if name == "multitask_unet" else dict(num_classes=2)
    spec = ref_cpu.model_spec(name, **kw)
    assert [n for n, _ in spec] == list(d["spec_names"])
    assert [",".join(map(str, s)) for _, s in spec] == list(d["spec_shapes"])


@pytest.mark.parametrize("name", MODELS)
def test_oracle_forward_backward_matches_reference(golden_dir, name):
    torch.set_num_threads(min(8, os.cpu_count() or 1))
    d = _load(golden_dir, name)
    kw = dict(num_classes=1) if name == "multitask_unet" else dict(num_classes=2)
    params, buffers = ref_cpu.split_state(make_torch_state(ref_cpu.model_spec(name, **kw)))
    x, y = torch.from_numpy(d["x"]), torch.from_numpy(d["y"])
    if name == "multitask_unet":
        seg, cls = ref_cpu.forward(name, params, buffers, x, train=True,
                                   dropout_mask=torch.from_numpy(d["dropout_mask"]))
        loss, sl, cl = ref_cpu.multitask_loss(seg, cls, y, torch.from_numpy(d["cls_t"]))
        np.testing.assert_allclose(seg.detach().numpy(), d["seg"], rtol=1e-4, atol=1e-4)
        np.testing.assert_allclose(cls.detach().numpy(), d["cls"], rtol=1e-4, atol=1e-4)
        np.testing.assert_allclose([loss.item(), sl.item(), cl.item()], d["loss"], rtol=1e-5)
    else:
        out = ref_cpu.forward(name, params, buffers, x, train=True)
        loss = ref_cpu.binary_segmentation_loss(out, y, "lovasz_hinge")
        np.testing.assert_allclose(out.detach().numpy(), d["out"], rtol=1e-4, atol=1e-4)
        bce = ref_cpu.binary_segmentation_loss(out, y, "bce")
        bce_pw = ref_cpu.binary_segmentation_loss(out, y, "bce", pos_weight=torch.tensor([2.5]))
        np.testing.assert_allclose([loss.item(), bce.item(), bce_pw.item()], d["loss"], rtol=1e-5)
    loss.backward()
    norms = {n: float(p.grad.double().norm()) for n, p in params.items()}
    ref = dict(zip(d["grad_names"], d["grad_norms"]))
    assert set(ref) == set(norms)
    for n in ref:
        assert abs(norms[n] - ref[n]) <= 1e-3 * ref[n] + 1e-6, (n, norms[n], ref[n])
    for k in d.files:
        if k.startswith("grad::"):
            np.testing.assert_allclose(params[k[6:]].grad.numpy(), d[k], rtol=1e-3, atol=1e-5)
        if k.startswith("state::"):
            np.testing.assert_allclose(buffers[k[7:]].numpy(), d[k], rtol=1e-5, atol=1e-6)
    # eval mode (running stats)
    with torch.no_grad():
        o = ref_cpu.forward(name, params, buffers, x, train=False)
        o = o[0] if isinstance(o, tuple) else o
        np.testing.assert_allclose(o.numpy(), d["eval_out"], rtol=1e-4, atol=2e-4)
        if "eval_conf" in d.files:
            assert list(ref_cpu.binary_confusion(o, y)) == list(d["eval_conf"])


@pytest.mark.parametrize("name", ["unet_plain", "unet_resnet50"])
def test_oracle_cpu_autocast_bf16_matches_reference(golden_dir, name):
    d = _load(golden_dir, name)
    params, buffers = ref_cpu.split_state(make_torch_state(ref_cpu.model_spec(name, num_classes=2)))
    with torch.no_grad(), torch.autocast("cpu", dtype=torch.bfloat16):
        out = ref_cpu.forward(name, params, buffers, torch.from_numpy(d["x"]), train=True).float()
    np.testing.assert_allclose(out.numpy(), d["out_bf16"], rtol=0, atol=1e-5)


def test_losses_match_reference(golden_dir):
    d = np.load(os.path.join(golden_dir, "losses.npz"))
    lg = torch.from_numpy(d["logits"]).requires_grad_(True)
    lv = ref_cpu.lovasz_hinge_loss(lg, torch.from_numpy(d["labels"]))
    lv.backward()
    np.testing.assert_allclose(lv.item(), d["lovasz"][0], rtol=1e-6)
    np.testing.assert_allclose(lg.grad.numpy(), d["lovasz_grad"], rtol=1e-5, atol=1e-9)
    lt = ref_cpu.lovasz_hinge_loss(torch.from_numpy(d["tied"]), torch.from_numpy(d["labels"]))
    np.testing.assert_allclose(lt.item(), d["lovasz_tied"][0], rtol=1e-6)
    two = torch.from_numpy(d["two"]).requires_grad_(True)
    b = ref_cpu.binary_segmentation_loss(two, torch.from_numpy(d["tgt"]), "bce", pos_weight=torch.tensor([1.7]))
    b.backward()
    np.testing.assert_allclose(b.item(), d["bce_pw"][0], rtol=1e-6)
    np.testing.assert_allclose(two.grad.numpy(), d["bce_grad"], rtol=1e-5, atol=1e-10)
    e = ref_cpu.lovasz_hinge_loss(torch.zeros(0, 4, 4), torch.zeros(0, 4, 4))
    assert float(e) == d["empty"][0] == 0.0


def test_metrics_match_reference(golden_dir):
    d = np.load(os.path.join(golden_dir, "metrics.npz"))
    conf = ref_cpu.binary_confusion(torch.from_numpy(d["outs"]), torch.from_numpy(d["tg"]))
    assert list(conf) == list(d["conf"])
    m = ref_cpu.binary_segmentation_metrics(*conf)
    np.testing.assert_allclose([m[k] for k in ("Dice", "IoU", "Precision", "Recall", "Accuracy")], d["met"], rtol=1e-12)


@pytest.mark.parametrize("E", [1, 5, 10, 50, 100, 300])
def test_lr_schedule_matches_reference(golden_dir, E):
    ref = np.load(os.path.join(golden_dir, f"lr_cos_E{E}.npy"))
    ours = [ref_cpu.warm_cos_lr(1e-4, 1e-6, E, e) for e in range(E)]
    np.testing.assert_allclose(ours, ref, rtol=1e-12)


def test_adam_trajectory_matches_reference(golden_dir):
    d = np.load(os.path.join(golden_dir, "trajectory_unet_plain.npz"))
    params, buffers = ref_cpu.split_state(make_torch_state(ref_cpu.model_spec("unet_plain", num_classes=2)))
    m1 = {k: torch.zeros_like(v) for k, v in params.items()}
    m2 = {k: torch.zeros_like(v) for k, v in params.items()}
    x, y = torch.from_numpy(d["x"]), torch.from_numpy(d["y"])
    losses = []
    for ep in range(5):
        lr = ref_cpu.warm_cos_lr(1e-4, 1e-6, 5, ep)
        loss, _, grads = ref_cpu.train_step("unet_plain", params, buffers, x, y)
        ref_cpu.adam_step(params, grads, m1, m2, ep + 1, lr)
        losses.append(loss.item())
    np.testing.assert_allclose(losses, d["loss"], rtol=1e-4)
    for k in d.files:
        if k.startswith("final::"):
            np.testing.assert_allclose(params[k[7:]].detach().numpy(), d[k], rtol=1e-4, atol=1e-6)
