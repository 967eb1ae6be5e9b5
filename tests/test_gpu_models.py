"""GPU: full-model parity of the HIP path against the CPU oracle (oracle/ref_cpu.py) on identical
hash-filled weights and seeded inputs (train-mode forward, loss, backward, BN running stats,
eval-mode forward and confusion counts).

Tolerances: per-pixel logits 1e-3 (absolute) in fp32 mode (BASELINE.json north_star).  Gradients are
judged against the fp64 oracle, relative to the fp32 oracle's own error (the backward is
ill-conditioned at these sizes).  bf16 mode is held to the reference's own CPU-bf16-autocast error
(which is ~0.5 on O(1) logits here, so a fixed 1e-2 bound cannot be met by any bf16 path).
"""
import numpy as np
import pytest
import torch

pytestmark = pytest.mark.gpu
DEV = "cuda"
MODELS = ["unet_plain", "unet_resnet50", "attention_unet", "multitask_unet"]


@pytest.fixture(scope="module", autouse=True)
def _need_gpu():
    if not torch.cuda.is_available():
        pytest.skip("no GPU")


def _kw(name):
    return dict(num_classes=1) if name == "multitask_unet" else dict(num_classes=2)


def _setup(name, S, B, seed):
    from model.model_factory import build_model
    from oracle import ref_cpu
    from oracle.weights import make_torch_state
    from utils.synthetic import make_batch

    state = make_torch_state(ref_cpu.model_spec(name, **_kw(name)))
    m = build_model(name, **_kw(name))
    m.load_state_dict(state)
    m = m.to(DEV).train()
    x, y, c = make_batch(B, S, seed=seed, with_cls=True)
    params, buffers = ref_cpu.split_state(state)
    return m, state, params, buffers, x, y, c


def _rel_l2(a, b):
    a, b = a.double().flatten(), b.double().flatten()
    return float((a - b).norm() / (b.norm() + 1e-30))


def _oracle_grads(name, state, x, y, c, mask, dtype, autocast_bf16=False):
    """oracle forward+loss+backward in `dtype` (fp64 = the exact reference for conditioning)"""
    from oracle import ref_cpu

    p, b = ref_cpu.split_state(state)
    p = {k: v.detach().to(dtype).requires_grad_(True) for k, v in p.items()}
    b = {k: (v.to(dtype) if v.is_floating_point() else v) for k, v in b.items()}
    with torch.autocast("cpu", dtype=torch.bfloat16, enabled=autocast_bf16):
        if name == "multitask_unet":
            seg, cls = ref_cpu.forward(name, p, b, x.to(dtype), True, mask.to(dtype))
            loss, _, _ = ref_cpu.multitask_loss(seg, cls, y, c)
            out = seg
        else:
            out = ref_cpu.forward(name, p, b, x.to(dtype), True)
            loss = ref_cpu.binary_segmentation_loss(out, y, "lovasz_hinge")
    loss.backward()
    return out.detach().double(), loss.item(), {k: v.grad.double() for k, v in p.items()}, b


def _grad_errors(g, ref, scale):
    return {k: float((g[k].double() - ref[k]).norm() / (ref[k].norm() + 1e-4 * scale)) for k in ref}


def _run_hip(m, name, x, y, c, mask):
    from unetseg_hip import losses

    if name == "multitask_unet":
        m.dropout_mask = mask
        seg, cls = m(x.to(DEV))
        loss, _, _ = losses.multitask_loss(seg, cls, y.to(DEV), c.to(DEV), 1.0, "bce")
        out = seg
    else:
        out = m(x.to(DEV))
        loss = losses.binary_segmentation_loss(out, y.to(DEV), "lovasz_hinge")
    loss.backward()
    g = {k: p.grad.detach().cpu().double() for k, p in m.named_parameters()}
    return out.detach().cpu().double(), loss.item(), g


@pytest.mark.parametrize("name", MODELS)
def test_model_fp32_parity(name):
    """fp32 mode: logits within 1e-3 of the fp32 oracle; gradients no further from the fp64 oracle
    than 2x the fp32 oracle's own distance from it.  The backward is ill-conditioned at B=2, 64^2
    (BN over a handful of pixels, lovasz sort order): scaling the input by 1 +- 1e-7 (one ulp) moves
    the fp32 oracle's own median error by ~2x (2.9e-4 -> 5.1e-4 on unet_plain), so the reference
    distance is the largest over the unperturbed and the two one-ulp-perturbed oracle runs --
    otherwise a rounding-level change in any HIP kernel flips the verdict."""
    from oracle import ref_cpu
    from unetseg_hip import losses

    torch.set_num_threads(16)
    m, state, params, buffers, x, y, c = _setup(name, 64, 2, seed=21)
    m.compute_dtype = "fp32"
    mask = (torch.rand(2, 512, generator=torch.Generator().manual_seed(3)) >= 0.5).float()
    out, loss, g = _run_hip(m, name, x, y, c, mask)
    o32, l32, g32, b32 = _oracle_grads(name, state, x, y, c, mask, torch.float32)
    o64, l64, g64, _ = _oracle_grads(name, state, x, y, c, mask, torch.float64)
    err = (out - o32).abs().max().item()
    assert err < 1e-3, err
    assert abs(loss - l32) < 1e-4 * max(1.0, abs(l32)), (loss, l32)
    scale = float(np.median([v.norm().item() for v in g64.values()]))
    e_hip = _grad_errors(g, g64, scale)
    e_runs = [_grad_errors(g32, g64, scale)]
    for d in (1e-7, -1e-7):
        e_runs.append(_grad_errors(_oracle_grads(name, state, x * (1 + d), y, c, mask, torch.float32)[2], g64, scale))
    med_h = np.median(list(e_hip.values()))
    med_c = max(np.median(list(e.values())) for e in e_runs)
    assert med_h <= 2.0 * med_c + 1e-4, (med_h, med_c)
    worst, worst_c = max(e_hip.values()), max(max(e.values()) for e in e_runs)
    assert worst <= 3.0 * worst_c + 1e-3, (worst, worst_c)
    msd = m.state_dict()
    for k, v in b32.items():
        if k.endswith("running_mean") or k.endswith("running_var"):
            np.testing.assert_allclose(msd[k].cpu().numpy(), v.numpy(), rtol=1e-4, atol=1e-5, err_msg=k)
        if k.endswith("num_batches_tracked"):
            assert int(msd[k]) == int(v), k


@pytest.mark.parametrize("name", MODELS)
def test_model_eval_fp32_and_confusion(name):
    """eval mode (running statistics) on the same hash weights/buffers: logits within 1e-3 and the
    confusion counts equal except for pixels whose class margin is below the fp32 tolerance."""
    from oracle import ref_cpu
    from unetseg_hip import losses

    torch.set_num_threads(16)
    m, state, params, buffers, x, y, c = _setup(name, 64, 2, seed=23)
    m.compute_dtype = "fp32"
    m.eval()
    with torch.no_grad():
        o = m(x.to(DEV))
        ro = ref_cpu.forward(name, params, buffers, x, train=False)
    if name == "multitask_unet":
        o, ro = o[0], ro[0]
    assert (o.cpu() - ro).abs().max() < 1e-3
    if name != "multitask_unet":
        conf = losses.binary_confusion(o, y.to(DEV)).cpu().tolist()
        rconf = list(ref_cpu.binary_confusion(ro, y))
        nflip = int(((ro[:, 1] - ro[:, 0]).abs() < 1e-4).sum())
        assert sum(abs(a - b) for a, b in zip(conf, rconf)) <= 2 * nflip, (conf, rconf)


@pytest.mark.parametrize("name", MODELS)
def test_model_bf16_parity(name):
    """bf16 mode: the HIP path's distance from the fp32 oracle is no larger than the reference's
    own CPU-bf16-autocast distance (logits: max and mean; gradients: median relative L2)."""
    torch.set_num_threads(16)
    m, state, params, buffers, x, y, c = _setup(name, 64, 2, seed=22)
    m.compute_dtype = "bf16"
    mask = (torch.rand(2, 512, generator=torch.Generator().manual_seed(4)) >= 0.5).float()
    out, loss, g = _run_hip(m, name, x, y, c, mask)
    o32, l32, g32, _ = _oracle_grads(name, state, x, y, c, mask, torch.float32)
    obf, lbf, gbf, _ = _oracle_grads(name, state, x, y, c, mask, torch.float32, autocast_bf16=True)
    e_hip, e_ref = (out - o32).abs(), (obf - o32).abs()
    assert e_hip.max() <= 1.5 * e_ref.max() + 1e-2, (e_hip.max().item(), e_ref.max().item())
    assert e_hip.mean() <= 1.5 * e_ref.mean() + 1e-3, (e_hip.mean().item(), e_ref.mean().item())
    assert abs(loss - l32) <= 2 * abs(lbf - l32) + 1e-2 * abs(l32), (loss, lbf, l32)
    scale = float(np.median([v.norm().item() for v in g32.values()]))
    eh = np.median(list(_grad_errors(g, g32, scale).values()))
    er = np.median(list(_grad_errors(gbf, g32, scale).values()))
    assert eh <= 2.0 * er + 1e-3, (eh, er)


def test_train_steps_trajectory_matches_reference(golden_dir):
    """5 Adam steps (fp32 mode) vs the reference's own loss trajectory (tests/golden)."""
    import os

    from model.unet_training import get_lr_scheduler, set_optimizer_lr
    from oracle import ref_cpu
    from oracle.weights import make_torch_state
    from unetseg_hip.arena import FusedAdam
    from unetseg_hip.losses import binary_segmentation_loss
    from model.model_factory import build_model

    d = np.load(os.path.join(golden_dir, "trajectory_unet_plain.npz"))
    m = build_model("unet_plain", num_classes=2)
    m.load_state_dict(make_torch_state(ref_cpu.model_spec("unet_plain", num_classes=2)))
    m = m.to(DEV).train()
    m.compute_dtype = "fp32"
    opt = FusedAdam(m, 1e-4, betas=(0.9, 0.999), weight_decay=1e-4)
    sched = get_lr_scheduler("cos", 1e-4, 1e-6, 5)
    x, y = torch.from_numpy(d["x"]).to(DEV), torch.from_numpy(d["y"]).to(DEV)
    traj = []
    for ep in range(5):
        set_optimizer_lr(opt, sched, ep)
        opt.zero_grad()
        loss = binary_segmentation_loss(m(x), y, "lovasz_hinge")
        loss.backward()
        opt.step()
        traj.append(loss.item())
    np.testing.assert_allclose(traj, d["loss"], rtol=5e-3)  # ill-conditioned at B=2
    sd = m.state_dict()
    for k in d.files:
        if k.startswith("final::"):
            np.testing.assert_allclose(sd[k[7:]].cpu().numpy(), d[k], rtol=1e-3, atol=2e-4)  # Adam moves <= 5*lr
