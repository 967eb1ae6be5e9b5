"""GPU: FusedAdam(overlap=True) -- Adam + conv-weight re-pack per gradient bucket on the
weight-gradient stream during backward (bench.py's step) -- gives bit-identical parameters, optimizer
moments and next-forward outputs to the plain backward -> step order, over several steps with an lr
change in between.  The element-wise update is the same kernel either way, so any difference is a
race (an update overtaking a read of the old weight or its packed image) or a missed re-pack."""
import pytest
import torch

pytestmark = pytest.mark.gpu
DEV = "cuda"


def _run(name, dt, size, batch, overlap, bucket_mb, steps=4, loss_name="lovasz_hinge"):
    from model.model_factory import build_model
    from unetseg_hip import losses
    from unetseg_hip.arena import FusedAdam
    from utils.synthetic import make_batch

    torch.manual_seed(0)
    kw = dict(num_classes=1) if name == "multitask_unet" else dict(num_classes=2)
    m = build_model(name, **kw).to(DEV).train()
    m.compute_dtype = dt
    opt = FusedAdam(m, lr=1e-3, betas=(0.9, 0.999), weight_decay=1e-4, overlap=overlap, bucket_mb=bucket_mb)
    losses_seen = []
    for it in range(steps):
        x, y, c = make_batch(batch, size, seed=40 + it, with_cls=True)
        x, y, c = x.to(DEV), y.to(DEV), c.to(DEV)
        if it == 2:
            opt.param_groups[0]["lr"] = 3e-4  # set before backward: the overlapped update reads it there
        opt.zero_grad()
        if name == "multitask_unet":
            seg, cls = m(x)  # dropout seeded by the model's step counter: same in both runs
            loss = losses.multitask_loss(seg, cls, y, c, 1.0, loss_name)[0]
        else:
            loss = losses.binary_segmentation_loss(m(x), y, loss_name)
        loss.backward()
        opt.step()
        losses_seen.append(loss.detach().clone())
    x, _ = make_batch(batch, size, seed=99)
    out = m(x.to(DEV))
    out = out[0] if isinstance(out, tuple) else out
    torch.cuda.synchronize()
    return (m._flat.clone(), opt._m.clone(), opt._v.clone(), out.detach().clone(), torch.stack(losses_seen),
            opt._step)


@pytest.mark.parametrize("name,dt,size,batch,bucket_mb", [
    ("unet_resnet50", "bf16", 128, 4, 8.0),
    ("unet_resnet50", "bf16", 128, 2, 1.0),  # many small buckets
    ("unet_resnet50", "fp32", 64, 2, 8.0),
    ("attention_unet", "bf16", 64, 2, 4.0),
    ("multitask_unet", "bf16", 64, 2, 8.0),
    ("unet_plain", "bf16", 64, 2, 2.0),
])
def test_overlapped_adam_matches_step(name, dt, size, batch, bucket_mb):
    a = _run(name, dt, size, batch, False, bucket_mb)
    b = _run(name, dt, size, batch, True, bucket_mb)
    assert a[5] == b[5] == 4
    assert torch.equal(a[4], b[4]), "per-step losses differ"
    for what, u, v in zip(("params", "exp_avg", "exp_avg_sq", "next forward"), a[:4], b[:4]):
        assert torch.equal(u, v), f"{what}: max |diff| {(u.float() - v.float()).abs().max().item():.3e}"


def test_overlap_refuses_grad_scale():
    from model.model_factory import build_model
    from unetseg_hip import losses
    from unetseg_hip.arena import FusedAdam
    from utils.synthetic import make_batch

    m = build_model("unet_plain", num_classes=2).to(DEV).train()
    opt = FusedAdam(m, lr=1e-3, overlap=True)
    x, y = make_batch(2, 64, seed=1)
    losses.binary_segmentation_loss(m(x.to(DEV)), y.to(DEV), "lovasz_hinge").backward()
    with pytest.raises(ValueError):
        opt.step(grad_scale=torch.ones(1, device=DEV))
    with pytest.raises(ValueError):
        FusedAdam(m, overlap=True, capturable=True)


def test_cu_masked_weight_gradient_stream(monkeypatch):
    """UNETSEG_SIDE_CUMASK (ops.side_stream -> unetseg_stream_create_cumask): the weight-gradient
    stream restricted to a quarter of the CUs runs the same kernels in the same order, so the
    overlapped step is bit-identical to the one on an unmasked side stream."""
    from unetseg_hip import ops

    a = _run("unet_resnet50", "bf16", 128, 2, True, 8.0, steps=2)
    monkeypatch.setattr(ops, "SIDE_CUMASK", "11111111")
    monkeypatch.setattr(ops, "_SIDE", {})
    b = _run("unet_resnet50", "bf16", 128, 2, True, 8.0, steps=2)
    assert ops._SIDE and all(isinstance(st, torch.cuda.ExternalStream) for st in ops._SIDE.values())
    for what, u, v in zip(("params", "exp_avg", "exp_avg_sq", "next forward", "losses"), a[:5], b[:5]):
        assert torch.equal(u, v), f"{what} differ with the CU-masked side stream"
