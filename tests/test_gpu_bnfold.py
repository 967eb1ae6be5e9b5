"""GPU: eval-mode BatchNorm folding (ops.conv_bn: in fp32 the BN scale and shift are applied to the
conv's accumulator in its epilogue, with ReLU) against the unfolded eval path (conv, then the
BN-apply pass with running statistics) -- bit-identical in fp32 -- and against the CPU oracle's
eval forward; bf16 eval keeps the unfolded path.

Reference semantics: model.eval() BatchNorm2d uses running_mean / running_var
(model/resnet_backbone.py:64-70, model/unet_plain.py:8-15, model/unet_dualdense.py:36-47)."""
import numpy as np
import pytest
import torch

pytestmark = pytest.mark.gpu
DEV = "cuda"


@pytest.mark.parametrize("name,size", [("unet_resnet50", 64), ("unet_plain", 48), ("dualdense_unet", 32),
                                       ("attention_unet", 32)])
@pytest.mark.parametrize("dtype", ["fp32", "bf16"])
def test_folded_eval_matches_unfolded(name, size, dtype, monkeypatch):
    from model.model_factory import build_model
    from oracle import ref_cpu
    from oracle.weights import make_torch_state
    from unetseg_hip import ops

    state = make_torch_state(ref_cpu.model_spec(name, num_classes=2))
    g = torch.Generator().manual_seed(3)
    for k in list(state):  # non-trivial running statistics
        if k.endswith("running_mean"):
            state[k] = 0.1 * torch.randn(state[k].shape, generator=g)
        elif k.endswith("running_var"):
            state[k] = 0.5 + torch.rand(state[k].shape, generator=g)
    m = build_model(name, num_classes=2)
    m.load_state_dict(state)
    m = m.to(DEV).eval()
    m.compute_dtype = dtype
    x = torch.rand(2, 3, size, size, generator=g)
    with torch.no_grad():
        monkeypatch.setattr(ops, "BN_FOLD", True)
        folded = m(x.to(DEV)).float().cpu()
        monkeypatch.setattr(ops, "BN_FOLD", False)
        plain = m(x.to(DEV)).float().cpu()
    params, buffers = ref_cpu.split_state(state)
    with torch.no_grad():
        ref = ref_cpu.forward(name, params, buffers, x, train=False)
    scale = ref.abs().max().item() + 1e-6
    assert torch.equal(folded, plain)  # same float arithmetic (fp32), or the same path (bf16)
    if dtype == "fp32":
        np.testing.assert_allclose(folded.numpy(), ref.numpy(), rtol=1e-3, atol=1e-3 * scale)


@pytest.mark.parametrize("name", ["unet_resnet50", "multitask_unet"])
def test_bn_prologue_train_step_matches_unfused(name, monkeypatch):
    """Training with bn2-ReLU applied inside the bottleneck conv3 (ops.bn(lazy=True)) gives the same
    forward, loss and every parameter gradient as materialising the activation first: the prologue
    stages the same bf16 values the bn_apply pass would store."""
    from model.model_factory import build_model
    from oracle import ref_cpu
    from oracle.weights import make_torch_state
    from unetseg_hip import ops

    kw = dict(num_classes=1, num_seg_classes=1, num_cls_classes=3) if name == "multitask_unet" else dict(num_classes=2)
    state = make_torch_state(ref_cpu.model_spec(name, **kw))
    g = torch.Generator().manual_seed(5)
    x = torch.rand(2, 3, 64, 64, generator=g).to(DEV)
    outs = []
    for on in (True, False):
        monkeypatch.setattr(ops, "BN_PROLOGUE", on)
        m = build_model(name, **kw)
        m.load_state_dict(state)
        m = m.to(DEV).train()
        m.compute_dtype = "bf16"
        o = m(x)
        o = o[0] if isinstance(o, tuple) else o
        (o.float() ** 2).mean().backward()
        torch.cuda.synchronize()
        outs.append((o.detach().float().cpu(), {n: p.grad.detach().cpu().clone() for n, p in m.named_parameters()}))
    (o1, g1), (o2, g2) = outs
    assert torch.equal(o1, o2)
    for n in g1:
        torch.testing.assert_close(g1[n], g2[n], rtol=1e-5, atol=1e-7, msg=n)
