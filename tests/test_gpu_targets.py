"""GPU: target handling at the loss boundary.

* the multitask classification CE follows nn.CrossEntropyLoss() (model/unet_multitask.py:116,134):
  targets of -100 are ignored (mean over the others, zero gradient rows); any other class outside
  [0, K) gives a NaN loss and gradient instead of an out-of-range read;
* float segmentation targets (MultiTaskLoss passes seg_targets.float(), unet_multitask.py:131) are
  accepted when they are 0/1 and refused otherwise (the kernels take 0/1 labels; BCE would take soft
  labels as given).
"""
import pytest
import torch
import torch.nn.functional as F

pytestmark = pytest.mark.gpu
DEV = "cuda"


def _mt(cls_t, seg_t=None):
    from unetseg_hip.losses import multitask_loss
    g = torch.Generator(device=DEV).manual_seed(3)
    seg = torch.randn(4, 1, 8, 8, generator=g, device=DEV, requires_grad=True)
    cls = torch.randn(4, 3, generator=g, device=DEV, requires_grad=True)
    if seg_t is None:
        seg_t = (torch.rand(4, 8, 8, generator=g, device=DEV) > 0.5).long()
    total, sl, cl = multitask_loss(seg, cls, seg_t, cls_t)
    total.backward()
    return seg, cls, seg_t, sl, cl


def test_ce_ignore_index():
    t = torch.tensor([0, -100, 2, 1], device=DEV)
    seg, cls, seg_t, sl, cl = _mt(t)
    c = cls.detach().clone().requires_grad_(True)
    ref = F.cross_entropy(c, t)
    ref.backward()
    torch.testing.assert_close(cl, ref.detach(), rtol=1e-6, atol=1e-6)
    torch.testing.assert_close(cls.grad, c.grad, rtol=1e-5, atol=1e-7)
    assert (cls.grad[1] == 0).all()


def test_ce_out_of_range_is_nan():
    seg, cls, seg_t, sl, cl = _mt(torch.tensor([0, 3, 2, 1], device=DEV))
    assert torch.isnan(cl).item() and torch.isnan(cls.grad).all().item()
    assert torch.isfinite(sl).item()


def test_float_seg_targets():
    g = torch.Generator(device=DEV).manual_seed(4)
    t01 = (torch.rand(4, 8, 8, generator=g, device=DEV) > 0.5).float()
    ct = torch.tensor([0, 1, 2, 1], device=DEV)
    _, _, _, sl_f, _ = _mt(ct, t01)
    _, _, _, sl_i, _ = _mt(ct, t01.long())
    torch.testing.assert_close(sl_f, sl_i)
    with pytest.raises(ValueError, match="0/1"):
        _mt(ct, t01 * 0.7)
