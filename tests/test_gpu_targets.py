"""GPU: target handling at the loss boundary.

* the multitask classification CE follows nn.CrossEntropyLoss() (model/unet_multitask.py:116,134):
  targets of -100 are ignored (mean over the others, zero gradient rows); any other class outside
  [0, K) gives a NaN loss and gradient instead of an out-of-range read;
* float segmentation targets (MultiTaskLoss passes seg_targets.float(), unet_multitask.py:131) are
  accepted when they are 0/1; a soft label (BCE would take it as given, the kernels take 0/1 labels)
  turns the seg loss and its gradient into NaN on the device -- no host sync -- and
  is reported as a ValueError by the multitask loops' once-per-epoch read;
* binary_segmentation_loss reads float targets as (targets == 1), the reference's own mapping
  (utils/train_and_eval.py:163);
* the multiclass CE / Focal treat a target outside [0, C) other than ignore_index the way
  nn.CrossEntropyLoss refuses it: NaN loss and gradient.
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
    from unetseg_hip.losses import raise_if_soft_targets
    raise_if_soft_targets(DEV)  # 0/1 float targets: nothing flagged
    seg, _, _, sl, cl = _mt(ct, t01 * 0.7)
    assert torch.isnan(sl).item() and torch.isnan(seg.grad).all().item() and torch.isfinite(cl).item()
    with pytest.raises(ValueError, match="seg targets must be 0 or 1"):
        raise_if_soft_targets(DEV)
    raise_if_soft_targets(DEV)  # the flag is cleared by the report


def test_soft_seg_target_two_reported_by_loop():
    """a float target of 2 in the multitask loop raises at the epoch's end instead of
    leaving a silent NaN loss (model/unet_multitask.py:131 feeds seg_targets.float() to BCE)"""
    from model.model_factory import build_model
    from model.unet_multitask import MultiTaskLoss
    from unetseg_hip.arena import FusedAdam
    from utils.train_and_eval import train_one_epoch_multitask
    torch.manual_seed(0)
    m = build_model("multitask_unet", 1).to(DEV)
    opt = FusedAdam(m, lr=1e-4)
    x = torch.rand(2, 3, 64, 64, device=DEV)
    seg_t = torch.zeros(2, 64, 64, device=DEV)
    seg_t[:, 10:20, 10:20] = 2.0
    loader = [(x, seg_t, None, torch.tensor([0, 2], device=DEV))]
    with pytest.raises(ValueError, match="seg targets must be 0 or 1"):
        train_one_epoch_multitask(m, opt, loader, torch.device(DEV), MultiTaskLoss(), None, amp=True)


def test_binary_loss_float_targets_as_reference():
    from unetseg_hip.losses import binary_segmentation_loss
    g = torch.Generator(device=DEV).manual_seed(5)
    out = torch.randn(2, 2, 16, 16, generator=g, device=DEV)
    t = torch.randint(0, 3, (2, 16, 16), generator=g, device=DEV).float() * 0.75  # 0, 0.75, 1.5: only ==1 is fg
    t[0, :4] = 1.0
    for kind in ("bce", "lovasz_hinge"):
        a = binary_segmentation_loss(out, t, kind)
        b = binary_segmentation_loss(out, (t == 1).long(), kind)
        torch.testing.assert_close(a, b, rtol=0, atol=0)


@pytest.mark.parametrize("fn", ["ce", "focal"])
def test_multiclass_out_of_range_target_is_nan(fn):
    from model.unet_training import CE_Loss, Focal_Loss
    g = torch.Generator(device=DEV).manual_seed(6)
    x = torch.randn(2, 4, 8, 8, generator=g, device=DEV, requires_grad=True)
    t = torch.randint(0, 4, (2, 8, 8), generator=g, device=DEV)
    w = torch.ones(4, device=DEV)
    f = CE_Loss if fn == "ce" else Focal_Loss
    ok = f(x, t, w, num_classes=4)           # ignore_index = num_classes = 4: fine
    t2 = t.clone()
    t2[0, 0, 0] = 4                           # the ignore label
    assert torch.isfinite(f(x, t2, w, num_classes=4)).item()
    t2[1, 2, 3] = 7                           # neither a class nor the ignore label
    bad = f(x, t2, w, num_classes=4)
    bad.backward()
    assert torch.isfinite(ok).item() and torch.isnan(bad).item() and torch.isnan(x.grad).all().item()
