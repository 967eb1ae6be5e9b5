"""Fused HIP loss / metric kernels behind autograd Functions.

binary_segmentation_loss(outputs [B,2,H,W] fp32, targets [B,H,W]) -> scalar, with the 2-class ->
logit difference (utils/train_and_eval.py:106-113) fused into the kernel:
  * "lovasz_hinge": per-image stable radix sort + Jaccard-gradient scan (model/unet_training.py:219-280)
  * "bce": BCE-with-logits mean, optional scalar pos_weight (model/unet_training.py:205-216)
multitask_loss: seg BCE/Lovasz + w * CE over the cls head (model/unet_multitask.py:119-139).
"""
from __future__ import annotations

import torch

from .lib import lib
from .ops import P, workspace


def _stream(dev):
    return torch.cuda.current_stream(dev).cuda_stream


def _prep(outputs, targets, ignore_index=None):
    """-> (fp32 outputs, int64 targets, soft): float targets are mapped the way the reference reads
    them, (targets == 1) (utils/train_and_eval.py:163, binary_segmentation_loss; ignore_index kept);
    `soft` is a device bool, True when some float target is neither 0 nor 1 -- MultiTaskLoss
    (model/unet_multitask.py:131) feeds seg_targets.float() straight to BCE, where such a soft label
    would count as given and the 0/1 kernels cannot represent it: that loss is poisoned to NaN on the
    device (_poison) instead of a host check, so no call syncs the stream."""
    if not outputs.is_cuda:
        raise RuntimeError("HIP losses need device tensors")
    out = outputs.detach().float().contiguous()
    soft = None
    t = targets.detach()
    if t.is_floating_point():
        soft = ((t != 0) & (t != 1)).any()
        tgt = (t == 1).to(torch.int64)
        if ignore_index is not None:
            tgt = torch.where(t == ignore_index, torch.full_like(tgt, int(ignore_index)), tgt)
        return out, tgt.contiguous(), soft
    return out, t.to(torch.int64).contiguous(), soft


def _poison(soft, *ts):
    """NaN-fill ts in place where `soft` (device bool) is set (no host sync), and remember it in the
    device's soft-label flag (raise_if_soft_targets reads it once per epoch / evaluation)"""
    if soft is not None:
        for t in ts:
            if t is not None:
                t.masked_fill_(soft, float("nan"))
        flag = _SOFT_SEEN.get(soft.device)
        if flag is None:
            flag = _SOFT_SEEN[soft.device] = torch.zeros((), dtype=torch.bool, device=soft.device)
        flag.logical_or_(soft)


#: per device: a MultiTaskLoss BCE call has seen a seg target that is neither 0 nor 1 since the last check
_SOFT_SEEN = {}


def raise_if_soft_targets(device=None):
    """ValueError if a MultiTaskLoss BCE call saw a seg target other than 0 / 1 since the last call
    (one host read; the loss itself was NaN-poisoned on the device).  The reference's
    BCEWithLogitsLoss would train on such soft labels (model/unet_multitask.py:131); the fused
    0/1 kernels cannot, so the data error is reported instead of training on NaN silently.  The
    multitask train / eval loops call this once per epoch / evaluation.  Under data parallelism the
    flag is all-reduced (MAX) first, so every rank raises together instead of the others blocking in
    the next collective (every rank must call this, as the loops do)."""
    import torch.distributed as dist

    dp = dist.is_available() and dist.is_initialized() and dist.get_world_size() > 1
    if device is not None:
        devs = [torch.device(device)]
    elif dp:  # exactly one collective per call on every rank: this rank's device
        devs = [torch.device("cuda", torch.cuda.current_device()) if torch.cuda.is_available() else torch.device("cpu")]
    else:
        devs = list(_SOFT_SEEN)
    for d in devs:
        if d.type == "cuda" and d.index is None:
            d = torch.device("cuda", torch.cuda.current_device())
        flag = _SOFT_SEEN.get(d)
        seen = flag is not None and bool(flag.item())
        if dp:
            on_dev = dist.get_backend() == "nccl"
            t = torch.tensor([int(seen)], dtype=torch.int32, device=d if on_dev else "cpu")
            dist.all_reduce(t, op=dist.ReduceOp.MAX)
            seen = bool(t.item())
        if seen:
            if flag is not None:
                flag.zero_()
            raise ValueError("MultiTaskLoss: seg targets must be 0 or 1 (the fused BCE kernel takes binary "
                             "labels; a soft / out-of-range target was seen and the loss was set to NaN)")


def _seg_forward(kind, out, nch, tgt, B, Pn, pos_weight, need_grad, ignore_index=None):
    dev = out.device
    st = _stream(dev)
    loss = torch.empty((), dtype=torch.float32, device=dev)
    gz = (torch.empty((B, Pn), dtype=torch.float32, device=dev)
          if (need_grad or kind in ("lovasz_hinge", "lovasz_image_masked")) else None)
    if ignore_index is not None and kind != "lovasz_image_masked":
        if kind not in ("bce", "lovasz_hinge"):
            raise ValueError(f"Unsupported loss_name: {kind}")
        if gz is None:
            gz = torch.empty((B, Pn), dtype=torch.float32, device=dev)
        pw = None
        if pos_weight is not None and kind == "bce":
            pw = torch.as_tensor(pos_weight, dtype=torch.float32, device=dev).reshape(-1)[:1].contiguous()
        nb = lib.masked_loss_workspace(B, Pn)
        ws = workspace(nb, dev)
        lib.masked_loss_fwd(P(out), nch, P(tgt), B, Pn, int(ignore_index), 0 if kind == "bce" else 1, P(pw), P(ws),
                            ws.numel(), P(gz), P(loss), st)
    elif kind == "lovasz_hinge":
        nb = lib.lovasz_workspace(B, Pn)
        ws = workspace(nb, dev)
        lib.lovasz_fwd(P(out), nch, P(tgt), B, Pn, P(ws), ws.numel(), P(gz), P(loss), st)
    elif kind == "lovasz_image_masked":  # lovasz_hinge_loss(..., ignore_index): per image, valid pixels
        nb = lib.lovasz_workspace(B, Pn)
        ws = workspace(nb, dev)
        lib.lovasz_fwd_masked(P(out), nch, P(tgt), B, Pn, int(ignore_index), P(ws), ws.numel(), P(gz), P(loss), st)
    elif kind == "bce":
        pw = None
        if pos_weight is not None:
            pw = torch.as_tensor(pos_weight, dtype=torch.float32, device=dev).reshape(-1)[:1].contiguous()
        nb = lib.bce_workspace(B, Pn)
        ws = workspace(nb, dev)
        lib.bce_fwd(P(out), nch, P(tgt), B, Pn, P(pw), P(ws), ws.numel(), P(gz), P(loss), st)
    else:
        raise ValueError(f"Unsupported loss_name: {kind}")
    return loss, gz


class _SegLossFn(torch.autograd.Function):
    @staticmethod
    def forward(fctx, outputs, targets, kind, pos_weight, ignore_index=None):
        out, tgt, _ = _prep(outputs, targets, ignore_index)
        B, nch = out.shape[0], out.shape[1]
        Pn = out[0, 0].numel()
        loss, gz = _seg_forward(kind, out, nch, tgt, B, Pn, pos_weight, outputs.requires_grad, ignore_index)
        fctx.save_for_backward(gz)
        fctx.meta = (B, nch, Pn, outputs.shape, outputs.dtype)
        return loss

    @staticmethod
    def backward(fctx, g):
        (gz,) = fctx.saved_tensors
        B, nch, Pn, shape, dtype = fctx.meta
        g = g.detach().float().reshape(1).contiguous()
        dout = torch.empty(shape, dtype=torch.float32, device=gz.device)
        scratch = torch.empty_like(gz)
        lib.dz_to_dout(P(gz), B, Pn, nch, P(g), 1.0, 0, 0.0, P(scratch), P(dout), _stream(gz.device))
        return dout.to(dtype), None, None, None, None


def binary_segmentation_loss(outputs, targets, loss_name, pos_weight=None, ignore_index=None):
    """utils/train_and_eval.py:155-182 on the HIP path.  With ignore_index the valid pixels are
    flattened across the batch (BCE: their mean; Lovasz: see unetseg_masked_loss_fwd)."""
    if outputs.dim() != 4 or outputs.size(1) != 2:
        raise ValueError(f"Expected output shape (N,2,H,W), got {tuple(outputs.shape)}")
    if loss_name not in ("bce", "lovasz_hinge"):
        raise ValueError(f"Unsupported loss_name: {loss_name}")
    return _SegLossFn.apply(outputs, targets, loss_name, pos_weight, ignore_index)


def seg_loss_1ch(logits, targets, kind):
    """loss on [B,1,H,W] (or [B,H,W]) logits, e.g. MultiTaskLoss's seg term"""
    if logits.dim() == 3:
        logits = logits.unsqueeze(1)
    return _SegLossFn.apply(logits, targets, kind, None)


class _MultiTaskFn(torch.autograd.Function):
    @staticmethod
    def forward(fctx, seg, cls, seg_t, cls_t, w, kind):
        out, tgt, soft = _prep(seg, seg_t)
        B = out.shape[0]
        Pn = out[0].numel()
        dev = out.device
        seg_loss, gz = _seg_forward(kind, out, 1, tgt, B, Pn, None, True)
        if kind == "bce":
            _poison(soft, seg_loss, gz)
        c = cls.detach().float().contiguous()
        ct = cls_t.detach().to(device=dev, dtype=torch.int64).contiguous()
        cls_loss = torch.empty((), dtype=torch.float32, device=dev)
        dlog = torch.empty_like(c)
        lib.ce_fwd(P(c), P(ct), c.shape[0], c.shape[1], P(cls_loss), P(dlog), _stream(dev))
        total = torch.empty((), dtype=torch.float32, device=dev)
        # total = 1 * (seg + w * cls)  (device scalars, no host sync)
        one = torch.ones(1, dtype=torch.float32, device=dev)
        lib.scale_grad(P(one), 1, P(seg_loss), 1.0, P(cls_loss), float(w), P(total), _stream(dev))
        fctx.save_for_backward(gz, dlog)
        fctx.meta = (B, Pn, seg.shape, float(w))
        return total, seg_loss, cls_loss

    @staticmethod
    def backward(fctx, g_total, g_seg, g_cls):
        gz, dlog = fctx.saved_tensors
        B, Pn, shape, w = fctx.meta
        dev = gz.device
        st = _stream(dev)
        zero = torch.zeros(1, dtype=torch.float32, device=dev)
        gt = g_total.float().reshape(1).contiguous() if g_total is not None else zero
        gs = g_seg.float().reshape(1).contiguous() if g_seg is not None else zero
        gc = g_cls.float().reshape(1).contiguous() if g_cls is not None else zero
        dseg = torch.empty(shape, dtype=torch.float32, device=dev)
        scratch = torch.empty_like(gz)
        # d seg = gz * (g_total + g_seg)
        tmp = torch.empty(1, dtype=torch.float32, device=dev)
        one = torch.ones(1, dtype=torch.float32, device=dev)
        lib.scale_grad(P(one), 1, P(gt), 1.0, P(gs), 1.0, P(tmp), st)
        lib.dz_to_dout(P(gz), B, Pn, 1, P(tmp), 1.0, 0, 0.0, P(scratch), P(dseg), st)
        dcls = torch.empty_like(dlog)
        lib.scale_grad(P(dlog), dlog.numel(), P(gt), w, P(gc), 1.0, P(dcls), st)
        return dseg, dcls, None, None, None, None


def multitask_loss(seg_logits, cls_logits, seg_targets, cls_targets, cls_loss_weight=1.0, kind="bce"):
    return _MultiTaskFn.apply(seg_logits, cls_logits, seg_targets, cls_targets, cls_loss_weight, kind)


def binary_confusion(outputs, targets, conf=None, ignore_index=None):
    """device uint64[4] (+)= (tp, fp, fn, tn).  outputs [B,2,H,W] (argmax, tie -> 0) or [B,1,H,W]
    (sigmoid > 0.5); pixels whose target is ignore_index are skipped.  No host sync: callers read
    the counters once per split."""
    out, tgt, _ = _prep(outputs, targets, ignore_index)
    B, nch = out.shape[0], out.shape[1]
    Pn = out[0, 0].numel()
    if conf is None:
        conf = torch.zeros(4, dtype=torch.int64, device=out.device)
    if ignore_index is None:
        lib.confusion(P(out), nch, P(tgt), B, Pn, P(conf), _stream(out.device))
    else:
        lib.confusion_masked(P(out), nch, P(tgt), B, Pn, int(ignore_index), P(conf), _stream(out.device))
    return conf


# ------------------------------------------------------------------------------------------------
# multiclass task (model/unet_training.py:9-91, utils/train_and_eval.py:20-103)
# ------------------------------------------------------------------------------------------------
MC_CE, MC_FOCAL, MC_NONE = 0, 1, 2


class _McLossFn(torch.autograd.Function):
    """One fused kernel pair (unetseg_mc_loss_fwd / _bwd): CE or Focal over argmax targets and/or
    Dice over a one-hot target, on fp32 planar logits [B][C][H][W]."""

    @staticmethod
    def forward(fctx, outputs, target, cls_w, kind, alpha, gamma, dice_t, beta, smooth, ignore_index):
        if not outputs.is_cuda:
            raise RuntimeError("HIP losses need device tensors")
        out = outputs.detach().float().contiguous()
        B, C = out.shape[0], out.shape[1]
        Pn = out[0, 0].numel()
        dev = out.device
        tgt = target.detach().to(device=dev, dtype=torch.int64).contiguous() if target is not None else None
        w = cls_w.detach().to(device=dev, dtype=torch.float32).contiguous() if cls_w is not None else None
        dt = dice_t.detach().to(device=dev, dtype=torch.float32).contiguous() if dice_t is not None else None
        ct = dt.shape[-1] if dt is not None else 0
        nb = lib.mc_loss_workspace(B, C, Pn)
        ws = torch.empty(nb, dtype=torch.uint8, device=dev)
        loss = torch.empty(3, dtype=torch.float32, device=dev)
        args = (P(out), P(tgt), B, C, Pn, P(w), int(ignore_index), int(kind), float(alpha), float(gamma), P(dt), ct,
                float(beta), float(smooth))
        lib.mc_loss_fwd(*args, P(ws), nb, P(loss), _stream(dev))
        fctx.keep = (out, tgt, w, dt, ws, args, outputs.shape, outputs.dtype)
        return loss[0]

    @staticmethod
    def backward(fctx, g):
        out, tgt, w, dt, ws, args, shape, dtype = fctx.keep
        g = g.detach().float().reshape(1).contiguous()
        dout = torch.empty(shape, dtype=torch.float32, device=out.device)
        lib.mc_loss_bwd(*args, P(ws), P(g), P(dout), _stream(out.device))
        fctx.keep = None
        return dout.to(dtype), None, None, None, None, None, None, None, None, None


def _check_mc(inputs, target_hw):
    n, c, h, w = inputs.size()
    ht, wt = target_hw
    if h != ht and w != wt:
        # the reference interpolates the logits (align_corners=True) to the label size first
        inputs = _ResizeLogitsFn.apply(inputs, int(ht), int(wt), True)
    return inputs


class _ResizeLogitsFn(torch.autograd.Function):
    """F.interpolate(bilinear) of fp32 planar logits [N][C][H][W] on the HIP resize kernels (the
    planes are N*C single-channel NHWC images)"""

    @staticmethod
    def forward(fctx, x, oh, ow, align):
        from .lib import DT_F32
        xc = x.detach().float().contiguous()
        N, C, H, W = xc.shape
        y = torch.empty((N, C, oh, ow), dtype=torch.float32, device=xc.device)
        lib.resize_bilinear_fwd(DT_F32, P(xc), 1, N * C, H, W, 1, oh, ow, int(align), P(y), 1, _stream(xc.device))
        fctx.meta = (N, C, H, W, oh, ow, align)
        return y

    @staticmethod
    def backward(fctx, g):
        from .lib import DT_F32
        N, C, H, W, oh, ow, align = fctx.meta
        gc = g.detach().float().contiguous()
        dx = torch.empty((N, C, H, W), dtype=torch.float32, device=gc.device)
        lib.resize_bilinear_bwd(DT_F32, P(gc), 1, N * C, H, W, 1, oh, ow, int(align), P(dx), 1, 0, _stream(gc.device))
        return dx, None, None, None


def ce_loss(inputs, target, cls_weights, num_classes=21):
    """CE_Loss (model/unet_training.py:9-24): weighted mean cross entropy, ignore_index=num_classes"""
    inputs = _check_mc(inputs, target.shape[-2:])
    return _McLossFn.apply(inputs, target, cls_weights, MC_CE, -1.0, 0.0, None, 1.0, 0.0, num_classes)


def focal_loss(inputs, target, cls_weights, num_classes=21, alpha=0.5, gamma=2):
    """Focal_Loss (model/unet_training.py:32-59): -(1-pt)^gamma * alpha * log pt, mean over all pixels"""
    inputs = _check_mc(inputs, target.shape[-2:])
    return _McLossFn.apply(inputs, target, cls_weights, MC_FOCAL, -1.0 if alpha is None else alpha, gamma, None, 1.0,
                           0.0, num_classes)


def dice_loss(inputs, target, beta=1, smooth=1e-5):
    """Dice_loss (model/unet_training.py:67-91) on a one-hot target [N,H,W,ct] (first C channels)"""
    inputs = _check_mc(inputs, target.shape[1:3])
    return _McLossFn.apply(inputs, None, None, MC_NONE, -1.0, 0.0, target, beta, smooth, -1)


def mc_confusion(outputs, target, hist=None):
    """device u64 [(C+1), C] (+)= (target class, argmax class); targets outside [0, C) -> row C"""
    out = outputs.detach().float().contiguous()
    B, C = out.shape[0], out.shape[1]
    tgt = target.detach().to(device=out.device, dtype=torch.int64).contiguous()
    if hist is None:
        hist = torch.zeros(C + 1, C, dtype=torch.int64, device=out.device)
    lib.mc_confusion(P(out), P(tgt), B, C, out[0, 0].numel(), P(hist), _stream(out.device))
    return hist


def mc_metrics_from_hist(hist):
    """pixel_accuracy / mean_accuracy / mean_iou / frequency_weighted_iou of utils/train_and_eval.py:20-103
    from one batch's histogram (host, float64; classes absent from the target are skipped as there)"""
    import numpy as np
    h = np.asarray(hist, dtype=np.float64)
    C = h.shape[1]
    total = h.sum()
    inter = np.array([h[i, i] for i in range(C)])
    tcount = h[:C].sum(1)
    pcount = h.sum(0)
    union = tcount + pcount - inter
    pixel_acc = float(inter.sum() / total) if total > 0 else 0.0
    present = tcount > 0
    accs = [inter[i] / tcount[i] for i in range(C) if present[i]]
    mean_acc = float(sum(accs) / len(accs)) if accs else 0.0
    ious = [(inter[i] / union[i]) if union[i] > 0 else 0.0 for i in range(C) if present[i]]
    miou = float(sum(ious) / len(ious)) if ious else 0.0
    iou_all = [(inter[i] / union[i]) if union[i] > 0 else 0.0 for i in range(C)]
    ft = tcount.sum()
    fw = float(sum(f * i for f, i in zip(tcount, iou_all)) / ft) if ft > 0 else 0.0
    return {"Pixel Accuracy": pixel_acc, "Mean Accuracy": mean_acc, "Mean IoU": miou, "Frequency Weighted IoU": fw}
