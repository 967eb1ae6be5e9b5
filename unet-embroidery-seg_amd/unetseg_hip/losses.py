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


def _prep(outputs, targets):
    if not outputs.is_cuda:
        raise RuntimeError("HIP losses need device tensors")
    out = outputs.detach().float().contiguous()
    tgt = targets.detach().to(torch.int64).contiguous()
    return out, tgt


def _seg_forward(kind, out, nch, tgt, B, Pn, pos_weight, need_grad):
    dev = out.device
    st = _stream(dev)
    loss = torch.empty((), dtype=torch.float32, device=dev)
    gz = torch.empty((B, Pn), dtype=torch.float32, device=dev) if (need_grad or kind == "lovasz_hinge") else None
    if kind == "lovasz_hinge":
        nb = lib.lovasz_workspace(B, Pn)
        ws = workspace(nb, dev)
        lib.lovasz_fwd(P(out), nch, P(tgt), B, Pn, P(ws), ws.numel(), P(gz), P(loss), st)
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
    def forward(fctx, outputs, targets, kind, pos_weight):
        out, tgt = _prep(outputs, targets)
        B, nch = out.shape[0], out.shape[1]
        Pn = out[0, 0].numel()
        loss, gz = _seg_forward(kind, out, nch, tgt, B, Pn, pos_weight, outputs.requires_grad)
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
        return dout.to(dtype), None, None, None


def binary_segmentation_loss(outputs, targets, loss_name, pos_weight=None, ignore_index=None):
    """utils/train_and_eval.py:155-182 on the HIP path (ignore_index must be None)."""
    if outputs.dim() != 4 or outputs.size(1) != 2:
        raise ValueError(f"Expected output shape (N,2,H,W), got {tuple(outputs.shape)}")
    if ignore_index is not None:
        raise NotImplementedError("ignore_index is not on the hot path (train.py always passes None)")
    if loss_name not in ("bce", "lovasz_hinge"):
        raise ValueError(f"Unsupported loss_name: {loss_name}")
    return _SegLossFn.apply(outputs, targets, loss_name, pos_weight)


def seg_loss_1ch(logits, targets, kind):
    """loss on [B,1,H,W] (or [B,H,W]) logits, e.g. MultiTaskLoss's seg term"""
    if logits.dim() == 3:
        logits = logits.unsqueeze(1)
    return _SegLossFn.apply(logits, targets, kind, None)


class _MultiTaskFn(torch.autograd.Function):
    @staticmethod
    def forward(fctx, seg, cls, seg_t, cls_t, w, kind):
        out, tgt = _prep(seg, seg_t)
        B = out.shape[0]
        Pn = out[0].numel()
        dev = out.device
        seg_loss, gz = _seg_forward(kind, out, 1, tgt, B, Pn, None, True)
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


def binary_confusion(outputs, targets, conf=None):
    """device uint64[4] (+)= (tp, fp, fn, tn).  outputs [B,2,H,W] (argmax, tie -> 0) or [B,1,H,W]
    (sigmoid > 0.5).  No host sync: callers read the counters once per split."""
    out, tgt = _prep(outputs, targets)
    B, nch = out.shape[0], out.shape[1]
    Pn = out[0, 0].numel()
    if conf is None:
        conf = torch.zeros(4, dtype=torch.int64, device=out.device)
    lib.confusion(P(out), nch, P(tgt), B, Pn, P(conf), _stream(out.device))
    return conf
