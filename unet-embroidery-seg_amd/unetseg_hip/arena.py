"""Fused Adam over a HIP model's flat parameter arena (torch.optim.Adam semantics, train.py:62-78)."""
from __future__ import annotations

import torch

from .lib import lib
from .ops import P


class FusedAdam(torch.optim.Optimizer):
    """Drop-in for ``optim.Adam(model.parameters(), lr, betas, weight_decay)`` on a HipModel.

    One kernel updates every parameter: the model keeps params, grads and the two moment buffers
    as flat fp32 arrays.  ``param_groups[0]['lr']`` is read at each step, so the reference's
    ``set_optimizer_lr`` (model/unet_training.py:192-199) works unchanged.

    ``capturable=True`` (as torch.optim.Adam's flag): lr and the step count live in device memory so
    the step can be captured in a HIP graph and replayed; ``step()`` outside a capture refreshes the
    device lr from ``param_groups`` (one small H2D copy when it changed).
    """

    def __init__(self, model, lr=1e-3, betas=(0.9, 0.999), eps=1e-8, weight_decay=0.0, capturable=False):
        if not hasattr(model, "_flat"):
            raise TypeError("FusedAdam needs a HipModel (flat parameter arena)")
        defaults = dict(lr=lr, betas=betas, eps=eps, weight_decay=weight_decay)
        super().__init__(model._param_list, defaults)
        self.model = model
        self._step = 0
        self._m = None
        self._v = None
        self.capturable = capturable
        self._hyper = None  # device [lr] (capturable)
        self._step_dev = None  # device int32 steps taken (capturable)
        self._lr_dev = None

    def zero_grad(self, set_to_none: bool = True):  # keep the grads as arena views
        self.model._attach_grads()
        self.model._flat_grad.zero_()

    @torch.no_grad()
    def step(self, closure=None, grad_scale=None):
        loss = closure() if closure is not None else None
        m = self.model
        flat, grad = m._flat, m._flat_grad
        if self._m is None or self._m.device != flat.device:
            self._m = torch.zeros_like(flat)
            self._v = torch.zeros_like(flat)
        m._attach_grads()
        g = self.param_groups[0]
        self._step += 1
        b1, b2 = g["betas"]
        st = torch.cuda.current_stream(flat.device).cuda_stream
        if self.capturable:
            if self._hyper is None or self._hyper.device != flat.device:
                self._hyper = torch.zeros(1, dtype=torch.float32, device=flat.device)
                self._step_dev = torch.full((1,), self._step - 1, dtype=torch.int32, device=flat.device)
                self._lr_dev = None
            if self._lr_dev != float(g["lr"]) and not torch.cuda.is_current_stream_capturing():
                self._hyper.fill_(float(g["lr"]))
                self._lr_dev = float(g["lr"])
            lib.adam_dev(P(flat), P(grad), P(self._m), P(self._v), flat.numel(), P(self._hyper), P(self._step_dev),
                         float(b1), float(b2), float(g["eps"]), float(g["weight_decay"]), P(grad_scale), st)
        else:
            lib.adam(P(flat), P(grad), P(self._m), P(self._v), flat.numel(), float(g["lr"]), float(b1), float(b2),
                     float(g["eps"]), float(g["weight_decay"]), self._step, P(grad_scale), st)
        return loss

    def state_dict(self):
        sd = super().state_dict()
        step = int(self._step_dev.item()) if (self.capturable and self._step_dev is not None) else self._step
        sd["flat_state"] = {"step": step, "exp_avg": self._m, "exp_avg_sq": self._v}
        return sd

    def load_state_dict(self, sd):
        fs = sd.pop("flat_state", None)
        super().load_state_dict(sd)
        if fs is not None:
            self._step = fs["step"]
            self._m, self._v = fs["exp_avg"], fs["exp_avg_sq"]
            self._hyper = self._step_dev = None  # rebuilt from the host values at the next step
