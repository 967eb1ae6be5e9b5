"""Fused Adam over a HIP model's flat parameter arena (torch.optim.Adam semantics, train.py:62-78)."""
from __future__ import annotations

import torch

from .lib import lib
from . import ops
from .ops import P
from .plan import py


class FusedAdam(torch.optim.Optimizer):
    """Drop-in for ``optim.Adam(model.parameters(), lr, betas, weight_decay)`` on a HipModel.

    One kernel updates every parameter: the model keeps params, grads and the two moment buffers
    as flat fp32 arrays.  ``param_groups[0]['lr']`` is read at each step, so the reference's
    ``set_optimizer_lr`` (model/unet_training.py:192-199) works unchanged.

    ``capturable=True`` (as torch.optim.Adam's flag): lr and the step count live in device memory so
    the step can be captured in a HIP graph and replayed; ``step()`` outside a capture refreshes the
    device lr from ``param_groups`` (one small H2D copy when it changed).

    ``overlap=True``: the update runs per gradient bucket (ddp.GradBuckets; one is created with
    ``allreduce=False`` when the model has none) on the weight-gradient stream DURING backward, right
    after the bucket's last gradient (and its all-reduce under DDP), followed by the re-pack of that
    bucket's conv weights into the GEMM images the next forward reads -- so neither the update nor
    the pack sits on the compute stream's critical path.  ``step()`` then only commits the step
    count.  The update uses ``param_groups[0]`` as read at that backward, so lr changes must come
    before ``backward()``; incompatible with a grad scaler (no ``grad_scale``), and a backward is
    always followed by ``step()`` (the update already happened).  bench.py uses it; train.py keeps
    the reference's backward -> step order.
    """

    def __init__(self, model, lr=1e-3, betas=(0.9, 0.999), eps=1e-8, weight_decay=0.0, capturable=False,
                 overlap=False, bucket_mb=8.0):
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
        self.overlap = overlap
        self._applied = False  # an overlapped update ran in the last backward
        if overlap:
            if capturable:
                raise ValueError("FusedAdam: overlap and capturable are exclusive")
            from .ddp import GradBuckets
            b = getattr(model, "_buckets", None)
            if b is None:
                b = GradBuckets(model, bucket_mb=bucket_mb, allreduce=False)
            b.actions.append(self._bucket_update)
            b.finish_actions.append(self._bucket_finish)

    def _state(self, flat):
        if self._m is None or self._m.device != flat.device:
            self._m = torch.zeros_like(flat)
            self._v = torch.zeros_like(flat)

    def _bucket_update(self, i, s, e, stream):
        """Adam over the arena slice [s, e) + re-pack of its convs, on `stream` (GradBuckets action)"""
        m = self.model
        flat, grad = m._flat, m._flat_grad
        self._state(flat)
        g = self.param_groups[0]
        b1, b2 = g["betas"]
        st = stream.cuda_stream if stream is not None else torch.cuda.current_stream(flat.device).cuda_stream
        lib.adam(P(flat[s:e]), P(grad[s:e]), P(self._m[s:e]), P(self._v[s:e]), e - s, float(g["lr"]), float(b1),
                 float(b2), float(g["eps"]), float(g["weight_decay"]), self._step + 1, None, st)
        m._pack_range(s, e)
        self._applied = True

    def _bucket_finish(self):
        if self._applied:
            self.model._mark_prepacked()

    def _commit_step(self):
        self._applied = False
        self._step += 1

    def zero_grad(self, set_to_none: bool = True):  # keep the grads as arena views
        m = self.model
        m._attach_grads()
        g = m._flat_grad
        if ops.OVERLAP and g.is_cuda and not torch.cuda.is_current_stream_capturing():
            # nothing writes the arena before backward: clear it on the weight-gradient stream, idle
            # during the forward, instead of in front of the forward on the compute stream; the
            # backward (and any step / grad read before it) waits for the side stream (which holds
            # nothing after the clear until then).  C-ABI stream waits: a step plan logs them
            cur = torch.cuda.current_stream(g.device)
            side = ops.side_stream(g.device)
            lib.stream_wait(side.cuda_stream, cur.cuda_stream)
            with torch.cuda.stream(side):
                g.zero_()
            m._grad_zero_side = side
        else:
            g.zero_()

    @torch.no_grad()
    def step(self, closure=None, grad_scale=None):
        loss = closure() if closure is not None else None
        m = self.model
        m._wait_grad_zero()
        if self._applied:
            if grad_scale is not None:
                raise ValueError("FusedAdam(overlap=True) cannot take a grad scale (the update ran in backward)")
            py(self._commit_step)  # host state: a step plan advances the count every replay
            return loss
        # host state (the step count, lr) is read inside a py() action, so a step plan re-reads it and
        # advances the count on every replay instead of repeating the recording step's update
        py(self._plain_step, grad_scale)
        return loss

    def _plain_step(self, grad_scale):
        """the whole-arena update on the current stream (non-overlapped path)"""
        m = self.model
        m._prepacked = None  # the weights change below: the next forward packs them
        flat, grad = m._flat, m._flat_grad
        self._state(flat)
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
