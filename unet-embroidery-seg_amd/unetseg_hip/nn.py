"""Parameter containers with the reference's module tree, the flat parameter arena and the
model-level autograd Function.

The containers (``Conv2d``, ``BatchNorm2d``, ``Linear``, ``Seq`` and parameterless placeholders)
reproduce the reference's ``state_dict`` keys and shapes exactly (e.g. ``resnet.layer1.0.conv1.weight``,
``up_conv.1.weight``, ``inc.net.0.weight``, ``cls_head.2.weight``) and consume torch's CPU RNG in the
same order as the reference's constructors, so a given seed yields the same initial weights.
They hold data only: their ``forward`` raises.  A ``HipModel``'s forward runs the model's
hand-written HIP program (``_run``) and records its reverse tape.

Parameters live in ONE flat fp32 buffer (``_flat``) laid out in reverse forward order, with a
parallel flat gradient buffer; ``param.data`` / ``param.grad`` are views into them.  The fused Adam
and the DDP all-reduce operate on these flat buffers.
"""
from __future__ import annotations

import math

import torch
import torch.nn as nn
from torch.nn import init

from . import ops
from .lib import DT_BF16, DT_F32


class _Leaf(nn.Module):
    def forward(self, *a, **k):  # pragma: no cover - guard
        raise RuntimeError(f"{type(self).__name__} is a parameter container of a HIP model; call the top-level model")


class Conv2d(_Leaf):
    """Same parameters/init as nn.Conv2d (kaiming_uniform a=sqrt(5), bias U(+-1/sqrt(fan_in)))."""

    def __init__(self, in_channels, out_channels, kernel_size, stride=1, padding=0, bias=True):
        super().__init__()
        self.in_channels, self.out_channels = in_channels, out_channels
        self.kernel_size = (kernel_size, kernel_size)
        self.stride, self.padding = stride, padding
        self.weight = nn.Parameter(torch.empty(out_channels, in_channels, kernel_size, kernel_size))
        self.bias = nn.Parameter(torch.empty(out_channels)) if bias else None
        init.kaiming_uniform_(self.weight, a=math.sqrt(5))
        if self.bias is not None:
            bound = 1.0 / math.sqrt(in_channels * kernel_size * kernel_size)
            init.uniform_(self.bias, -bound, bound)


class Linear(_Leaf):
    def __init__(self, in_features, out_features):
        super().__init__()
        self.in_features, self.out_features = in_features, out_features
        self.weight = nn.Parameter(torch.empty(out_features, in_features))
        self.bias = nn.Parameter(torch.empty(out_features))
        init.kaiming_uniform_(self.weight, a=math.sqrt(5))
        bound = 1.0 / math.sqrt(in_features)
        init.uniform_(self.bias, -bound, bound)


class BatchNorm2d(_Leaf):
    def __init__(self, num_features, eps=1e-5, momentum=0.1):
        super().__init__()
        self.num_features, self.eps, self.momentum = num_features, eps, momentum
        self.weight = nn.Parameter(torch.ones(num_features))
        self.bias = nn.Parameter(torch.zeros(num_features))
        self.register_buffer("running_mean", torch.zeros(num_features))
        self.register_buffer("running_var", torch.ones(num_features))
        self.register_buffer("num_batches_tracked", torch.tensor(0, dtype=torch.long))


class ReLU(_Leaf):
    pass


class Sigmoid(_Leaf):
    pass


class Flatten(_Leaf):
    pass


class AdaptiveAvgPool2d(_Leaf):
    def __init__(self, output_size=1):
        super().__init__()
        self.output_size = output_size


class MaxPool2d(_Leaf):
    def __init__(self, kernel_size, stride=None, padding=0, ceil_mode=False):
        super().__init__()
        self.kernel_size, self.stride = kernel_size, stride or kernel_size
        self.padding, self.ceil_mode = padding, ceil_mode


class Upsample(_Leaf):
    def __init__(self, scale_factor=2, align_corners=False):
        super().__init__()
        self.scale_factor, self.align_corners = scale_factor, align_corners


class Dropout(_Leaf):
    def __init__(self, p=0.5):
        super().__init__()
        self.p = p


class Seq(nn.Module):
    """nn.Sequential-compatible container (keys '0', '1', ...); not callable."""

    def __init__(self, *mods):
        super().__init__()
        for i, m in enumerate(mods):
            self.add_module(str(i), m)

    def __getitem__(self, i):
        return self._modules[str(i)]

    def __len__(self):
        return len(self._modules)

    def forward(self, *a):  # pragma: no cover
        raise RuntimeError("Seq is a parameter container of a HIP model; call the top-level model")


# ------------------------------------------------------------------------------------------------
# model base
# ------------------------------------------------------------------------------------------------
class _ModelFn(torch.autograd.Function):
    @staticmethod
    def forward(fctx, model, x, dt, *params):
        ctx = ops.Ctx(dt, model.training, True, x.device)
        outs = model._run(ctx, x)
        fctx.hctx = ctx
        fctx.model = model
        fctx.nparams = len(params)
        return outs if isinstance(outs, tuple) else (outs,)

    @staticmethod
    def backward(fctx, *grads):
        ctx = fctx.hctx
        model = fctx.model
        for holder, g in zip(ctx.out_holders, grads):
            holder["grad"] = g
        model._wait_grad_zero()
        model._attach_grads()
        ctx.grad_hook = model._grad_hook
        ctx.finish_hook = model._after_backward  # inside backward: before the streams join
        ctx.backward()
        fctx.hctx = None
        return (None, None, None) + (None,) * fctx.nparams


def _is_autocast():
    try:
        return torch.is_autocast_enabled("cuda")
    except TypeError:  # older signature
        return torch.is_autocast_enabled()


class HipModel(nn.Module):
    """Base class: flat parameter arena + forward dispatch to the HIP program ``_run``."""

    #: "auto" -> bf16 under torch.autocast (the reference's AMP path), fp32 otherwise; or "bf16"/"fp32"
    compute_dtype = "auto"

    def _finalize(self):
        params = [p for _, p in self.named_parameters()]
        # reverse forward order: backward finishes gradients front-to-back (contiguous DDP buckets)
        order = list(reversed(params))
        total = sum(p.numel() for p in order)
        flat = torch.zeros(total, dtype=torch.float32)
        off = 0
        self._slices = {}
        for p in order:
            n = p.numel()
            flat[off:off + n].copy_(p.data.reshape(-1))
            self._slices[id(p)] = (off, n)
            off += n
        self._flat = flat
        self._flat_grad = torch.zeros_like(flat)
        self._param_list = params
        self._repoint()
        self._grad_hook = None
        self._after_backward = None
        self._packed = []
        for m in self.modules():
            if isinstance(m, Conv2d) and m.out_channels % 8 == 0:  # Cout 1/2 heads use the pointwise kernels
                cpad = 8 if m.in_channels < 8 else None
                m._pc = ops.PackedConv(m, cpad)
                self._packed.append(m._pc)

    def _wait_grad_zero(self):
        """the compute stream waits for a gradient-arena clear enqueued on the side stream (FusedAdam.zero_grad)"""
        side = getattr(self, "_grad_zero_side", None)
        if side is not None:
            from .lib import lib
            lib.stream_wait(torch.cuda.current_stream(self._flat_grad.device).cuda_stream, side.cuda_stream)
            self._grad_zero_side = None

    def _repoint(self):
        for p in self._param_list:
            off, n = self._slices[id(p)]
            p.data = self._flat[off:off + n].view(p.shape)
        self._attach_grads(force=True)

    def _attach_grads(self, force=False):
        """make every param.grad a view of the flat gradient arena (None -> zeros, foreign -> copied)"""
        views = getattr(self, "_grad_views", None)
        if not force and views is not None and all(p.grad is v for p, v in views):
            return  # fast path (every step): nothing was detached or replaced
        base = self._flat_grad.data_ptr()
        esz = self._flat_grad.element_size()
        for p in self._param_list:
            off, n = self._slices[id(p)]
            g = p.grad
            if not force and g is not None and g.data_ptr() == base + off * esz:
                continue
            view = self._flat_grad[off:off + n].view(p.shape)
            if not force:
                if g is None:
                    view.zero_()
                else:
                    view.copy_(g)
            p.grad = view
        self._grad_views = [(p, p.grad) for p in self._param_list]

    def flat_slice(self, p):
        return self._slices[id(p)]

    def _apply(self, fn, recurse=True):
        # move the arena as a whole, then the buffers; params/grads stay views of the arena
        self._flat = fn(self._flat)
        self._flat_grad = fn(self._flat_grad)
        if self._flat.dtype != torch.float32:
            raise TypeError("HIP models keep fp32 master parameters (use autocast for bf16 compute)")
        for p in self._param_list:
            p.grad = None
        self._repoint()
        for m in self.modules():
            for k, b in list(m._buffers.items()):
                if b is not None:
                    m._buffers[k] = fn(b)
        for pc in self._packed:
            pc.wk = pc.wt = None
        self._prepacked = None
        self._range_tables = {}
        return self

    def _dtype(self):
        if self.compute_dtype == "bf16":
            return DT_BF16
        if self.compute_dtype == "fp32":
            return DT_F32
        return DT_BF16 if _is_autocast() else DT_F32

    def _pack_weights(self, ctx, need_t):
        if not self._packed:
            return
        # convs on the (padded) image need no data gradient -- unless an input op with parameters
        # sits in front of them (dualdense's BN-ReLU on the image: force_t)
        flags = [need_t and (pc.conv.in_channels >= 8 or getattr(pc, "force_t", False)) for pc in self._packed]
        key = (ctx.dt, str(ctx.device), tuple(flags))
        pre = getattr(self, "_prepacked", None)
        self._prepacked = None
        if need_t:
            self._pack_key = key  # the flags the per-bucket re-pack reuses (recording forwards only)
        if pre == key:
            return  # an overlapped optimizer update re-packed every conv right after writing it
        if getattr(self, "_pack_table", None) is None:
            self._pack_table = ops.PackTable()
        self._pack_table.run(ctx, self._packed, flags)

    def _pack_range(self, s, e):
        """re-pack the convs whose weights lie in arena range [s, e) -- on the current stream, with
        the dtype / transposed-image flags of the last forward (FusedAdam(overlap=True), per bucket)"""
        key = getattr(self, "_pack_key", None)
        if key is None or not self._packed:
            return
        tabs = self.__dict__.setdefault("_range_tables", {})
        ent = tabs.get((s, e))
        if ent is None:
            sel = [i for i, pc in enumerate(self._packed) if s <= self._slices[id(pc.conv.weight)][0] < e]
            ent = tabs[(s, e)] = (sel, ops.PackTable())
        sel, table = ent
        if not sel:
            return
        dt, dev, flags = key
        ctx = ops.Ctx(dt, True, False, torch.device(dev))
        table.run(ctx, [self._packed[i] for i in sel], [flags[i] for i in sel])

    def _mark_prepacked(self):
        """every bucket's convs were re-packed after the update: the next forward with the same
        dtype / flags skips its pack"""
        self._prepacked = getattr(self, "_pack_key", None)

    def load_state_dict(self, *a, **k):
        self._prepacked = None
        return super().load_state_dict(*a, **k)

    def forward(self, x):
        if not x.is_cuda:
            raise RuntimeError("HIP U-Net models run on a HIP device only (no CPU path): move the model and input to cuda")
        if self._flat.device != x.device:
            raise RuntimeError(f"model is on {self._flat.device}, input on {x.device}")
        dt = self._dtype()
        record = torch.is_grad_enabled() and any(p.requires_grad for p in self._param_list)
        if record:
            outs = _ModelFn.apply(self, x, dt, *self._param_list)
            return outs if len(outs) > 1 else outs[0]
        ctx = ops.Ctx(dt, self.training, False, x.device)
        with torch.no_grad():
            return self._run(ctx, x)

    def _run(self, ctx, x):  # pragma: no cover - abstract
        raise NotImplementedError
