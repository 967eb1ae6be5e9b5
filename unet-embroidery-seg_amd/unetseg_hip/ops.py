"""Host-side op layer: launches the HIP kernels and records the reverse-mode tape.

Every activation is a ``Node`` holding an NHWC tensor view (``stride(-1) == 1``; the pixel stride
``stride(-2)`` may exceed the channel count, so channel slices of a concat buffer are addressed in
place).  Forward ops push a closure onto ``Ctx.tape``; ``Ctx.backward()`` runs them in reverse.
Gradients of activations are accumulated in-kernel (``accumulate`` flags) and parameter gradients
go straight into the model's flat fp32 gradient arena.  PyTorch supplies device memory and the
stream only; all arithmetic is in libunetseg_hip.so.
"""
from __future__ import annotations

import math
import os

import numpy as np
import torch

from .lib import DT_BF16, DT_F32, lib
from .lib import dgrad_config as _dgrad_config

BN_TILE = 128  # == unetseg_conv_tile_m(): M tile of the conv kernel, hence of its BN partials


def P(t):
    return 0 if t is None else t.data_ptr()


def ldp(t):
    """pixel stride (elements) of an NHWC view"""
    return 0 if t is None else t.stride(-2)


_QMEMO = {}

#: dispatch switches the library reads on every call (not once per process): tests flip them
#: in-process, so each is part of the query memo's key (conv.hip / conv_fast.hip / elem.hip getenv)
_CALL_SWITCHES = ("UNETSEG_TN_NO_HALO_RING", "UNETSEG_TN_CFG", "UNETSEG_TN_CFG_NO23", "UNETSEG_NO_FAST",
                  "UNETSEG_RED_TARGET", "UNETSEG_MAXPOOL_GENERIC")
_ENV = os.environ


def _q(name, *args):
    """a host-only shape query of the C ABI (tile counts, partial rows, workspace sizes), memoised: its
    result depends on the integer arguments only, so callers pass 0 for every pointer and the stream"""
    key = (name, tuple(map(_ENV.get, _CALL_SWITCHES))) + args
    v = _QMEMO.get(key)
    if v is None:
        v = _QMEMO[key] = getattr(lib, name)(*args)
    return v


class Node:
    """An activation.  ``uses`` counts the ops that consumed it; ``fuse`` describes the ReLU that
    produced it, so that a sole consumer conv can apply that op's backward mask and first reduction
    in its data-gradient epilogue (``fused`` then holds the partials for the producer's backward).
    ``lazy`` (a BNState): the node stands for relu(BN(data)) that was never stored -- ``data`` is the
    BN input and the consuming conv applies BN-ReLU on load (``bn(..., lazy=True)``).  ``kpad`` (Kp > K):
    the gradient buffer is allocated as the first K channels of a zeroed Kp-channel tensor (``gpad``),
    which the producing conv's padded-K backward reads as it is (see conv)."""

    __slots__ = ("data", "grad", "need_grad", "uses", "fuse", "fused", "lazy", "head", "mbits", "kpad", "gpad")

    def __init__(self, data, need_grad=True):
        self.data = data
        self.grad = None
        self.need_grad = need_grad
        self.uses = 0
        self.fuse = None
        self.fused = None
        self.lazy = None
        self.head = None  # (head Conv2d, fp32 logits) computed by the producing conv's epilogue
        self.mbits = None  # packed ReLU mask of data (unetseg_conv2d_fwd_mask), read by post 4
        self.kpad = 0
        self.gpad = None

    @property
    def shape(self):
        return self.data.shape


def use(*nodes):
    for n in nodes:
        if n is not None:
            n.uses += 1


#: fuse ReLU / BN-ReLU backward pass 1 into the consumer conv's dgrad (UNETSEG_NO_FUSE=1 disables)
FUSE = os.environ.get("UNETSEG_NO_FUSE", "0") != "1"
#: the model's 1x1 head computed in the epilogue of the conv before it (UNETSEG_NO_HEAD_FUSE=1 disables)
FUSE_HEAD = os.environ.get("UNETSEG_NO_HEAD_FUSE", "0") != "1"
#: the ReLU backward of an upsample's input inside the upsample backward (UNETSEG_NO_UP_FUSE=1 disables)
FUSE_UP = os.environ.get("UNETSEG_NO_UP_FUSE", "0") != "1"
#: a 64-channel halo conv + bias + ReLU stores its ReLU mask as bits for the consumer's data gradient
#: (post 4) instead of that dgrad re-reading the activation (UNETSEG_NO_RELU_BITS=1 disables)
RELU_BITS = os.environ.get("UNETSEG_NO_RELU_BITS", "0") != "1"


_WORKSPACES = {}

#: when a list, conv calls append (kernel, algorithmic_flops, kernel_launches, start_event, end_event)
#: (bench.py probe; a stride-2 dgrad call launches one GEMM per output parity class)
PROBE = None


#: test hook (tests/test_gpu_teacher.py): an object with ``op(ctx, kind, out, ins, info)`` and
#: ``mark(ctx, name)``, told about every op a recording forward runs and about the model's block
#: boundaries, so a test can rebuild each block's backward in float64 from the tensors this path
#: stored; None outside that test (no cost)
TAP = None


def _tap(ctx, kind, out, ins, **info):
    if TAP is not None and ctx.tape is not None:
        TAP.op(ctx, kind, out, ins, info)


def tap_mark(ctx, name):
    """block boundary (model code): the ops recorded since the previous mark form one block"""
    if TAP is not None and ctx.tape is not None:
        TAP.mark(ctx, name)


class _probe:
    """HIP events around one op's launches, recorded on the stream the kernels run on."""

    def __init__(self, kind, flops, launches=1, desc=None, stream=None):
        self.kind, self.flops, self.launches, self.desc, self.stream = kind, flops, launches, desc, stream

    def __enter__(self):
        if PROBE is not None:
            self.e0 = torch.cuda.Event(enable_timing=True)
            self.e1 = torch.cuda.Event(enable_timing=True)
            self.e0.record(self.stream)
        return self

    def __exit__(self, *a):
        if PROBE is not None:
            self.e1.record(self.stream)
            PROBE.append((self.kind, self.flops, self.launches, self.e0, self.e1, self.desc))


#: weight gradients run on a second HIP stream, concurrent with the data-gradient chain of the
#: backward pass (UNETSEG_NO_OVERLAP=1 keeps everything on the compute stream)
OVERLAP = os.environ.get("UNETSEG_NO_OVERLAP", "0") != "1"
_SIDE = {}


#: priority of the weight-gradient stream (torch convention: lower = higher priority)
SIDE_PRIORITY = int(os.environ.get("UNETSEG_SIDE_PRIORITY", "0"))


#: UNETSEG_SIDE_CUMASK=<hex word>: the weight-gradient stream runs only on the CUs of that 32-bit
#: pattern, repeated over the chip (e.g. 55555555: every other CU), so its persistent kernels, which
#: hold a CU's LDS for their whole life, never keep a compute-stream kernel off every CU
SIDE_CUMASK = os.environ.get("UNETSEG_SIDE_CUMASK")


def side_stream(device):
    key = (device.type, device.index)
    if key not in _SIDE:
        if SIDE_CUMASK:
            import ctypes
            n = (torch.cuda.get_device_properties(device).multi_processor_count + 31) // 32
            words = (ctypes.c_uint32 * n)(*([int(SIDE_CUMASK, 16) & 0xFFFFFFFF] * n))
            out = ctypes.c_void_p()
            with torch.cuda.device(device):
                lib.stream_create_cumask(ctypes.addressof(words), n, ctypes.addressof(out))
            _SIDE[key] = torch.cuda.ExternalStream(out.value, device=device)
        else:
            _SIDE[key] = torch.cuda.Stream(device, priority=SIDE_PRIORITY)
    return _SIDE[key]


def workspace(nbytes, device, stream_key=0):
    """Stream-ordered scratch shared by consecutive launches on one stream (never shrunk: captured
    graphs keep pointers into every buffer ever handed out)."""
    key = (device.type, device.index, stream_key)
    lst = _WORKSPACES.setdefault(key, [])
    if not lst or lst[-1].numel() < nbytes:
        lst.append(torch.empty(max(int(nbytes), 1 << 20), dtype=torch.uint8, device=device))
    return lst[-1]


#: measurement hook (tools/tail_probe.py): called with the Ctx at the end of backward, after the tape,
#: the held-back weight gradients and the finish hook, right before the compute stream joins the side
ON_JOIN = None


class Ctx:
    def __init__(self, dt, training, record, device):
        self.dt = dt
        self.tdtype = torch.bfloat16 if dt == DT_BF16 else torch.float32
        self.training = training
        self.tape = [] if record else None
        self.device = device
        self.main = torch.cuda.current_stream(device)
        self.stream = self.main.cuda_stream
        self.grad_hook = None  # called with a param after its gradient is final (DDP bucketing)
        self.finish_hook = None  # called once the tape is done, before the compute stream joins the side
        self.side = None  # weight-gradient stream, set while backward runs with OVERLAP
        self.deferred = []  # weight-gradient launches held back until a flush point (defer_wgrad)
        self.flushed = False  # the flush marker has run in this backward
        self.has_marker = False  # the forward recorded a flush marker (models without one defer nothing)
        self.layer = None  # the encoder layer the forward is in (flush_point), for WG_SERIAL_LAYERS

    def push(self, fn):
        if self.tape is not None:
            self.tape.append(fn)

    def empty(self, *shape, dtype=None):
        return torch.empty(shape, dtype=dtype or self.tdtype, device=self.device)

    def f32(self, *shape):
        return torch.empty(shape, dtype=torch.float32, device=self.device)

    def backward(self):
        tape, self.tape = self.tape, None
        if OVERLAP:
            self.side = side_stream(self.device)
            lib.stream_wait(self.side.cuda_stream, self.stream)
        try:
            # pop each closure as it runs: its tensors are released during the pass (lower peak,
            # and the host frees them while it would otherwise wait on the launch queue, not in
            # one burst between the last backward launch and the optimizer)
            while tape:
                fn = tape.pop()
                fn()
                del fn
            self.flush_deferred()
            if self.finish_hook is not None:
                # the last buckets' collectives / optimizer updates, enqueued before the join below
                from .plan import py
                py(self.finish_hook)
        finally:
            if ON_JOIN is not None:
                ON_JOIN(self)
            if self.side is not None:
                # everything after backward (optimizer, frees of tape tensors) follows the wgrads
                lib.stream_wait(self.stream, self.side.cuda_stream)
                self.side = None

    def flush_deferred(self):
        while self.deferred:
            self.deferred.pop(0)()

    def param_done(self, *params, stream=None):
        """report parameters whose gradient is final AND that no later compute-stream kernel of this
        backward reads (nor its packed image): a bucket's all-reduce / optimizer update may run on the
        side stream right after (stand-in tensors that are not model parameters, e.g. a re-laid-out
        weight, are ignored by the hook).  stream: the weight-gradient stream when the gradients were
        written there and that stream's last launch is their writer (the bucket fences on an event
        recorded now, not on whatever the stream holds when the bucket completes); None = the
        compute stream"""
        if self.grad_hook is not None:
            for p in params:
                if p is not None:
                    self.grad_hook(p, stream)


#: weight gradients of 3x3 convs whose output has >= this many pixels per image are held back in
#: backward until a flush marker (flush_point): they then run on the side stream beside the encoder's
#: memory-bound layers instead of beside the data gradients of their own layers.  Default: the
#: decoder's virtual-concat convs (MFMA-bound, each used to share the CUs with its own equally heavy data
#: gradient), released when the backward reaches layer4 -- step A/B +0.45 % (three interleaved repeats);
#: holding back every decoder 3x3 wgrad, or releasing at layer3, measured neutral to -3 %
#: (0 = off; UNETSEG_WG_DEFER_HW, UNETSEG_WG_DEFER_CAT, UNETSEG_WG_FLUSH)
WG_DEFER_HW = int(os.environ.get("UNETSEG_WG_DEFER_HW", "1024"))
#: where the flush marker sits in forward order: "decoder" (before the decoder), "layer4" / "layer3" / "layer2"
#: (before that encoder layer: in backward the held-back gradients start once that layer's backward is done)
#: (round 5, replayed step plan: layer3 +0.1-0.3 % over layer4; round 4's eager host had layer4 best)
WG_FLUSH = os.environ.get("UNETSEG_WG_FLUSH", "layer3")


#: weight gradients of 3x3 convs whose output has >= this many pixels per image run on the compute stream
#: right after their data gradient instead of beside it on the side stream (0 = never): two persistent
#: one-block-per-CU halo kernels sharing the CUs each take ~2x their isolated time (UNETSEG_WG_SERIAL_HW)
WG_SERIAL_HW = int(os.environ.get("UNETSEG_WG_SERIAL_HW", "0"))
#: encoder layers ("stem", "layer1", ...) whose weight gradients run on the compute stream: at the end of
#: the backward the weight-gradient stream lags the compute stream (UNETSEG_WG_SERIAL_LAYERS, comma list).
#: Round 4 (eager host) measured stem + layer1 best; with the step plan's replayed host (round 5, two
#: interleaved repeats each) the stem alone: C2 1007-1011 vs 997-998 img/s, C5 807-810 vs 797-799
#: (layer1 serial no better than stem + layer1; none equal to stem within noise)
WG_SERIAL_LAYERS = frozenset(v for v in os.environ.get("UNETSEG_WG_SERIAL_LAYERS", "stem").split(",") if v)

#: the side-stream weight gradient is enqueued after its layer's data gradient and waits for it
#: (UNETSEG_WG_AFTER_DGRAD=1): the data gradient -- the critical path -- then gets the CUs first instead
#: of both becoming ready on the same event and sharing them (round 6 experiment)
WG_AFTER_DGRAD = os.environ.get("UNETSEG_WG_AFTER_DGRAD", "0") == "1"

#: only the virtual-concat convs (the decoder's unetUp conv1) are held back (UNETSEG_WG_DEFER_CAT=0: every 3x3)
WG_DEFER_CAT = os.environ.get("UNETSEG_WG_DEFER_CAT", "1") == "1"


def defer_wgrad(ctx, N, Pq, Qq, R, S, x2):
    """hold this conv's weight gradient until the flush marker (never after it has run: the
    encoder's own gradients are not pushed to the end of the backward)"""
    return (bool(WG_DEFER_HW) and ctx.side is not None and ctx.has_marker and not ctx.flushed
            and Pq * Qq >= WG_DEFER_HW and R * S > 1
            and (x2 is not None or not WG_DEFER_CAT))


def flush_point(ctx, where):
    """forward marker: in backward, the deferred weight gradients are launched when the tape reaches it"""
    ctx.layer = where
    if WG_DEFER_HW and where == WG_FLUSH and ctx.tape is not None:
        ctx.has_marker = True

        def marker():
            ctx.flushed = True
            ctx.flush_deferred()
        ctx.push(marker)


def gbuf(ctx, node):
    """gradient buffer of node: (tensor, accumulate flag)"""
    if node.grad is None:
        if node.kpad:
            shape = node.data.shape
            node.gpad = torch.zeros(*shape[:-1], node.kpad, dtype=ctx.tdtype, device=ctx.device)
            node.grad = node.gpad[..., :shape[-1]]
        else:
            node.grad = ctx.empty(*node.data.shape)
        return node.grad, 0
    return node.grad, 1


def give_grad(ctx, node, g):
    """node.grad += g (g is an NHWC view); adopts g without a copy when node has no gradient yet"""
    if not node.need_grad:
        return
    if node.grad is None:
        node.grad = g
        return
    N, H, W, C = g.shape
    lib.add(ctx.dt, P(g), ldp(g), P(node.grad), ldp(node.grad), N * H * W, C, ctx.stream)


# ------------------------------------------------------------------------------------------------
# weights
# ------------------------------------------------------------------------------------------------
class PackedConv:
    """bf16/fp32 GEMM images of one conv weight: wk [K][R][S][Cpad] (fwd), wt [C][R][S][Kld] (dgrad).
    Kld = K, except for the narrow 1x1 convs whose gradients run through a 64-channel zero-padded dY
    (PAD_K, bf16): their wt rows are Kp = 64-rounded wide with zero columns K..Kp, which is the B
    operand that padded data gradient reads -- packed in place by the batched pack (UnetsegPackDesc
    Kld), no per-step padded copy."""

    def __init__(self, conv, cpad=None):
        self.conv = conv
        K, C, R, S = conv.weight.shape
        self.K, self.C, self.R, self.S = K, C, R, S
        self.cpad = cpad or C
        self.wk = self.wt = None
        self.dt = None
        self.kld = K

    def padk(self, dt):
        """the one place that decides whether this conv's gradients run through a 64-padded dY (conv()
        reads it for out.kpad; the padded data gradient needs wt rows Kld wide): narrow bf16 1x1
        stride-1 convs.  conv() also requires a single input (no virtual concat)."""
        K = self.K
        return (PAD_K and dt == DT_BF16 and self.R == 1 and self.S == 1 and K % 64 != 0 and K % 8 == 0 and
                self.conv.stride in (1, (1, 1)))

    def ensure(self, ctx, need_t):
        """allocate the packed images for ctx's dtype/device (no launch)"""
        K, C, R, S = self.K, self.C, self.R, self.S
        if self.wk is None or self.dt != ctx.dt or self.wk.device != ctx.device:
            self.wk = ctx.empty(K, R, S, self.cpad)
            self.wt = None
            self.dt = ctx.dt
            self.kld = -(-K // 64) * 64 if self.padk(ctx.dt) else K
        if need_t and self.wt is None:
            # [Cpad][R][S][Kld]: the padded input channels' rows (and padded K columns) stay zero (the pack
            # writes C rows x K columns), so a data gradient over all Cpad channels is well defined
            self.wt = torch.zeros((self.cpad, R, S, self.kld), dtype=ctx.tdtype, device=ctx.device)

    def pack(self, ctx, need_t):
        K, C, R, S = self.K, self.C, self.R, self.S
        self.ensure(ctx, need_t)
        if need_t and self.kld != K:  # the single-conv pack writes K-wide rows: stage, then widen
            tmp = torch.empty((self.cpad, R, S, K), dtype=ctx.tdtype, device=ctx.device)
            lib.pack_conv_weight(ctx.dt, P(self.conv.weight), K, C, R, S, self.cpad, P(self.wk), P(tmp), ctx.stream)
            self.wt.zero_()  # lib.add accumulates: a re-pack must not add onto the previous image
            lib.add(ctx.dt, P(tmp), K, P(self.wt), self.kld, self.cpad * R * S, K, ctx.stream)
            return
        lib.pack_conv_weight(ctx.dt, P(self.conv.weight), K, C, R, S, self.cpad, P(self.wk),
                             P(self.wt) if need_t else 0, ctx.stream)


_PACK_DESC = np.dtype([("w", "<u8"), ("wk", "<u8"), ("wt", "<u8"), ("start", "<i8"), ("K", "<i4"), ("C", "<i4"),
                       ("R", "<i4"), ("S", "<i4"), ("Cpad", "<i4"), ("Kld", "<i4")])  # UnetsegPackDesc


class PackTable:
    """Device descriptor table for packing every conv weight of a model in ONE launch
    (unetseg_pack_conv_weights); rebuilt only when a buffer address changes."""

    def __init__(self):
        self.key = None
        self.desc = None
        self.total = 0

    def run(self, ctx, pcs, need_t):
        for pc, nt in zip(pcs, need_t):
            pc.ensure(ctx, nt)
        key = (ctx.dt, str(ctx.device)) + tuple(
            (pc.conv.weight.data_ptr(), pc.wk.data_ptr(), pc.wt.data_ptr() if (nt and pc.wt is not None) else 0)
            for pc, nt in zip(pcs, need_t))
        if key != self.key:
            d = np.zeros(len(pcs), dtype=_PACK_DESC)
            start = 0
            for i, (pc, nt) in enumerate(zip(pcs, need_t)):
                d[i] = (pc.conv.weight.data_ptr(), pc.wk.data_ptr(), pc.wt.data_ptr() if nt else 0, start,
                        pc.K, pc.C, pc.R, pc.S, pc.cpad, pc.kld)
                start += lib.pack_tiles(pc.K, pc.cpad, pc.R * pc.S)
            self.desc = torch.from_numpy(d.view(np.uint8).copy()).to(ctx.device)
            self.total = start
            self.key = key
        lib.pack_conv_weights(ctx.dt, P(self.desc), len(pcs), self.total, ctx.stream)


# ------------------------------------------------------------------------------------------------
# ops
# ------------------------------------------------------------------------------------------------
def pack_input(ctx, x, cpad=8):
    """NCHW fp32 image batch -> NHWC node with channels zero-padded to cpad"""
    x = x.contiguous()
    if x.dtype != torch.float32:
        x = x.float()
    N, C, H, W = x.shape
    y = ctx.empty(N, H, W, cpad)
    lib.pack_input(ctx.dt, P(x), N, C, H, W, cpad, P(y), ctx.stream)
    out = Node(y, need_grad=False)
    _tap(ctx, "input", out, [], image=x)
    return out


#: narrow 1x1 conv gradients through a 64-channel zero-padded dY (UNETSEG_NO_PADK=1: generic kernels)
PAD_K = os.environ.get("UNETSEG_NO_PADK", "0") != "1"


def _dgrad_launches(ctx, ldy, N, Pq, Qq, K, C, R, S, stride, pad, H, W):
    """kernel launches of one data-gradient call (probe bookkeeping only): one per parity class,
    the classes merged into one launch (configs multi*) counting once"""
    if stride == 1 or PROBE is None:
        return stride * stride
    cfgs = _dgrad_config(ctx.dt, ldy, N, Pq, Qq, K, C, R, S, stride, pad, C, H, W)
    merged = sum(1 for c in cfgs if c.startswith("multi"))
    return len(cfgs) - merged + (1 if merged else 0)


def conv(ctx, x1, pc, x2=None, relu=False, stats=False, out=None, head=None):
    """y = conv(cat[x1, x2]) (+bias if the conv has one, ReLU).  Stride/padding come from the
    Conv2d container.  out: an NHWC view (pixel stride >= K) to write y into, e.g. a channel slice
    of a dense block's concatenation buffer.  head: the 1x1 Conv2d (1 or 2 outputs) that consumes y
    next -- its logits come out of this conv's epilogue when the shape runs on the halo kernel
    (unetseg_conv2d_fwd_head) and ride on the returned node for pw_head.  Returns (Node y, BN
    partials or None)."""
    stride, pad = pc.conv.stride, pc.conv.padding
    lazy = x1.lazy
    if lazy is not None and not (x2 is None and ctx.dt == DT_BF16 and pc.R == 1 and pc.S == 1 and stride == 1 and
                                 pad == 0 and x1.data.shape[-1] % 64 == 0 and pc.K % 64 == 0):
        _materialize(ctx, x1)
        lazy = None
    use(x1, x2)
    # x1's first consumer in the forward delivers the last contribution to its gradient in the backward
    last_grad = x1.uses == 1
    layer = ctx.layer
    X1 = x1.data
    N, H, W, C1 = X1.shape
    X2 = x2.data if x2 is not None else None
    C2 = X2.shape[-1] if X2 is not None else 0
    K, R, S = pc.K, pc.R, pc.S
    Pq = (H + 2 * pad - R) // stride + 1
    Qq = (W + 2 * pad - S) // stride + 1
    M = N * Pq * Qq
    y = ctx.empty(N, Pq, Qq, K) if out is None else out
    st = None
    stats = stats and ctx.training  # eval-mode BN normalises with the running statistics
    if stats:
        tile = _q("conv2d_fwd_tile_m", ctx.dt, C1, ldp(X1), C2, ldp(X2), N, H, W, K, R, S, stride, pad)
        st = (ctx.f32(math.ceil(M / tile), 2, K), tile)  # [row tiles][sum, M2][K]
    b = pc.conv.bias
    flops = 2.0 * M * K * pc.C * R * S  # algorithmic (unpadded Cin)
    # probe descriptor: (N, H, W, C1, C2, K, R, S, stride, pad, ld1, ld2); bench/tools map it to the
    # kernel configuration through the unetseg_conv2d_*_config queries
    desc = (N, H, W, C1, C2, K, R, S, stride, pad, ldp(X1), ldp(X2))
    mbits = None
    if lazy is not None:
        with _probe("igemm_tn", flops, 1, ("fwd_bnrelu_in",) + desc):
            lib.conv2d_fwd_bnrelu_in(ctx.dt, P(X1), C1, ldp(X1), N, H, W, P(pc.wk), K, P(lazy.sc), P(lazy.sh), P(b),
                                     int(relu), P(y), ldp(y), P(st[0] if st else None), ctx.stream)
    elif head is not None and (FUSE_HEAD and x2 is None and relu and st is None and b is not None and
                               head.bias is not None and K == 64 and
                               C1 == 64 and (R, S, stride, pad) == (3, 3, 1, 1) and
                               _q("conv2d_fwd_head_ok", ctx.dt, ldp(X1), N, H, W, ldp(y), head.weight.shape[0])):
        Kh = head.weight.shape[0]
        logits = torch.empty((N, Kh, Pq, Qq), dtype=torch.float32, device=ctx.device)
        with _probe("igemm_tn", flops, 1, ("fwd",) + desc):
            lib.conv2d_fwd_head(ctx.dt, P(X1), ldp(X1), N, H, W, P(pc.wk), P(b), P(y), ldp(y), Kh, P(head.weight),
                                P(head.bias), P(logits), ctx.stream)
        head = (head, logits)
    else:
        head = None
        if (RELU_BITS and FUSE and relu and b is not None and x2 is None and st is None and ctx.training and
                ctx.tape is not None and K == 64 and C1 == 64 and (R, S, stride, pad) == (3, 3, 1, 1) and
                _q("conv2d_fwd_mask", ctx.dt, 0, ldp(X1), N, H, W, 0, 0, 0, ldp(y), 0, 0) == 1):
            mbits = torch.empty(M * 8, dtype=torch.uint8, device=ctx.device)
            with _probe("igemm_tn", flops, 1, ("fwd",) + desc):
                rc = lib.conv2d_fwd_mask(ctx.dt, P(X1), ldp(X1), N, H, W, P(pc.wk), P(b), P(y), ldp(y), P(mbits),
                                         ctx.stream)
            if rc != 0:
                raise RuntimeError(f"unetseg_conv2d_fwd_mask failed ({rc}): {lib_last_error()}")
        else:
            with _probe("igemm_tn", flops, 1, ("fwd",) + desc):
                lib.conv2d_fwd(ctx.dt, P(X1), C1, ldp(X1), P(X2), C2, ldp(X2), N, H, W, P(pc.wk), K, R, S, stride,
                               pad, P(b), int(relu), P(y), ldp(y), P(st[0] if st else None), ctx.stream)
    out = Node(y)
    out.head = head
    if x2 is None and pc.padk(ctx.dt):
        out.kpad = -(-K // 64) * 64
    if mbits is not None:
        out.mbits = mbits
    if relu:
        out.fuse = (1, y, None)
    _tap(ctx, "conv", out, [x1, x2], conv=pc.conv, relu=relu)

    def bwd():
        dA = out.grad
        if dA is None:
            return
        dev = ctx.device
        if relu and out.fused is not None:
            # the consumer's dgrad stored the masked gradient and the bias partials
            part, rows = out.fused
            dY = dA
            if b is not None:
                part, rows, _ = _merge_rows(ctx, part, K, rows, 2)
                lib.colsum_rows(P(part), K, rows, 0, P(b.grad), 1, ctx.stream)
        elif relu:
            Gr = _q("reduce_tiles", ctx.dt, M, K, None, None)
            part = ctx.f32(K, Gr)
            dY = ctx.empty(N, Pq, Qq, K)
            lib.relu_bwd_bias(ctx.dt, P(dA), ldp(dA), P(y), ldp(y), P(dY), K, M, K, P(part), Gr, ctx.stream)
            if b is not None:
                lib.colsum_finalize(P(part), K, Gr, P(b.grad), 1, ctx.stream)
        else:
            assert b is None, "conv with bias and no ReLU is not on the hot path"
            dY = dA
        # 1x1 convs with a narrow output (the attention gates' theta/phi, K = inter = 32): both
        # gradient GEMMs reduce over or produce K, below the fast tiles' 64-channel granule, so dY
        # is zero-padded to Kp channels and the padded rows of dW / columns of W^T are zero.  The
        # consumer's backward wrote dY into the zeroed padded buffer (out.kpad, gbuf); a gradient
        # adopted from elsewhere is copied into one
        Kp = K
        if out.kpad:
            Kp = out.kpad
            if out.gpad is not None and dY is out.grad:
                dY = out.gpad
            else:
                dYp = torch.zeros(N, Pq, Qq, Kp, dtype=ctx.tdtype, device=dev)
                lib.add(ctx.dt, P(dY), ldp(dY), P(dYp), Kp, M, K, ctx.stream)
                dY = dYp
        cin = C1 + C2

        def launch_wgrad(serial=False):
            """weight gradient: on the side stream when overlapping (it only needs dY and the inputs,
            and nothing in the data-gradient chain reads its output); returns that stream or None"""
            ws_bytes = _q("conv2d_wgrad_workspace", ctx.dt, N, Pq, Qq, Kp, cin, R, S)
            side = None if serial else ctx.side
            if side is not None:
                lib.stream_wait(side.cuda_stream, ctx.stream)
                # dY, the inputs and the input prologue's BN coefficients may be freed (compute-stream
                # order) before the wgrad has run on the side stream, which lags the compute stream
                for t in (dY, X1, X2) + ((lazy.sc, lazy.sh) if lazy is not None else ()):
                    if t is not None:
                        t.record_stream(side)
                ws = workspace(ws_bytes, dev, 1)
                wst = side.cuda_stream
            else:
                ws = workspace(ws_bytes, dev)
                wst = ctx.stream
            if Kp != K:
                # the Kp-row GEMM (dY's padded columns are zero) reduced straight into the K-row gradient
                with _probe("wgrad", flops, 1, ("wgrad_padk",) + desc, stream=side):
                    lib.conv2d_wgrad_rows(ctx.dt, P(X1), C1, ldp(X1), N, H, W, P(dY), Kp, Kp, 1, 1, 1, 0, P(ws),
                                          ws.numel(), P(pc.conv.weight.grad), pc.C, 1, K, wst)
            elif lazy is not None:
                with _probe("wgrad", flops, 1, ("wgrad_bnrelu_in",) + desc, stream=side):
                    lib.conv2d_wgrad_bnrelu_in(ctx.dt, P(X1), C1, ldp(X1), N, H, W, P(dY), ldp(dY), K, P(lazy.sc),
                                               P(lazy.sh), P(ws), ws.numel(), P(pc.conv.weight.grad), pc.C, 1, wst)
            else:
                with _probe("wgrad", flops, 1, ("wgrad",) + desc, stream=side):
                    lib.conv2d_wgrad(ctx.dt, P(X1), C1, ldp(X1), P(X2), C2, ldp(X2), N, H, W, P(dY), ldp(dY), K, R, S,
                                     stride, pad, P(ws), ws.numel(), P(pc.conv.weight.grad), pc.C, 1, wst)
            return side

        deferred = defer_wgrad(ctx, N, Pq, Qq, R, S, x2)
        serial = not deferred and ((bool(WG_SERIAL_HW) and Pq * Qq >= WG_SERIAL_HW and R * S > 1) or
                                   layer in WG_SERIAL_LAYERS)
        wstream = None
        after = WG_AFTER_DGRAD and not deferred and not serial
        if not deferred and not serial and not after:
            wstream = launch_wgrad()
        # data gradient (reads the packed weight pc.wt: the parameter is reported done after it)
        if Kp != K:
            if x1.need_grad:
                assert pc.kld == Kp, "the padded-K data gradient reads the Kp-wide packed wt (PackedConv.kld)"
                g, acc = gbuf(ctx, x1)
                with _probe("igemm_tn", flops, 1, ("dgrad_padk",) + desc):
                    lib.conv2d_dgrad(ctx.dt, P(dY), Kp, N, Pq, Qq, P(pc.wt), Kp, C1, 1, 1, 1, 0, P(g), ldp(g), H, W,
                                     acc, ctx.stream)
        elif x2 is None:
            assert pc.wt is None or pc.kld == K, "a plain data gradient reads K-wide wt rows (PackedConv.kld)"
            if x1.need_grad and not _dgrad_fused(ctx, x1, dY, pc, N, H, W, C1, Pq, Qq, flops, desc, last_grad):
                g, acc = gbuf(ctx, x1)
                with _probe("igemm_tn", flops, _dgrad_launches(ctx, ldp(dY), N, Pq, Qq, K, C1, R, S, stride, pad, H, W),
                            ("dgrad",) + desc):
                    lib.conv2d_dgrad(ctx.dt, P(dY), ldp(dY), N, Pq, Qq, P(pc.wt), K, C1, R, S, stride, pad, P(g),
                                     ldp(g), H, W, acc, ctx.stream)
        elif x1.need_grad or x2.need_grad:
            assert pc.wt is None or pc.kld == K, "a concat data gradient reads K-wide wt rows (PackedConv.kld)"
            g = ctx.empty(N, H, W, cin)
            with _probe("igemm_tn", flops, _dgrad_launches(ctx, ldp(dY), N, Pq, Qq, K, cin, R, S, stride, pad, H, W),
                        ("dgrad",) + desc):
                lib.conv2d_dgrad(ctx.dt, P(dY), ldp(dY), N, Pq, Qq, P(pc.wt), K, cin, R, S, stride, pad, P(g), cin,
                                 H, W, 0, ctx.stream)
            give_grad(ctx, x1, g[..., :C1])
            give_grad(ctx, x2, g[..., C1:])
        if after:
            wstream = launch_wgrad()  # the side stream waits for the data gradient just enqueued
        if serial:
            launch_wgrad(serial=True)  # after the data gradient, on the compute stream
        if deferred:
            def late():
                ctx.param_done(pc.conv.weight, stream=launch_wgrad())
                ctx.param_done(b)
            ctx.deferred.append(late)
        else:
            # the side stream's last launch is still this wgrad (only the data gradient, on the compute
            # stream, was enqueued since)
            ctx.param_done(pc.conv.weight, stream=wstream)
            ctx.param_done(b)

    ctx.push(bwd)
    return out, st


#: eval-mode BatchNorm folded into the preceding conv (UNETSEG_NO_BN_FOLD=1: separate BN pass)
BN_FOLD = os.environ.get("UNETSEG_NO_BN_FOLD", "0") != "1"


def conv_bn(ctx, x, pc, bnm, x2=None, lazy=False):
    """relu(BN(conv(cat[x, x2]))) for a conv whose only consumer is that BN (model/resnet_backbone.py:
    58-61 bottleneck conv1/conv2, model/unet_plain.py:8-15 DoubleConv).  Training: the conv writes
    BN partial statistics in its epilogue, then the BN-ReLU pass (or, lazy, the consumer applies it on
    load; see bn).  Eval in fp32 (the reference's
    evaluate / val / predict precision; no autograd tape): BN and ReLU run in the conv's epilogue on
    the fp32 accumulator, one launch (unetseg_conv2d_fwd_affine with unetseg_bn_fold's coefficients,
    the same float arithmetic as the separate pass, so the result is unchanged).  bf16 eval keeps
    the separate pass: its kernels round the conv output before BN, which is what the bf16
    emulation in the parity tests models."""
    if ctx.training or ctx.tape is not None or not BN_FOLD or ctx.dt != DT_F32:
        y, st = conv(ctx, x, pc, x2=x2, stats=True)
        return bn(ctx, y, st, bnm, relu=True, lazy=lazy)
    K, C, R, S = pc.K, pc.C, pc.R, pc.S
    kscale, bias = ctx.f32(K), ctx.f32(K)
    lib.bn_fold(K, P(bnm.weight), P(bnm.bias), P(bnm.running_mean), P(bnm.running_var), bnm.eps, P(pc.conv.bias),
                P(kscale), P(bias), ctx.stream)
    use(x, x2)
    X1, X2 = x.data, (x2.data if x2 is not None else None)
    N, H, W, C1 = X1.shape
    C2 = X2.shape[-1] if X2 is not None else 0
    stride, pad = pc.conv.stride, pc.conv.padding
    Pq, Qq = (H + 2 * pad - R) // stride + 1, (W + 2 * pad - S) // stride + 1
    y = ctx.empty(N, Pq, Qq, K)
    desc = (N, H, W, C1, C2, K, R, S, stride, pad, ldp(X1), ldp(X2))
    with _probe("igemm_tn", 2.0 * N * Pq * Qq * K * C * R * S, 1, ("fwd_affine",) + desc):
        lib.conv2d_fwd_affine(ctx.dt, P(X1), C1, ldp(X1), P(X2), C2, ldp(X2), N, H, W, P(pc.wk), K, R, S, stride, pad,
                              P(kscale), P(bias), 1, P(y), K, ctx.stream)
    return Node(y)


#: the residual BN-add-ReLU backward's first pass in the next block's conv1 data gradient
#: (unetseg_conv2d_dgrad_post_res; UNETSEG_NO_POST_RES=1: separate bn_bwd_reduce pass)
FUSE_RES = os.environ.get("UNETSEG_NO_POST_RES", "0") != "1"
#: ... also when the block output has more consumers than the next block (a layer's last block: the next
#: layer's downsample conv and the decoder's skip concat) (UNETSEG_NO_POST_RES_MULTI=1: next block only)
FUSE_RES_MULTI = os.environ.get("UNETSEG_NO_POST_RES_MULTI", "0") != "1"


def _dgrad_fused_res(ctx, x1, dY, pc, N, H, W, C1, Pq, Qq, flops, desc, last_grad):
    """x1 is a bottleneck output relu(BN3(y3) + residual) (model/resnet_backbone.py:110-113) consumed by
    this 1x1 conv (the next block's conv1) and by others whose gradients are already in x1.grad (the
    next block's residual add; for a layer's last block, the next layer's downsample conv and the
    decoder's skip concat): when this conv delivers the last contribution, accumulate the dgrad onto
    x1.grad, mask with the stored ReLU bits and write BN3's backward partials in the epilogue (and the
    downsample BN's, block 0) -- the producer's bn_bwd_reduce pass over the gradient is not run."""
    if not (FUSE_RES and x1.fuse is not None and x1.fuse[0] == 3 and x1.grad is not None and last_grad and
            (x1.uses == 2 or (FUSE_RES_MULTI and x1.uses > 2)) and ctx.dt == DT_BF16 and (pc.R, pc.S) == (1, 1) and pc.conv.stride in (1, (1, 1)) and
            x1.grad.stride(-1) == 1 and ldp(x1.grad) % 8 == 0 and H == Pq and W == Qq):
        return False
    _, y3, s1, mbits, y2, s2 = x1.fuse
    K = pc.K
    g = x1.grad
    rows = _q("conv2d_dgrad_post_res", ctx.dt, 0, ldp(dY), N, Pq, Qq, 0, K, C1, 0, ldp(g), 0, ldp(y3),
              0, 0, 0, 0, 0, 0, 0, 0, 0, 0)
    if rows <= 0:
        return False
    nq = 3 if y2 is not None else 2
    part = ctx.f32(rows, nq, C1)
    with _probe("igemm_tn", flops, 1, ("dgrad_post3",) + desc):
        lib.conv2d_dgrad_post_res(ctx.dt, P(dY), ldp(dY), N, Pq, Qq, P(pc.wt), K, C1, P(g), ldp(g), P(y3), ldp(y3),
                                  P(s1.mean), P(s1.inv), P(mbits), P(y2), ldp(y2), P(s2.mean if s2 else None),
                                  P(s2.inv if s2 else None), P(part), rows, ctx.stream)
    x1.fused = (part, rows, nq)
    return True


def _dgrad_fused(ctx, x1, dY, pc, N, H, W, C1, Pq, Qq, flops, desc, last_grad=False):
    """dgrad into x1.grad with the backward mask + first reduction of the ReLU / BN-ReLU that
    produced x1 fused into the epilogue.  Only when this conv is x1's sole consumer (so its dgrad
    is x1's whole gradient) and the shape has a fused kernel; returns False otherwise."""
    if _dgrad_fused_res(ctx, x1, dY, pc, N, H, W, C1, Pq, Qq, flops, desc, last_grad):
        return True
    if not (FUSE and x1.fuse is not None and x1.fuse[0] != 3 and x1.grad is None and x1.uses == 1 and
            ctx.dt == DT_BF16):
        return False
    kind, aux, st = x1.fuse
    K, R, S = pc.K, pc.R, pc.S
    stride, pad = pc.conv.stride, pc.conv.padding
    args = [ctx.dt, P(dY), ldp(dY), N, Pq, Qq, P(pc.wt), K, C1, R, S, stride, pad]
    coeffs = [P(st.sc), P(st.sh), P(st.mean), P(st.inv)] if kind == 2 else [0, 0, 0, 0]
    qargs = (ctx.dt, 0, ldp(dY), N, Pq, Qq, 0, K, C1, R, S, stride, pad, 0, C1, H, W)
    rows = -1
    if kind == 1 and x1.mbits is not None:
        # the producer stored its ReLU mask as bits: post 4 reads them instead of the activation
        rows = _q("conv2d_dgrad_post", *qargs, 4, 0, 0, 0, 0, 0, 0, 0, 0, 0)
        if rows > 0:
            kind, aux = 4, x1.mbits
    if rows <= 0:
        rows = _q("conv2d_dgrad_post", *qargs, kind, 0, ldp(aux), 0, 0, 0, 0, 0, 0, 0)
    if rows <= 0:
        return False
    g = ctx.empty(N, H, W, C1)
    part = ctx.f32(rows, 2, C1)
    with _probe("igemm_tn", flops, _dgrad_launches(ctx, ldp(dY), N, Pq, Qq, K, C1, R, S, stride, pad, H, W),
                (f"dgrad_post{kind}",) + desc):
        rc = lib.conv2d_dgrad_post(*args, P(g), C1, H, W, kind, P(aux), 0 if kind == 4 else ldp(aux), *coeffs,
                                   P(part), rows, ctx.stream)
    if rc != 0:
        raise RuntimeError(f"unetseg_conv2d_dgrad_post failed ({rc}): {lib_last_error()}")
    x1.grad = g
    x1.fused = (part, rows)
    return True


def lib_last_error():
    from .lib import last_error
    return last_error()


#: the 7x7/s2 ResNet stem on the fast kernels in bf16 (UNETSEG_NO_FAST_STEM=1: generic conv path)
STEM_FAST = os.environ.get("UNETSEG_NO_FAST_STEM", "0") != "1"


def stem_conv(ctx, x, conv_mod):
    """model/resnet_backbone.py:126-131 ``conv1`` (7x7, stride 2, pad 3, no bias) from the NCHW fp32
    image batch, bf16 only: the input is packed width-padded so one filter row's 8 taps x 8 channels
    are 128 contiguous bytes, and the conv runs as a K = 7 x 64 implicit GEMM on the fast kernels
    (unetseg_stem_fwd / unetseg_stem_wgrad).  Returns (Node y, BN partial stats) like conv()."""
    x = x.contiguous()
    if x.dtype != torch.float32:
        x = x.float()
    N, C, H, W = x.shape
    K = conv_mod.weight.shape[0]
    xp = ctx.empty(N, H, W + 8, 8)
    lib.pack_input_stem(P(x), N, C, H, W, P(xp), ctx.stream)
    wk = ctx.empty(K, 7, 64)
    lib.stem_pack_weight(P(conv_mod.weight), K, C, P(wk), ctx.stream)
    Pq, Qq = (H - 1) // 2 + 1, (W - 1) // 2 + 1
    M = N * Pq * Qq
    y = ctx.empty(N, Pq, Qq, K)
    tile = lib.stem_fwd_tile_m(N, H, W, K)
    st = (ctx.f32(math.ceil(M / tile), 2, K), tile)
    flops = 2.0 * M * K * C * 49
    desc = (N, H, W, C, 0, K, 7, 7, 2, 3, 8, 0)
    with _probe("igemm_tn", flops, 1, ("stem_fwd",) + desc):
        lib.stem_fwd(P(xp), N, H, W, P(wk), K, P(y), K, P(st[0]), ctx.stream)
    out = Node(y)
    _tap(ctx, "stem", out, [], conv=conv_mod, image=x)

    def bwd():
        dY = out.grad
        if dY is None:
            return
        ws_bytes = lib.stem_wgrad_workspace(N, H, W, K)
        side = None if "stem" in WG_SERIAL_LAYERS else ctx.side
        if side is not None:
            lib.stream_wait(side.cuda_stream, ctx.stream)
            for t in (dY, xp):
                t.record_stream(side)
            ws = workspace(ws_bytes, ctx.device, 1)
            wst = side.cuda_stream
        else:
            ws = workspace(ws_bytes, ctx.device)
            wst = ctx.stream
        with _probe("wgrad", flops, 1, ("stem_wgrad",) + desc, stream=side):
            lib.stem_wgrad(P(xp), N, H, W, P(dY), ldp(dY), K, P(ws), ws.numel(), P(conv_mod.weight.grad), C, 1, wst)
        ctx.param_done(conv_mod.weight, stream=side)

    ctx.push(bwd)
    return out, st


class BNState:
    """per-call BN coefficients"""

    __slots__ = ("mean", "inv", "sc", "sh")


#: finalize row partials with more rows than this (2048: measured best of 512 / 1024 / 2048) are first
#: merged 16 to 1 (unetseg_fin_merge_rows);
#: UNETSEG_FIN_MERGE=0 finalizes them directly
FIN_MERGE_MIN = int(os.environ.get("UNETSEG_FIN_MERGE_MIN", "2048"))
FIN_MERGE = os.environ.get("UNETSEG_FIN_MERGE", "1") != "0"


def _merge_rows(ctx, part, C, G, nq, M=0, tile=0):
    """(partials, rows, tile) for a finalize: large row counts merged 16 to 1 on the device"""
    if not FIN_MERGE or G <= FIN_MERGE_MIN:
        return part, G, tile
    G2 = (G + 15) // 16
    out = ctx.f32(G2, nq, C)
    lib.fin_merge_rows(P(part), C, G, M, tile, nq, P(out), ctx.stream)
    return out, G2, tile * 16


def _bn_coeffs(ctx, bn, st, M, tile=None):
    """st: (partials [G][2][C], row tile) from conv(), or a bare partials tensor with `tile` given"""
    if isinstance(st, tuple):
        st, tile = st
    C = bn.weight.shape[0]
    s = BNState()
    if ctx.training:
        # one allocation for the four coefficient vectors (the host cost of a step is per allocation)
        s.sc, s.sh, s.mean, s.inv = ctx.f32(4, C).unbind(0)
        st, G, tile = _merge_rows(ctx, st, C, st.shape[0], 2, M, tile)
        lib.bn_finalize(P(st), C, G, M, tile, P(bn.weight), P(bn.bias), P(bn.running_mean), P(bn.running_var),
                        P(bn.num_batches_tracked), bn.momentum, bn.eps, P(s.mean), P(s.inv), P(s.sc), P(s.sh),
                        ctx.stream)
    else:
        s.sc, s.sh = ctx.f32(2, C).unbind(0)
        s.mean = s.inv = None
        lib.bn_eval_coeffs(C, P(bn.weight), P(bn.bias), P(bn.running_mean), P(bn.running_var), bn.eps, P(s.sc),
                           P(s.sh), ctx.stream)
    return s


#: residual BN-add-ReLU stores a packed ReLU mask for its backward (UNETSEG_NO_MASK_BITS=1: read the activation)
MASK_BITS = os.environ.get("UNETSEG_NO_MASK_BITS", "0") != "1"

#: BN-ReLU applied by the consuming 1x1 conv on load instead of a separate pass (UNETSEG_NO_BN_PROLOGUE=1: off)
BN_PROLOGUE = os.environ.get("UNETSEG_NO_BN_PROLOGUE", "0") != "1"


def _materialize(ctx, node):
    """store relu(BN(data)) of a lazy node (a consumer that cannot apply it on load)"""
    s = node.lazy
    Y = node.data
    N, H, W, C = Y.shape
    a = ctx.empty(N, H, W, C)
    lib.bn_apply(ctx.dt, P(Y), ldp(Y), P(s.sc), P(s.sh), 0, 0, 0, 0, 0, 1, P(a), C, N * H * W, C, ctx.stream)
    node.data = a
    node.lazy = None


def bn(ctx, y, st, bnm, relu=True, res=None, res_bn=None, lazy=False):
    """a = act(BN(y) [+ res | + BN2(y2)]).  y: conv output Node with partial stats st.
    res: raw residual Node; res_bn: (Node y2, stats2, bn module 2).  lazy (plain BN-ReLU in bf16
    training): no apply pass -- the returned node carries y and the coefficients, and its consumer
    (a 1x1 conv: model/resnet_backbone.py:62 conv3 after bn2) applies BN-ReLU on load, forward and
    weight gradient; the backward below needs only y, so nothing else changes."""
    use(y, res, res_bn[0] if res_bn is not None else None)
    Y = y.data
    N, H, W, C = Y.shape
    M = N * H * W
    s1 = _bn_coeffs(ctx, bnm, st, M)
    mode, R, s2 = 0, None, None
    if res is not None:
        mode, R = 1, res.data
    elif res_bn is not None:
        mode, R = 2, res_bn[0].data
        s2 = _bn_coeffs(ctx, res_bn[2], res_bn[1], M)
    mbits = None
    if lazy and BN_PROLOGUE and relu and mode == 0 and ctx.training and ctx.dt == DT_BF16:
        out = Node(Y)
        out.lazy = s1
    elif MASK_BITS and relu and mode != 0 and ctx.training and ctx.dt == DT_BF16:
        # residual BN-add-ReLU: the backward reads the packed ReLU mask (1/16 of the activation)
        a = ctx.empty(N, H, W, C)
        mbits = torch.empty(M * (C // 8), dtype=torch.uint8, device=ctx.device)
        lib.bn_apply_mask(ctx.dt, P(Y), ldp(Y), P(s1.sc), P(s1.sh), P(R), ldp(R), P(s2.sc if s2 else None),
                          P(s2.sh if s2 else None), mode, P(a), C, M, C, P(mbits), ctx.stream)
        out = Node(a)
        # a consumer conv that delivers this output's gradient last may run BN3's backward pass 1
        # (and the downsample BN's) in its data-gradient epilogue (_dgrad_fused_res)
        out.fuse = (3, Y, s1, mbits, res_bn[0].data if res_bn is not None else None, s2)
    else:
        a = ctx.empty(N, H, W, C)
        lib.bn_apply(ctx.dt, P(Y), ldp(Y), P(s1.sc), P(s1.sh), P(R), ldp(R), P(s2.sc if s2 else None),
                     P(s2.sh if s2 else None), mode, int(relu), P(a), C, M, C, ctx.stream)
        out = Node(a)
    _tap(ctx, "bn", out, [y, res, res_bn[0] if res_bn is not None else None], bn=bnm,
         bn2=res_bn[2] if res_bn is not None else None, relu=relu, lazy=out.lazy is not None)
    plain_relu = relu and res is None and res_bn is None
    if plain_relu and ctx.training:
        out.fuse = (2, Y, s1)

    def bwd():
        dA = out.grad
        if dA is None:
            return
        if not ctx.training:
            raise NotImplementedError("backward through eval-mode BatchNorm is not on the hot path")
        if out.fused is not None and len(out.fused) == 3:
            # residual BN-add-ReLU: the next block's conv1 dgrad stored dz = mask * dA in dA's buffer and
            # the (sum dz, sum dz*xhat1 [, sum dz*xhat2]) row partials (_dgrad_fused_res)
            part, rows, nq = out.fused
            part, rows, _ = _merge_rows(ctx, part, C, rows, nq)
            coef = ctx.f32(6, C)
            b2 = res_bn[2] if res_bn is not None else None
            y2 = res_bn[0] if res_bn is not None else None
            lib.bn_bwd_finalize_rows_res(P(part), C, rows, M, nq - 1, P(bnm.weight), P(s1.inv), P(bnm.weight.grad),
                                         P(bnm.bias.grad), P(b2.weight if b2 else None), P(s2.inv if s2 else None),
                                         P(b2.weight.grad if b2 else None), P(b2.bias.grad if b2 else None), P(coef),
                                         ctx.stream)
            ctx.param_done(bnm.weight, bnm.bias)
            if b2 is not None:
                ctx.param_done(b2.weight, b2.bias)
            dy1, acc1 = gbuf(ctx, y)
            assert acc1 == 0
            dy2 = Y2 = None
            if y2 is not None:
                Y2 = y2.data
                dy2, acc2 = gbuf(ctx, y2)
                assert acc2 == 0
            if res is not None and res.need_grad:
                # the residual gradient IS dz: the block input's gradient starts as this buffer (the
                # block's conv1 dgrad accumulates onto it later; nothing reads dz after this apply)
                assert res.grad is None
                res.grad = dA
            lib.bn_bwd_apply(ctx.dt, P(dA), ldp(dA), 0, C, 0, 0, P(Y), ldp(Y), P(s1.mean), P(s1.inv), P(dy1), ldp(dy1),
                             P(Y2), ldp(Y2), P(s2.mean if s2 else None), P(s2.inv if s2 else None), P(dy2), ldp(dy2),
                             P(coef), 0, 0, 0, M, C, ctx.stream)
            return
        if out.fused is not None:
            # the consumer's dgrad stored dz = dA * mask and the (sum dz, sum dz*xhat) row partials
            part, rows = out.fused
            part, rows, _ = _merge_rows(ctx, part, C, rows, 2)
            coef = ctx.f32(6, C)
            lib.bn_bwd_finalize_rows(P(part), C, rows, M, P(bnm.weight), P(s1.inv), P(bnm.weight.grad),
                                     P(bnm.bias.grad), P(coef), ctx.stream)
            ctx.param_done(bnm.weight, bnm.bias)
            dy1, acc1 = gbuf(ctx, y)
            assert acc1 == 0
            lib.bn_bwd_apply(ctx.dt, P(dA), ldp(dA), 0, C, 0, 0, P(Y), ldp(Y), P(s1.mean), P(s1.inv),
                             P(dy1), ldp(dy1), 0, 0, 0, 0, 0, 0, P(coef), 0, 0, 0, M, C, ctx.stream)
            return
        Gr = _q("reduce_tiles", ctx.dt, M, C, None, None)
        part = ctx.f32(3, C, Gr)
        y2 = res_bn[0] if res_bn is not None else None
        Y2 = y2.data if y2 is not None else None
        # plain BN-ReLU: the mask is recomputed from y (no read of the activation)
        plain = relu and res is None and res_bn is None
        mA = 0 if (plain or not relu) else P(out.data)
        lda = C
        if mbits is not None:  # the packed mask written by the forward (lda 0 flags it)
            mA, lda = P(mbits), 0
        msc, msh = (P(s1.sc), P(s1.sh)) if plain else (0, 0)
        lib.bn_bwd_reduce(ctx.dt, P(dA), ldp(dA), mA, lda, msc, msh, P(Y), ldp(Y), P(s1.mean), P(s1.inv),
                          P(Y2), ldp(Y2), P(s2.mean if s2 else None), P(s2.inv if s2 else None), M, C, P(part), Gr,
                          ctx.stream)
        coef = ctx.f32(6, C)
        nb = 2 if y2 is not None else 1
        b2 = res_bn[2] if res_bn is not None else None
        lib.bn_bwd_finalize(P(part), C, Gr, M, nb, P(bnm.weight), P(s1.inv), P(bnm.weight.grad), P(bnm.bias.grad),
                            P(b2.weight if b2 else None), P(s2.inv if s2 else None),
                            P(b2.weight.grad if b2 else None), P(b2.bias.grad if b2 else None), P(coef), ctx.stream)
        ctx.param_done(bnm.weight, bnm.bias)
        if b2 is not None:
            ctx.param_done(b2.weight, b2.bias)
        dy1, acc1 = gbuf(ctx, y)
        assert acc1 == 0
        dy2 = None
        if y2 is not None:
            dy2, acc2 = gbuf(ctx, y2)
            assert acc2 == 0
        dz, dzacc = None, 0
        if res is not None and res.need_grad:
            dz, dzacc = gbuf(ctx, res)
        lib.bn_bwd_apply(ctx.dt, P(dA), ldp(dA), mA, lda, msc, msh, P(Y), ldp(Y), P(s1.mean), P(s1.inv),
                         P(dy1), ldp(dy1), P(Y2), ldp(Y2), P(s2.mean if s2 else None), P(s2.inv if s2 else None),
                         P(dy2), ldp(dy2), P(coef), P(dz), ldp(dz), dzacc, M, C, ctx.stream)

    ctx.push(bwd)
    return out


def pool_out(h, k, s, ceil_mode):
    """ATen pooling_output_shape (pad 0, dilation 1)"""
    o = (h - k + (s - 1 if ceil_mode else 0)) // s + 1
    if ceil_mode and (o - 1) * s >= h:
        o -= 1
    return o


def maxpool(ctx, x, k, s, ceil_mode):
    use(x)
    X = x.data
    N, H, W, C = X.shape
    Pq, Qq = pool_out(H, k, s, ceil_mode), pool_out(W, k, s, ceil_mode)
    y = ctx.empty(N, Pq, Qq, C)
    idx = torch.empty((N, Pq, Qq, C), dtype=torch.uint8, device=ctx.device)
    lib.maxpool_fwd(ctx.dt, P(X), ldp(X), N, H, W, C, k, s, int(ceil_mode), P(y), C, P(idx), 0, 0, ctx.stream)
    out = Node(y)
    _tap(ctx, "maxpool", out, [x], k=k, s=s, ceil_mode=ceil_mode)

    def bwd():
        if out.grad is None or not x.need_grad:
            return
        g, acc = gbuf(ctx, x)
        lib.maxpool_bwd(ctx.dt, P(out.grad), ldp(out.grad), P(idx), N, H, W, C, k, s, Pq, Qq, P(g), ldp(g), acc,
                        ctx.stream)

    ctx.push(bwd)
    return out


def upsample2x(ctx, x, align_corners):
    use(x)
    X = x.data
    N, H, W, C = X.shape
    y = ctx.empty(N, 2 * H, 2 * W, C)
    lib.upsample2x_fwd(ctx.dt, P(X), ldp(X), N, H, W, C, int(align_corners), P(y), C, ctx.stream)
    out = Node(y)
    _tap(ctx, "resize", out, [x], size=(2 * H, 2 * W), align_corners=bool(align_corners))

    def bwd():
        if out.grad is None or not x.need_grad:
            return
        _upsample_bwd(ctx, x, out.grad, align_corners)

    ctx.push(bwd)
    return out


def _upsample_bwd(ctx, x, gout, align_corners):
    """x.grad (+)= the backward of y = upsample2x(x) for the gradient gout of y"""
    X = x.data
    N, H, W, C = X.shape
    if (FUSE and FUSE_UP and ctx.dt == DT_BF16 and x.fuse is not None and x.fuse[0] == 1 and x.fuse[1] is X
            and x.grad is None and x.uses == 1):
        # x is a ReLU output consumed only here (unetUp conv2 -> next block's upsample): its
        # backward mask and the producer conv's bias-gradient partials ride along
        rows = _q("upsample2x_bwd_tiles", ctx.dt, N, H, W, C)
        g = ctx.empty(N, H, W, C)
        part = ctx.f32(rows, 2, C)
        lib.upsample2x_bwd_relu(ctx.dt, P(gout), ldp(gout), N, H, W, C, int(align_corners), P(X), ldp(X), P(g),
                                ldp(g), P(part), rows, ctx.stream)
        x.grad = g
        x.fused = (part, rows)
        return
    g, acc = gbuf(ctx, x)
    lib.upsample2x_bwd(ctx.dt, P(gout), ldp(gout), N, H, W, C, int(align_corners), P(g), ldp(g), acc, ctx.stream)


def resize_bilinear(ctx, x, oh, ow, align_corners):
    """F.interpolate(x, size=(oh, ow), mode="bilinear") for sizes that are not an exact x2
    (model/unet_attention.py:31-33,52-53, model/unet_dualdense.py:57-58)"""
    use(x)
    X = x.data
    N, H, W, C = X.shape
    y = ctx.empty(N, oh, ow, C)
    lib.resize_bilinear_fwd(ctx.dt, P(X), ldp(X), N, H, W, C, oh, ow, int(align_corners), P(y), C, ctx.stream)
    out = Node(y)
    _tap(ctx, "resize", out, [x], size=(oh, ow), align_corners=bool(align_corners))

    def bwd():
        if out.grad is None or not x.need_grad:
            return
        g, acc = gbuf(ctx, x)
        lib.resize_bilinear_bwd(ctx.dt, P(out.grad), ldp(out.grad), N, H, W, C, oh, ow, int(align_corners), P(g),
                                ldp(g), acc, ctx.stream)

    ctx.push(bwd)
    return out


def pad2d(ctx, x, top, left, oh, ow):
    """F.pad(x, [left, right, top, bottom]) with zeros (model/unet_plain.py:42-45)"""
    use(x)
    X = x.data
    N, H, W, C = X.shape
    y = ctx.empty(N, oh, ow, C)
    lib.pad2d_fwd(ctx.dt, P(X), ldp(X), N, H, W, C, top, left, oh, ow, P(y), C, ctx.stream)
    out = Node(y)
    _tap(ctx, "pad", out, [x], top=top, left=left, size=(oh, ow))

    def bwd():
        if out.grad is None or not x.need_grad:
            return
        g, acc = gbuf(ctx, x)
        lib.pad2d_bwd(ctx.dt, P(out.grad), ldp(out.grad), N, H, W, C, top, left, oh, ow, P(g), ldp(g), acc,
                      ctx.stream)

    ctx.push(bwd)
    return out


def match_hw(ctx, x, skip, mode):
    """x resized ("interpolate", align_corners=False) or zero-padded ("pad", centred as the
    reference's F.pad) to skip's spatial size; x itself when the sizes already agree"""
    h, w = x.data.shape[1:3]
    sh, sw = skip.data.shape[1:3]
    if (h, w) == (sh, sw):
        return x
    if mode == "pad":
        dh, dw = sh - h, sw - w
        if dh < 0 or dw < 0:
            raise RuntimeError(f"pad-then-cat needs the upsampled map ({h}x{w}) no larger than the skip ({sh}x{sw})")
        return pad2d(ctx, x, dh // 2, dw // 2, sh, sw)
    return resize_bilinear(ctx, x, sh, sw, False)


def pw_head(ctx, x, conv_mod):
    """1x1 conv head -> fp32 NCHW logits (the reference's output layout): Cout in {1, 2} on the
    vectorised pw_small kernels (binary / multitask heads), 3..32 classes (the multiclass task's
    outc / final, model/unet_resnet.py:78, model/unet_plain.py:69) on pw_head"""
    use(x)
    X = x.data
    N, H, W, C = X.shape
    K = conv_mod.weight.shape[0]
    M = N * H * W
    if x.head is not None and x.head[0] is conv_mod:
        y = x.head[1]  # computed by the producing conv's epilogue (conv(..., head=conv_mod))
    elif K > 2:
        y = torch.empty((N, K, H, W), dtype=torch.float32, device=ctx.device)
        lib.pw_head_fwd(ctx.dt, P(X), ldp(X), M, H * W, C, K, P(conv_mod.weight), P(conv_mod.bias), P(y), ctx.stream)
    else:
        y = torch.empty((N, K, H, W), dtype=torch.float32, device=ctx.device)
        lib.pw_small_fwd(ctx.dt, P(X), ldp(X), M, H * W, C, K, P(conv_mod.weight), P(conv_mod.bias), P(y), 0,
                         ctx.stream)
    holder = {}
    _tap(ctx, "head", y, [x], conv=conv_mod, holder=holder)

    def bwd():
        dy = holder.get("grad")
        if dy is None:
            return
        dy = dy.contiguous().float()
        if K > 2:
            G = lib.pw_head_tiles(M)
            pw, pb = ctx.f32(K, C, G), ctx.f32(K, G)
            dx, acc = (gbuf(ctx, x) if x.need_grad else (None, 0))
            lib.pw_head_bwd(ctx.dt, P(dy), P(X), ldp(X), M, H * W, C, K, P(conv_mod.weight), P(dx), ldp(dx), acc,
                            P(pw), P(pb), ctx.stream)
            lib.colsum_finalize(P(pw), K * C, G, P(conv_mod.weight.grad), 1, ctx.stream)
            lib.colsum_finalize(P(pb), K, G, P(conv_mod.bias.grad), 1, ctx.stream)
            ctx.param_done(conv_mod.weight, conv_mod.bias)
            return
        G = _q("pw_small_tiles", M)
        pw, pb = ctx.f32(K, C, G), ctx.f32(K, G)
        if (FUSE and x.need_grad and x.fuse is not None and x.fuse[0] == 1 and x.fuse[1] is X
                and x.grad is None and x.uses == 1 and ctx.dt == DT_BF16):
            # x is a ReLU output consumed only here: its backward mask and the producer conv's
            # bias-gradient partials ride along (conv() reads them back from x.fused)
            dx = ctx.empty(N, H, W, C)
            part = ctx.f32(G, 2, C)
            lib.pw_small_bwd_relu(ctx.dt, P(dy), P(X), ldp(X), M, H * W, C, K, P(conv_mod.weight), P(dx), ldp(dx),
                                  P(pw), P(pb), P(part), ctx.stream)
            x.grad = dx
            x.fused = (part, G)
        else:
            dx, acc = (gbuf(ctx, x) if x.need_grad else (None, 0))
            lib.pw_small_bwd(ctx.dt, P(dy), P(X), ldp(X), M, H * W, C, K, P(conv_mod.weight), P(dx), ldp(dx), acc,
                             P(pw), P(pb), ctx.stream)
        lib.colsum_finalize(P(pw), K * C, G, P(conv_mod.weight.grad), 1, ctx.stream)
        lib.colsum_finalize(P(pb), K, G, P(conv_mod.bias.grad), 1, ctx.stream)
        ctx.param_done(conv_mod.weight, conv_mod.bias)

    ctx.push(bwd)
    return y, holder


def attention_gate(ctx, skip, gate, gm, pth, pph):
    """model/unet_attention.py:30-35.  gm: AttentionGate container; pth/pph: packed theta/phi convs.
    Returns the gated skip Node (skip * alpha).  A gate of another size is first resized to the
    skip's (bilinear, align_corners=False, unet_attention.py:31-33)."""
    gate = match_hw(ctx, gate, skip, "interpolate")
    use(skip)  # read again by attn_apply
    th, st_t = conv(ctx, skip, pth, stats=True)
    ph, st_p = conv(ctx, gate, pph, stats=True)
    f = bn(ctx, th, st_t, gm.theta[1], relu=True, res_bn=(ph, st_p, gm.phi[1]))
    F_ = f.data
    N, H, W, Ci = F_.shape
    M = N * H * W
    psi_conv, psi_bn = gm.psi[0], gm.psi[1]
    psi = ctx.f32(M)
    G = lib.pw_small_tiles(M)
    pst = ctx.f32(G, 2, 1)
    lib.pw_small_fwd(ctx.dt, P(F_), ldp(F_), M, M, Ci, 1, P(psi_conv.weight), P(psi_conv.bias), P(psi),
                     P(pst) if ctx.training else 0, ctx.stream)
    s = _bn_coeffs(ctx, psi_bn, pst, M, lib.pw_small_tile(M))
    S_ = skip.data
    Cs = S_.shape[-1]
    alpha = ctx.f32(M)
    gated = ctx.empty(N, H, W, Cs)
    lib.attn_apply(ctx.dt, P(S_), ldp(S_), P(psi), P(s.sc), P(s.sh), P(alpha), P(gated), Cs, M, Cs, ctx.stream)
    out = Node(gated)
    _tap(ctx, "attn", out, [f, skip], psi_conv=psi_conv, psi_bn=psi_bn, psi=psi, alpha=alpha)

    def bwd():
        dg = out.grad
        if dg is None:
            return
        dpsibn = ctx.f32(M)
        G1 = lib.attn_bwd1_tiles(M)
        part = ctx.f32(3, 1, G1)
        ds, dsacc = gbuf(ctx, skip)
        lib.attn_bwd1(ctx.dt, P(dg), ldp(dg), P(S_), ldp(S_), P(alpha), P(psi), P(s.mean), P(s.inv), P(ds), ldp(ds),
                      dsacc, P(dpsibn), M, Cs, P(part), ctx.stream)
        coef = ctx.f32(6, 1)
        lib.bn_bwd_finalize(P(part), 1, G1, M, 1, P(psi_bn.weight), P(s.inv), P(psi_bn.weight.grad),
                            P(psi_bn.bias.grad), 0, 0, 0, 0, P(coef), ctx.stream)
        ctx.param_done(psi_bn.weight, psi_bn.bias)
        dzf, acc = gbuf(ctx, f)
        assert acc == 0
        pw, pb = ctx.f32(Ci, G), ctx.f32(1, G)
        lib.attn_bwd2(ctx.dt, P(dpsibn), P(psi), P(s.mean), P(s.inv), P(coef), P(F_), ldp(F_), P(psi_conv.weight),
                      P(dzf), ldp(dzf), M, Ci, P(pw), P(pb), ctx.stream)
        lib.colsum_finalize(P(pw), Ci, G, P(psi_conv.weight.grad), 1, ctx.stream)
        lib.colsum_finalize(P(pb), 1, G, P(psi_conv.bias.grad), 1, ctx.stream)
        ctx.param_done(psi_conv.weight, psi_conv.bias)

    ctx.push(bwd)
    return out


def cls_head(ctx, feat, head, dropout_mask=None, seed=0):
    """model/unet_multitask.py:73-80: GAP -> FC 2048->512 -> ReLU -> Dropout(0.5) -> FC 512->3"""
    use(feat)
    X = feat.data
    N, H, W, C = X.shape
    fc1, fc2 = head[2], head[5]
    p_drop = head[4].p if ctx.training else 0.0
    O1, O2 = fc1.weight.shape[0], fc2.weight.shape[0]
    g = ctx.f32(N, C)
    lib.gap_fwd(ctx.dt, P(X), ldp(X), N, H * W, C, P(g), ctx.stream)
    pre, h, mask = ctx.f32(N, O1), ctx.f32(N, O1), ctx.f32(N, O1)
    act = 2 if ctx.training else 1
    if dropout_mask is not None:
        dropout_mask = dropout_mask.to(device=ctx.device, dtype=torch.float32).contiguous()
    lib.linear_fwd(P(g), P(fc1.weight), P(fc1.bias), N, C, O1, act, p_drop, seed, P(dropout_mask), P(mask), P(pre),
                   P(h), ctx.stream)
    y = torch.empty((N, O2), dtype=torch.float32, device=ctx.device)
    lib.linear_fwd(P(h), P(fc2.weight), P(fc2.bias), N, O1, O2, 0, 0.0, 0, 0, 0, 0, P(y), ctx.stream)
    holder = {}
    _tap(ctx, "cls", y, [feat], fc1=fc1, fc2=fc2, p_drop=p_drop, keep=mask, pre=pre, hidden=h, holder=holder)

    def bwd():
        dy = holder.get("grad")
        if dy is None:
            return
        dy = dy.contiguous().float()
        dh = ctx.f32(N, O1)
        scratch = ctx.f32(N, max(O1, O2))
        lib.linear_bwd(P(dy), 0, 0, 0.0, 0, P(h), P(fc2.weight), N, O1, O2, P(dh), P(fc2.weight.grad),
                       P(fc2.bias.grad), P(scratch), ctx.stream)
        dg = ctx.f32(N, C)
        lib.linear_bwd(P(dh), P(pre), P(mask), p_drop, act, P(g), P(fc1.weight), N, C, O1, P(dg), P(fc1.weight.grad),
                       P(fc1.bias.grad), P(scratch), ctx.stream)
        ctx.param_done(fc2.weight, fc2.bias, fc1.weight, fc1.bias)
        dx, acc = gbuf(ctx, feat)
        lib.gap_bwd(ctx.dt, P(dg), N, H * W, C, P(dx), ldp(dx), acc, ctx.stream)

    ctx.push(bwd)
    return y, holder, mask


# ------------------------------------------------------------------------------------------------
# dense blocks (model/unet_dualdense.py): concatenation buffer, BN-ReLU over its channel prefix
# ------------------------------------------------------------------------------------------------
def copy_into(ctx, src, block, c0):
    """block.data[..., c0:c0+C] = src.data (the block buffer starts zeroed); backward hands the
    matching channel slice of block.grad to src"""
    use(src)
    S_ = src.data
    N, H, W, C = S_.shape
    B_ = block.data
    lib.add(ctx.dt, P(S_), ldp(S_), P(B_[..., c0:]), ldp(B_), N * H * W, C, ctx.stream)

    def bwd():
        if block.grad is None or not src.need_grad:
            return
        give_grad(ctx, src, block.grad[..., c0:c0 + C])

    ctx.push(bwd)


def link_grad(ctx, node, block, c0):
    """at backward time, node.grad := the channel slice of block.grad that node's data occupies
    (node was written into the block buffer by its producer)"""
    C = node.data.shape[-1]

    def bwd():
        if block.grad is not None:
            node.grad = block.grad[..., c0:c0 + C]

    ctx.push(bwd)


STATS_TILE = 256


def bn_relu_prefix(ctx, block, width, bnm, idx=None):
    """a = ReLU(BN(block.data[..., :width])) (model/unet_dualdense.py:9-11: BatchNorm2d + ReLU over the
    dense concatenation) -> new contiguous Node.  idx (LongTensor, device): physical channel of each of
    the BN's logical channels when the buffer holds padding channels (the 3-channel image padded to
    8); padding channels get gamma = beta = 0, i.e. output 0.  Backward adds into block.grad."""
    use(block)
    Y = block.data[..., :width]
    N, H, W, _ = Y.shape
    M = N * H * W
    C = width
    dev = ctx.device
    if idx is None:
        g, b, rm, rv = bnm.weight, bnm.bias, bnm.running_mean, bnm.running_var
    else:
        def phys(v):
            t = torch.zeros(C, dtype=torch.float32, device=dev)
            return t.index_copy_(0, idx, v.detach())
        g, b, rm, rv = phys(bnm.weight), phys(bnm.bias), phys(bnm.running_mean), phys(bnm.running_var)
    s = BNState()
    s.sc, s.sh = ctx.f32(C), ctx.f32(C)
    if ctx.training:
        G = lib.channel_stats_tiles(M, STATS_TILE)
        part = ctx.f32(G, 2, C)
        lib.channel_stats(ctx.dt, P(Y), ldp(Y), M, C, STATS_TILE, P(part), ctx.stream)
        s.mean, s.inv = ctx.f32(C), ctx.f32(C)
        lib.bn_finalize(P(part), C, G, M, STATS_TILE, P(g), P(b), P(rm), P(rv), P(bnm.num_batches_tracked),
                        bnm.momentum, bnm.eps, P(s.mean), P(s.inv), P(s.sc), P(s.sh), ctx.stream)
        if idx is not None:
            with torch.no_grad():
                bnm.running_mean.copy_(rm.index_select(0, idx))
                bnm.running_var.copy_(rv.index_select(0, idx))
    else:
        s.mean = s.inv = None
        lib.bn_eval_coeffs(C, P(g), P(b), P(rm), P(rv), bnm.eps, P(s.sc), P(s.sh), ctx.stream)
    a = ctx.empty(N, H, W, C)
    lib.bn_apply(ctx.dt, P(Y), ldp(Y), P(s.sc), P(s.sh), 0, 0, 0, 0, 0, 1, P(a), C, M, C, ctx.stream)
    out = Node(a)

    def bwd():
        dA = out.grad
        if dA is None:
            return
        if not ctx.training:
            raise NotImplementedError("backward through eval-mode BatchNorm is not on the hot path")
        Gr = lib.reduce_tiles(ctx.dt, M, C, None, None)
        part = ctx.f32(3, C, Gr)
        lib.bn_bwd_reduce(ctx.dt, P(dA), ldp(dA), 0, C, P(s.sc), P(s.sh), P(Y), ldp(Y), P(s.mean), P(s.inv), 0, 0,
                          0, 0, M, C, P(part), Gr, ctx.stream)
        coef = ctx.f32(6, C)
        dg, db = (bnm.weight.grad, bnm.bias.grad) if idx is None else (ctx.f32(C), ctx.f32(C))
        if idx is not None:
            dg.zero_()
            db.zero_()
        lib.bn_bwd_finalize(P(part), C, Gr, M, 1, P(g), P(s.inv), P(dg), P(db), 0, 0, 0, 0, P(coef), ctx.stream)
        if idx is not None:
            with torch.no_grad():
                bnm.weight.grad.add_(dg.index_select(0, idx))
                bnm.bias.grad.add_(db.index_select(0, idx))
        ctx.param_done(bnm.weight, bnm.bias)
        dy = ctx.empty(N, H, W, C)
        lib.bn_bwd_apply(ctx.dt, P(dA), ldp(dA), 0, C, P(s.sc), P(s.sh), P(Y), ldp(Y), P(s.mean), P(s.inv),
                         P(dy), C, 0, 0, 0, 0, 0, 0, P(coef), 0, 0, 0, M, C, ctx.stream)
        if block.grad is None:
            block.grad = torch.zeros_like(block.data)
        G_ = block.grad
        lib.add(ctx.dt, P(dy), C, P(G_), ldp(G_), M, C, ctx.stream)

    ctx.push(bwd)
    return out
