"""Teacher-forced per-block backward check (test infrastructure for tests/test_gpu_teacher.py).

``Recorder`` is installed as ``unetseg_hip.ops.TAP`` around ONE training step of the real product
path (bf16 kernels, weight gradients on the side stream, held-back concat weight gradients,
per-bucket Adam + re-pack during backward -- everything bench.py runs).  The model code marks block
boundaries (``ops.tap_mark``: the ResNet stem, every bottleneck, every decoder block, the heads), so
the ops between two marks form one *segment*.  During the forward the recorder copies every tensor
the path stores (the bf16 activations, fp32 logits / gate maps / head intermediates); during the
backward a closure at each mark copies the gradients that cross it:

* the gradient arriving at each segment's outputs (HIP's, as stored: bf16 NHWC, possibly already
  masked by a consumer's fused ReLU backward),
* each segment input's gradient before and after the segment's backward ran.

``check_segment`` then rebuilds the segment in float64 torch from those tensors and runs its backward
from HIP's incoming gradient, so every parameter gradient and every input-gradient contribution of
the segment is compared individually -- the chaotic amplification of an end-to-end comparison
(50+ layers of BN backward) never enters.  Forward values are teacher-forced: each op's output
is computed in float64 from the stored inputs (that difference is reported as the op's forward
error) and then replaced by the stored value, whose gradient flows through the float64 op.

``emu=True`` also rounds every gradient to bf16 where the HIP path stores it (every bf16 node's
gradient) and rounds the never-stored BN-ReLU input of the bottleneck conv3 (applied on load), so
the residual difference is accumulation order + the rounding flips it causes.  ``emu=False`` is the
plain float64 backward of the same forward values (the effect of bf16 gradient storage itself).

Reference: model/resnet_backbone.py:80-115, model/unet_resnet.py:25-42,80-104,
model/unet_attention.py:30-55, model/unet_multitask.py:73-106 (what each segment computes).
"""
from __future__ import annotations

import torch
import torch.nn.functional as F

F64 = torch.float64


class _Forced(torch.autograd.Function):
    """value := the stored tensor; the gradient flows to the computed value (rounded to bf16 first
    when ``rnd``: the HIP path stores this node's gradient in bf16)"""

    @staticmethod
    def forward(fctx, computed, stored, rnd):
        fctx.rnd = rnd
        return stored.clone()

    @staticmethod
    def backward(fctx, g):
        if fctx.rnd:
            g = g.to(torch.bfloat16).to(g.dtype)
        return g, None, None


class _RoundGrad(torch.autograd.Function):
    @staticmethod
    def forward(fctx, x):
        return x.clone()

    @staticmethod
    def backward(fctx, g):
        return g.to(torch.bfloat16).to(g.dtype)


def _bf16_value(x):
    """x rounded to bf16 (forward), gradient straight through"""
    return x + (x.to(torch.bfloat16).to(x.dtype) - x).detach()


def nchw64(t, dt=F64):
    """stored node data / gradient (N, H, W, C) -> float64 (or dt) NCHW"""
    return t.to(dt).permute(0, 3, 1, 2).contiguous()


def rel_l2(a, b):
    """||a - b|| / ||b|| (float64); 0 when both are 0"""
    a, b = a.to(F64), b.to(F64)
    nb = b.norm().item()
    d = (a - b).norm().item()
    if nb == 0.0:
        return 0.0 if d == 0.0 else float("inf")
    return d / nb


class Recorder:
    """ops.TAP implementation: see the module docstring"""

    def __init__(self):
        self.idx = {}          # id(obj) -> index (objects kept alive in self.objs until "end")
        self.objs = []         # index -> Node / tensor (dropped at "end")
        self.meta = []         # index -> dict(node=bool, need_grad, lazy, bf16)
        self.stored = {}       # index -> copy of the stored forward value
        self.ops = []          # (segment, kind, out, ins, info)
        self.marks = []        # (name, cell)
        self.caps = []         # per mark: {index: (grad copy or None, fused flag)}
        self.holder_grads = {}  # index of a head / cls output -> incoming gradient (fp32)
        self.done = False

    # -- recording (forward) ------------------------------------------------------------------
    def _id(self, obj, node=True):
        k = id(obj)
        if k not in self.idx:
            self.idx[k] = len(self.objs)
            self.objs.append(obj)
            self.meta.append(dict(node=node, need_grad=getattr(obj, "need_grad", False), lazy=False,
                                  bf16=False))
        return self.idx[k]

    def op(self, ctx, kind, out, ins, info):
        if not self.marks:
            raise RuntimeError(f"op {kind} before the first block mark")
        seg = len(self.marks) - 1
        is_node = not torch.is_tensor(out)
        o = self._id(out, node=is_node)
        m = self.meta[o]
        ii = [self._id(x) if x is not None else None for x in ins]
        info = dict(info)
        if is_node:
            m["need_grad"] = out.need_grad
            m["bf16"] = out.data.dtype == torch.bfloat16
            m["lazy"] = bool(info.get("lazy"))
            if not m["lazy"]:
                self.stored[o] = out.data.detach().clone()
        else:
            self.stored[o] = out.detach().clone()
        for key in ("image", "psi", "alpha", "keep", "pre", "hidden"):
            if key in info:
                info[key] = info[key].detach().clone()
        self.ops.append((seg, kind, o, ii, info))

    def mark(self, ctx, name):
        cell = {}
        k = len(self.marks)
        self.marks.append((name, cell))
        self.caps.append({})
        main = ctx.main

        def capture():
            cap = self.caps[k]
            with torch.cuda.stream(main):
                for i, node in cell.get("nodes", ()):
                    g = node.grad
                    cap[i] = (g.detach().clone() if g is not None else None, node.fused is not None)
                for i, holder in cell.get("holders", ()):
                    g = holder.get("grad")
                    self.holder_grads[i] = g.detach().float().clone() if g is not None else None
            cell.clear()

        ctx.push(capture)
        if name == "end":
            self._finalize()

    def _finalize(self):
        """fill each mark's capture list (node refs live only in the closures' cells, which the
        backward pops as it passes them: no activation outlives its product-path lifetime)"""
        nseg = len(self.marks)
        prod, cons = {}, {}
        for seg, kind, o, ii, info in self.ops:
            prod[o] = seg
            for i in ii:
                if i is not None:
                    cons.setdefault(i, set()).add(seg)
        for k, (name, cell) in enumerate(self.marks):
            want = set()
            for x, segs in cons.items():
                p = prod.get(x, -1)
                later = any(c >= k for c in segs)
                if k in segs and p < k:                      # inputs of the segment after the mark
                    want.add(x)
                if p == k - 1 and later:                     # outputs of the segment before it
                    want.add(x)
                if (k - 1) in segs and p < k - 1 and later:  # inputs of the segment before it, used later
                    want.add(x)
            cell["nodes"] = [(x, self.objs[x]) for x in sorted(want) if self.meta[x]["node"]]
            if k == nseg - 1:
                cell["holders"] = [(o, info["holder"]) for seg, kind, o, ii, info in self.ops
                                   if kind in ("head", "cls")]
        self.prod, self.cons = prod, cons
        self.objs = None  # forward references dropped; the cells hold what the backward needs
        self.done = True

    def segments(self):
        return [(k, name) for k, (name, _) in enumerate(self.marks) if any(o[0] == k for o in self.ops)]

    def outputs(self):
        """(index, stored value) of the model outputs (head / cls ops)"""
        return [(o, self.stored[o]) for seg, kind, o, ii, info in self.ops if kind in ("head", "cls")]


def check_segment(rec, k, weights, hip_grads, emu=True, dt=F64):
    """Rebuild segment k in float64 (or ``dt``: float32 gives the accumulation-noise reference) and
    compare.  weights(p) -> the parameter's value in the forward (pre-step snapshot); hip_grads(p)
    -> its HIP gradient.  Returns a dict of {"params": [(param, rel, reference gradient)], "bias_l1":
    {id(bias): (L1, L2) norms of its gradient's summands},
    "inputs": [(index, rel)], "fwd": [(kind, rel)]}."""
    ops_k = [op for op in rec.ops if op[0] == k]
    vals, leaves, params = {}, {}, {}
    bias_l1 = {}  # id(conv.bias) -> (L1, L2) of d loss / d conv output (the bias gradient's summands)
    fwd = []

    def pleaf(p, rnd):
        if id(p) not in params:
            w = weights(p).to(F64)
            if rnd:
                w = w.to(torch.bfloat16).to(F64)
            w = w.to(dt)
            params[id(p)] = (p, w.requires_grad_(True))
        return params[id(p)][1]

    def val(i):
        if i in vals:
            return vals[i]
        m = rec.meta[i]
        if m["lazy"]:
            raise RuntimeError("a lazy BN-ReLU node crosses a block boundary")
        t = nchw64(rec.stored[i], dt)
        if m["need_grad"]:
            t.requires_grad_(True)
        vals[i] = leaves[i] = t
        return t

    def force(i, computed, stored64, kind, rnd_grad):
        fwd.append((kind, rel_l2(computed.detach(), stored64)))
        return _Forced.apply(computed, stored64, bool(rnd_grad))

    for seg, kind, o, ii, info in ops_k:
        m = rec.meta[o]
        rnd = emu and m["bf16"]
        xs = [val(i) if i is not None else None for i in ii]
        if kind == "input":
            vals[o] = nchw64(rec.stored[o], dt)
            continue
        if kind == "stem":
            conv = info["conv"]
            img = info["image"].to(torch.bfloat16).to(dt)  # the packed bf16 input
            y = F.conv2d(img, pleaf(conv.weight, True), None, conv.stride, conv.padding)
        elif kind == "conv":
            conv = info["conv"]
            x = xs[0] if xs[1] is None else torch.cat([xs[0], xs[1]], 1)
            w = pleaf(conv.weight, True)
            if x.shape[1] > w.shape[1]:  # input channels zero-padded (the packed image)
                x = x[:, :w.shape[1]]
            b = pleaf(conv.bias, False) if conv.bias is not None else None
            y = F.conv2d(x, w, b, conv.stride, conv.padding)
            if b is not None and y.requires_grad:
                # the bias gradient is the sum of these terms: their norms size the rounding of the
                # bf16-stored summands (the bound of an analytically zero bias gradient)
                y.register_hook(lambda g, pid=id(conv.bias): bias_l1.__setitem__(
                    pid, (float(g.abs().sum()), float(g.double().norm()))))
            if info["relu"]:
                y = F.relu(y)
        elif kind == "bn":
            bn, bn2 = info["bn"], info["bn2"]
            y = F.batch_norm(xs[0], None, None, pleaf(bn.weight, False), pleaf(bn.bias, False), True, 0.0, bn.eps)
            if xs[1] is not None:
                y = y + xs[1]
            if xs[2] is not None:
                y = y + F.batch_norm(xs[2], None, None, pleaf(bn2.weight, False), pleaf(bn2.bias, False), True, 0.0,
                                     bn2.eps)
            if info["relu"]:
                y = F.relu(y)
            if m["lazy"]:
                # never stored: the consuming 1x1 conv applies it on load and feeds bf16 to the MFMA;
                # the consumer's data gradient stores this node's (masked) gradient in bf16
                y = _bf16_value(y)
                vals[o] = _RoundGrad.apply(y) if emu else y
                continue
        elif kind == "maxpool":
            y = F.max_pool2d(xs[0], info["k"], info["s"], 0, ceil_mode=info["ceil_mode"])
        elif kind == "resize":
            y = F.interpolate(xs[0], size=info["size"], mode="bilinear", align_corners=info["align_corners"])
        elif kind == "pad":
            x = xs[0]
            oh, ow = info["size"]
            t, lft = info["top"], info["left"]
            y = F.pad(x, [lft, ow - x.shape[3] - lft, t, oh - x.shape[2] - t])
        elif kind == "head":
            conv = info["conv"]
            y = F.conv2d(xs[0], pleaf(conv.weight, False), pleaf(conv.bias, False))
            vals[o] = force(o, y, rec.stored[o].to(dt), kind, False)
            continue
        elif kind == "attn":
            f, skip = xs
            N, _, H, W = f.shape
            pc, pb = info["psi_conv"], info["psi_bn"]
            psi = F.conv2d(f, pleaf(pc.weight, False), pleaf(pc.bias, False))
            if psi.requires_grad:  # the psi bias gradient's summands (see the conv branch)
                psi.register_hook(lambda g, pid=id(pc.bias): bias_l1.__setitem__(
                    pid, (float(g.abs().sum()), float(g.double().norm()))))
            psi = force(o, psi, info["psi"].to(dt).reshape(N, H, W, 1).permute(0, 3, 1, 2), "attn_psi", False)
            s = F.batch_norm(psi, None, None, pleaf(pb.weight, False), pleaf(pb.bias, False), True, 0.0, pb.eps)
            alpha = force(o, torch.sigmoid(s), info["alpha"].to(dt).reshape(N, H, W, 1).permute(0, 3, 1, 2),
                          "attn_alpha", False)
            y = skip * alpha
        elif kind == "cls":
            fc1, fc2 = info["fc1"], info["fc2"]
            g = xs[0].mean(dim=(2, 3))
            pre = force(o, F.linear(g, pleaf(fc1.weight, False), pleaf(fc1.bias, False)), info["pre"].to(dt),
                        "cls_fc1", False)
            h = F.relu(pre) * info["keep"].to(dt) / (1.0 - info["p_drop"])
            h = force(o, h, info["hidden"].to(dt), "cls_hidden", False)
            y = F.linear(h, pleaf(fc2.weight, False), pleaf(fc2.bias, False))
            vals[o] = force(o, y, rec.stored[o].to(dt), kind, False)
            continue
        else:
            raise NotImplementedError(kind)
        vals[o] = force(o, y, nchw64(rec.stored[o], dt), kind, rnd)

    # incoming gradients: the node outputs crossing the next mark, the head / cls outputs' holders
    outs, grads = [], []
    nxt = rec.caps[k + 1] if k + 1 < len(rec.caps) else {}
    for seg, kind, o, ii, info in ops_k:
        if kind in ("head", "cls"):
            g = rec.holder_grads.get(o)
            if g is not None:
                outs.append(vals[o])
                grads.append(g.to(dt))
        elif o in nxt and nxt[o][0] is not None and vals[o].requires_grad:
            outs.append(vals[o])
            grads.append(nchw64(nxt[o][0], dt))
    if outs:
        torch.autograd.backward(outs, grads)

    res = {"params": [], "inputs": [], "fwd": fwd, "bias_l1": bias_l1}
    for p, leaf in params.values():
        ref = leaf.grad if leaf.grad is not None else torch.zeros_like(leaf)
        res["params"].append((p, rel_l2(hip_grads(p), ref), ref.detach()))
    here = rec.caps[k]
    for i, leaf in leaves.items():
        if not rec.meta[i]["need_grad"]:
            continue
        g_after, fused_after = here.get(i, (None, False))
        g_before, fused_before = nxt.get(i, (None, False))
        ref = leaf.grad if leaf.grad is not None else torch.zeros_like(leaf)
        ref = ref.detach()
        if g_before is not None:
            ref = ref + nchw64(g_before)
        if fused_after and not fused_before:
            # a consumer in this segment ran the producer's ReLU backward in its data gradient
            ref = ref * (leaf.detach() > 0)
        if g_after is None:
            r = 0.0 if ref.abs().max().item() == 0 else float("inf")
        else:
            r = rel_l2(nchw64(g_after), ref)
        res["inputs"].append((i, r))
    return res
