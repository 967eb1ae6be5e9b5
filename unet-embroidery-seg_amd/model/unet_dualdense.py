"""``dualdense_unet`` (reference: model/unet_dualdense.py:5-104): U-Net whose stages are dense
blocks -- each layer is BN -> ReLU -> conv3x3(growth) over the concatenation of the block input and
every earlier layer's output; a 1x1 transition conv + BN + ReLU closes the block.

HIP program: a block owns one NHWC concatenation buffer.  The input is copied into its first
channels and every layer's conv writes its ``growth`` channels straight into the next slot, so the
torch.cat of the reference (unet_dualdense.py:29-33) is never materialised; each layer's BN-ReLU
reads the buffer's channel prefix (batch statistics by ``unetseg_channel_stats``) and the backward
adds every layer's input gradient into the buffer's gradient.  The 3-channel image of ``inc`` is
held padded to 8 channels; its BN parameters and conv weights are re-laid-out onto those physical
channels (zero gamma / weights on the padding).
"""
import torch
import torch.nn as nn

from unetseg_hip import ops
from unetseg_hip.nn import BatchNorm2d, Conv2d, HipModel, MaxPool2d, ReLU, Seq, Upsample


class _DenseLayer(nn.Module):
    """unet_dualdense.py:5-15"""

    def __init__(self, in_channels: int, growth_rate: int):
        super().__init__()
        self.net = Seq(BatchNorm2d(in_channels), ReLU(), Conv2d(in_channels, growth_rate, 3, padding=1, bias=False))

    def forward(self, x):  # pragma: no cover - container
        raise RuntimeError("_DenseLayer is part of a HIP model; call the top-level model")


class DenseBlock(nn.Module):
    """unet_dualdense.py:18-33"""

    def __init__(self, in_channels: int, growth_rate: int, num_layers: int):
        super().__init__()
        self.layers = nn.ModuleList()
        cur = in_channels
        for _ in range(num_layers):
            self.layers.append(_DenseLayer(cur, growth_rate))
            cur += growth_rate
        self.out_channels = cur

    def forward(self, x):  # pragma: no cover - container
        raise RuntimeError("DenseBlock is part of a HIP model; call the top-level model")


class DenseConvBlock(nn.Module):
    """unet_dualdense.py:36-47"""

    def __init__(self, in_channels: int, out_channels: int, growth_rate: int = 32, num_layers: int = 3):
        super().__init__()
        self.dense = DenseBlock(in_channels, growth_rate=growth_rate, num_layers=num_layers)
        self.trans = Seq(Conv2d(self.dense.out_channels, out_channels, 1, bias=False), BatchNorm2d(out_channels), ReLU())

    def forward(self, x):  # pragma: no cover - container
        raise RuntimeError("DenseConvBlock is part of a HIP model; call the top-level model")


class UpDense(nn.Module):
    """unet_dualdense.py:50-61"""

    def __init__(self, in_channels: int, skip_channels: int, out_channels: int, growth_rate: int = 32,
                 num_layers: int = 3):
        super().__init__()
        self.up = Upsample(scale_factor=2, align_corners=False)
        self.conv = DenseConvBlock(in_channels + skip_channels, out_channels, growth_rate=growth_rate,
                                   num_layers=num_layers)

    def forward(self, x, skip):  # pragma: no cover - container
        raise RuntimeError("UpDense is part of a HIP model; call the top-level model")


class _RelaidConv:
    """Stand-in conv whose input channels are re-laid-out onto the padded physical channels of a
    concatenation buffer: weight_phys[:, idx] = weight (zeros elsewhere), refreshed every forward;
    its weight gradient is gathered back onto the logical weight after the conv's backward."""

    def __init__(self, conv, phys_channels):
        self.conv = conv
        self.cphys = phys_channels
        self.stride, self.padding, self.bias = conv.stride, conv.padding, None
        self.weight = None
        self.pc = None

    def refresh(self, ctx, idx):
        K, C, R, S = self.conv.weight.shape
        w = torch.zeros(K, self.cphys, R, S, dtype=torch.float32, device=ctx.device)
        w.index_copy_(1, idx, self.conv.weight.detach())
        self.weight = w
        self.weight.grad = torch.zeros_like(w)
        self.pc = ops.PackedConv(self)
        self.pc.pack(ctx, need_t=ctx.tape is not None)

    def gather_grad(self, ctx, idx):
        """tape hook: logical grad += physical grad[:, idx] once the conv's wgrad has run"""
        conv, relaid = self.conv, self

        def bwd():
            if ctx.side is not None:  # the weight gradient ran on the side stream
                ops.lib.stream_wait(ctx.stream, ctx.side.cuda_stream)
            with torch.no_grad():
                conv.weight.grad.add_(relaid.weight.grad.index_select(1, idx))
            ctx.param_done(conv.weight)

        ctx.push(bwd)


def _phys_index(c_img_logical, c_img_phys, width_logical, device):
    """logical channel -> physical channel of a buffer whose first part (the image) is padded"""
    idx = list(range(c_img_logical)) + [c_img_phys + j for j in range(width_logical - c_img_logical)]
    return torch.tensor(idx, dtype=torch.long, device=device)


def run_dense_conv_block(ctx, blk, parts, img=None):
    """unet_dualdense.py:29-47.  parts: Nodes whose channel concatenation is the block input.
    img = (logical, physical) channels of parts[0] when it is the padded image (inc)."""
    N, H, W = parts[0].data.shape[:3]
    growth = blk.dense.layers[0].net[2].out_channels
    c0 = sum(p.data.shape[-1] for p in parts)
    L = len(blk.dense.layers)
    total = c0 + L * growth
    buf = ops.Node(torch.zeros(N, H, W, total, dtype=ctx.tdtype, device=ctx.device))
    off = 0
    for p in parts:
        ops.copy_into(ctx, p, buf, off)
        off += p.data.shape[-1]
    c_log = c0 if img is None else c0 - (img[1] - img[0])
    for li, layer in enumerate(blk.dense.layers):
        width = c0 + li * growth
        idx = None if img is None else _phys_index(img[0], img[1], c_log + li * growth, ctx.device)
        a = ops.bn_relu_prefix(ctx, buf, width, layer.net[0], idx)
        conv = layer.net[2]
        if img is not None and li > 0:
            rc = _RelaidConv(conv, width)
            rc.refresh(ctx, idx)
            rc.gather_grad(ctx, idx)
            pc = rc.pc
        else:
            pc = conv._pc
        f, _ = ops.conv(ctx, a, pc, out=buf.data[..., width:width + growth])
        ops.link_grad(ctx, f, buf, width)
    tconv, tbn = blk.trans[0], blk.trans[1]
    if img is not None:
        idx = _phys_index(img[0], img[1], c_log + L * growth, ctx.device)
        rc = _RelaidConv(tconv, total)
        rc.refresh(ctx, idx)
        rc.gather_grad(ctx, idx)
        pc = rc.pc
    else:
        pc = tconv._pc
    return ops.conv_bn(ctx, buf, pc, tbn)


class DualDenseUNet(HipModel):
    """unet_dualdense.py:64-103"""

    def __init__(self, num_classes: int = 2, base_channels: int = 64, growth_rate: int = 32, num_layers: int = 3):
        super().__init__()
        b = base_channels
        self.inc = DenseConvBlock(3, b, growth_rate=growth_rate, num_layers=num_layers)
        self.down1 = Seq(MaxPool2d(2), DenseConvBlock(b, b * 2, growth_rate, num_layers))
        self.down2 = Seq(MaxPool2d(2), DenseConvBlock(b * 2, b * 4, growth_rate, num_layers))
        self.down3 = Seq(MaxPool2d(2), DenseConvBlock(b * 4, b * 8, growth_rate, num_layers))
        self.down4 = Seq(MaxPool2d(2), DenseConvBlock(b * 8, b * 16, growth_rate, num_layers))
        self.up1 = UpDense(b * 16, b * 8, b * 8, growth_rate, num_layers)
        self.up2 = UpDense(b * 8, b * 4, b * 4, growth_rate, num_layers)
        self.up3 = UpDense(b * 4, b * 2, b * 2, growth_rate, num_layers)
        self.up4 = UpDense(b * 2, b, b, growth_rate, num_layers)
        self.outc = Conv2d(b, num_classes, 1)
        self.num_classes = num_classes
        self._finalize()
        # inc's convs beyond the first read the padded image: they are packed per forward from a
        # re-laid-out copy (_RelaidConv), not by the model-wide batched pack
        relaid = {id(l.net[2]) for l in list(self.inc.dense.layers)[1:]} | {id(self.inc.trans[0])}
        self._packed = [pc for pc in self._packed if id(pc.conv) not in relaid]
        # the first dense conv reads BN-ReLU(image): its data gradient feeds that BN's parameters
        self.inc.dense.layers[0].net[2]._pc.force_t = True

    def _run(self, ctx, x):
        self._pack_weights(ctx, ctx.tape is not None)
        x0 = ops.pack_input(ctx, x, 8)
        xs = [run_dense_conv_block(ctx, self.inc, [x0], img=(x.shape[1], 8))]
        for d in (self.down1, self.down2, self.down3, self.down4):
            h = ops.maxpool(ctx, xs[-1], 2, 2, False)
            xs.append(run_dense_conv_block(ctx, d[1], [h]))
        h = xs[4]
        for up, skip in ((self.up1, xs[3]), (self.up2, xs[2]), (self.up3, xs[1]), (self.up4, xs[0])):
            u = ops.upsample2x(ctx, h, align_corners=False)
            u = ops.match_hw(ctx, u, skip, "interpolate")  # unet_dualdense.py:57-58 (odd sizes)
            h = run_dense_conv_block(ctx, up.conv, [skip, u])
        logits, holder = ops.pw_head(ctx, h, self.outc)
        ctx.out_holders = [holder]
        return logits
