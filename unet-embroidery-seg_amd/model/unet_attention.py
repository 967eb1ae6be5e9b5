"""``attention_unet`` (reference: model/unet_attention.py:7-90): U-Net whose skips are gated by an
Oktay attention gate alpha = sigmoid(BN(psi(ReLU(BN(theta skip) + BN(phi gate))))), skip * alpha."""
import torch.nn as nn

from unetseg_hip import ops
from unetseg_hip.nn import BatchNorm2d, Conv2d, HipModel, MaxPool2d, ReLU, Seq, Sigmoid, Upsample

from .unet_plain import DoubleConv, run_double_conv


class AttentionGate(nn.Module):
    """unet_attention.py:7-35"""

    def __init__(self, gate_channels: int, skip_channels: int, inter_channels: int):
        super().__init__()
        self.theta = Seq(Conv2d(skip_channels, inter_channels, 1, bias=False), BatchNorm2d(inter_channels))
        self.phi = Seq(Conv2d(gate_channels, inter_channels, 1, bias=False), BatchNorm2d(inter_channels))
        self.psi = Seq(Conv2d(inter_channels, 1, 1, bias=True), BatchNorm2d(1), Sigmoid())
        self.relu = ReLU()

    def forward(self, skip, gate):  # pragma: no cover - container
        raise RuntimeError("AttentionGate is part of a HIP model; call the top-level model")


class UpAttn(nn.Module):
    """unet_attention.py:38-55"""

    def __init__(self, in_channels: int, skip_channels: int, out_channels: int):
        super().__init__()
        self.up = Upsample(scale_factor=2, align_corners=False)
        self.attn = AttentionGate(gate_channels=in_channels, skip_channels=skip_channels,
                                  inter_channels=max(out_channels // 2, 16))
        self.conv = DoubleConv(in_channels + skip_channels, out_channels)

    def forward(self, x, skip):  # pragma: no cover - container
        raise RuntimeError("UpAttn is part of a HIP model; call the top-level model")


class AttentionUNet(HipModel):
    """unet_attention.py:58-89"""

    def __init__(self, num_classes: int = 2, base_channels: int = 64):
        super().__init__()
        b = base_channels
        self.inc = DoubleConv(3, b)
        self.down1 = Seq(MaxPool2d(2), DoubleConv(b, b * 2))
        self.down2 = Seq(MaxPool2d(2), DoubleConv(b * 2, b * 4))
        self.down3 = Seq(MaxPool2d(2), DoubleConv(b * 4, b * 8))
        self.down4 = Seq(MaxPool2d(2), DoubleConv(b * 8, b * 16))
        self.up1 = UpAttn(b * 16, b * 8, b * 8)
        self.up2 = UpAttn(b * 8, b * 4, b * 4)
        self.up3 = UpAttn(b * 4, b * 2, b * 2)
        self.up4 = UpAttn(b * 2, b, b)
        self.outc = Conv2d(b, num_classes, 1)
        self._finalize()

    def _run(self, ctx, x):
        self._pack_weights(ctx, ctx.tape is not None)
        ops.tap_mark(ctx, "inc")
        xs = [run_double_conv(ctx, self.inc, ops.pack_input(ctx, x, 8))]
        for i, d in enumerate((self.down1, self.down2, self.down3, self.down4), start=1):
            ops.tap_mark(ctx, f"down{i}")
            h = ops.maxpool(ctx, xs[-1], 2, 2, False)
            xs.append(run_double_conv(ctx, d[1], h))
        h = xs[4]
        for i, (up, skip) in enumerate(((self.up1, xs[3]), (self.up2, xs[2]), (self.up3, xs[1]), (self.up4, xs[0])),
                                       start=1):
            ops.tap_mark(ctx, f"up{i}")
            u = ops.upsample2x(ctx, h, align_corners=False)
            a = up.attn
            g = ops.attention_gate(ctx, skip, u, a, a.theta[0]._pc, a.phi[0]._pc)
            u = ops.match_hw(ctx, u, skip, "interpolate")  # unet_attention.py:52-53 (odd sizes)
            h = run_double_conv(ctx, up.conv, g, x2=u)
        ops.tap_mark(ctx, "outc")
        logits, holder = ops.pw_head(ctx, h, self.outc)
        ops.tap_mark(ctx, "end")
        ctx.out_holders = [holder]
        return logits
