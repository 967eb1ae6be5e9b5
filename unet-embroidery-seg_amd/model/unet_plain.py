"""``unet_plain`` (reference: model/unet_plain.py:5-83): classic U-Net, DoubleConv =
2x[conv3x3 (no bias) -> BN -> ReLU], MaxPool2 down, bilinear (align_corners=False) up,
cat[skip, x] (virtual) -> DoubleConv, 1x1 head."""
import torch.nn as nn

from unetseg_hip import ops
from unetseg_hip.nn import BatchNorm2d, Conv2d, HipModel, MaxPool2d, ReLU, Seq, Upsample


class DoubleConv(nn.Module):
    """unet_plain.py:5-18"""

    def __init__(self, in_channels, out_channels):
        super().__init__()
        self.net = Seq(Conv2d(in_channels, out_channels, 3, padding=1, bias=False), BatchNorm2d(out_channels), ReLU(),
                       Conv2d(out_channels, out_channels, 3, padding=1, bias=False), BatchNorm2d(out_channels), ReLU())

    def forward(self, x):  # pragma: no cover - container
        raise RuntimeError("DoubleConv is part of a HIP model; call the top-level model")


def run_double_conv(ctx, dc, x, x2=None):
    a = ops.conv_bn(ctx, x, dc.net[0]._pc, dc.net[1], x2=x2)
    return ops.conv_bn(ctx, a, dc.net[3]._pc, dc.net[4])


class Down(nn.Module):
    """unet_plain.py:21-30"""

    def __init__(self, in_channels, out_channels):
        super().__init__()
        self.net = Seq(MaxPool2d(2, 2), DoubleConv(in_channels, out_channels))

    def forward(self, x):  # pragma: no cover - container
        raise RuntimeError("Down is part of a HIP model; call the top-level model")


class Up(nn.Module):
    """unet_plain.py:33-47"""

    def __init__(self, in_channels, out_channels):
        super().__init__()
        self.up = Upsample(scale_factor=2, align_corners=False)
        self.conv = DoubleConv(in_channels, out_channels)

    def forward(self, x, skip):  # pragma: no cover - container
        raise RuntimeError("Up is part of a HIP model; call the top-level model")


class UNetPlain(HipModel):
    """unet_plain.py:50-82"""

    def __init__(self, num_classes: int = 2, base_channels: int = 64):
        super().__init__()
        b = base_channels
        self.inc = DoubleConv(3, b)
        self.down1 = Down(b, b * 2)
        self.down2 = Down(b * 2, b * 4)
        self.down3 = Down(b * 4, b * 8)
        self.down4 = Down(b * 8, b * 16)
        self.up1 = Up(b * 16 + b * 8, b * 8)
        self.up2 = Up(b * 8 + b * 4, b * 4)
        self.up3 = Up(b * 4 + b * 2, b * 2)
        self.up4 = Up(b * 2 + b, b)
        self.outc = Conv2d(b, num_classes, 1)
        self._finalize()

    def _run(self, ctx, x):
        self._pack_weights(ctx, ctx.tape is not None)
        ops.tap_mark(ctx, "inc")
        xs = [run_double_conv(ctx, self.inc, ops.pack_input(ctx, x, 8))]
        for i, d in enumerate((self.down1, self.down2, self.down3, self.down4), start=1):
            ops.tap_mark(ctx, f"down{i}")
            h = ops.maxpool(ctx, xs[-1], 2, 2, False)
            xs.append(run_double_conv(ctx, d.net[1], h))
        h = xs[4]
        for i, (up, skip) in enumerate(((self.up1, xs[3]), (self.up2, xs[2]), (self.up3, xs[1]), (self.up4, xs[0])),
                                       start=1):
            ops.tap_mark(ctx, f"up{i}")
            u = ops.upsample2x(ctx, h, align_corners=False)
            u = ops.match_hw(ctx, u, skip, "pad")  # unet_plain.py:42-45 (odd sizes)
            h = run_double_conv(ctx, up.conv, skip, x2=u)
        ops.tap_mark(ctx, "outc")
        logits, holder = ops.pw_head(ctx, h, self.outc)
        ops.tap_mark(ctx, "end")
        ctx.out_holders = [holder]
        return logits
