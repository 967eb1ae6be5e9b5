"""``unet_resnet50`` (reference: model/unet_resnet.py:7-104).

ResNet-50 encoder + four ``unetUp`` blocks.  Each block is cat[skip, up2x(x)] (bilinear,
align_corners=True) -> conv3x3+bias -> ReLU -> conv3x3+bias -> ReLU; the concat is virtual (the
conv's A-loader reads both sources) and bias+ReLU are fused into the conv epilogue.
"""
import torch.nn as nn

from unetseg_hip import ops
from unetseg_hip.nn import Conv2d, HipModel, ReLU, Seq, Upsample

from .resnet_backbone import resnet50, run_resnet


class unetUp(nn.Module):  # noqa: N801 - reference name
    """unet_resnet.py:7-42"""

    def __init__(self, in_size, out_size):
        super().__init__()
        self.conv1 = Conv2d(in_size, out_size, 3, padding=1)
        self.conv2 = Conv2d(out_size, out_size, 3, padding=1)
        self.up = Upsample(scale_factor=2, align_corners=True)
        self.relu = ReLU()

    def forward(self, inputs1, inputs2):  # pragma: no cover - container
        raise RuntimeError("unetUp is part of a HIP model; call the top-level model")


def run_unet_up(ctx, m, skip, x):
    u = ops.upsample2x(ctx, x, align_corners=True)
    h, _ = ops.conv(ctx, skip, m.conv1._pc, x2=u, relu=True)
    h, _ = ops.conv(ctx, h, m.conv2._pc, relu=True)
    return h


def run_resnet_decoder(ctx, m, feats, head=None):
    """unet_resnet.py:92-100 (shared by MultiTaskUNet).  head: the model's 1x1 head conv, fused into
    the last conv's epilogue where the shape allows (ops.pw_head then reuses those logits)"""
    f1, f2, f3, f4, f5 = feats
    ops.flush_point(ctx, "decoder")
    u = f5
    for name, skip in (("up_concat4", f4), ("up_concat3", f3), ("up_concat2", f2), ("up_concat1", f1)):
        ops.tap_mark(ctx, name)
        u = run_unet_up(ctx, getattr(m, name), skip, u)
    ops.tap_mark(ctx, "up_conv")
    u = ops.upsample2x(ctx, u, align_corners=True)
    u, _ = ops.conv(ctx, u, m.up_conv[1]._pc, relu=True)
    u, _ = ops.conv(ctx, u, m.up_conv[3]._pc, relu=True, head=head)
    return u


class Unet(HipModel):
    """unet_resnet.py:46-104"""

    def __init__(self, num_classes=21):
        super().__init__()
        self.resnet = resnet50()
        in_filters = [192, 512, 1024, 3072]
        out_filters = [64, 128, 256, 512]
        self.up_concat4 = unetUp(in_filters[3], out_filters[3])
        self.up_concat3 = unetUp(in_filters[2], out_filters[2])
        self.up_concat2 = unetUp(in_filters[1], out_filters[1])
        self.up_concat1 = unetUp(in_filters[0], out_filters[0])
        self.up_conv = Seq(Upsample(scale_factor=2, align_corners=True),
                           Conv2d(out_filters[0], out_filters[0], 3, padding=1), ReLU(),
                           Conv2d(out_filters[0], out_filters[0], 3, padding=1), ReLU())
        self.final = Conv2d(out_filters[0], num_classes, 1)
        self.num_classes = num_classes
        self._finalize()

    def _run(self, ctx, x):
        self._pack_weights(ctx, ctx.tape is not None)
        feats = run_resnet(ctx, self.resnet, x)
        u = run_resnet_decoder(ctx, self, feats, head=self.final)
        logits, holder = ops.pw_head(ctx, u, self.final)
        ops.tap_mark(ctx, "end")
        ctx.out_holders = [holder]
        return logits
