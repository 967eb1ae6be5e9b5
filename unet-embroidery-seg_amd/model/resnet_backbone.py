"""ResNet-50 encoder (reference: model/resnet_backbone.py:6-217).

Same module tree, parameter names and constructor RNG order as the reference; the forward is the
HIP program in ``run_resnet`` (stem conv7x7/s2 -> BN -> ReLU -> maxpool 3x3/s2 ceil, then
Bottleneck stages [3,4,6,3] with the stride on the 3x3, returning feat1..feat5).
"""
import math

import torch.nn as nn

from unetseg_hip import ops
from unetseg_hip.lib import DT_BF16
from unetseg_hip.nn import AdaptiveAvgPool2d, BatchNorm2d, Conv2d, Linear, MaxPool2d, ReLU, Seq


def conv3x3(in_planes, out_planes, stride=1, groups=1, dilation=1):
    """resnet_backbone.py:6-20"""
    if groups != 1 or dilation != 1:
        raise NotImplementedError("grouped/dilated convs are not on the hot path")
    return Conv2d(in_planes, out_planes, 3, stride=stride, padding=dilation, bias=False)


def conv1x1(in_planes, out_planes, stride=1):
    """resnet_backbone.py:23-33"""
    return Conv2d(in_planes, out_planes, 1, stride=stride, bias=False)


class Bottleneck(nn.Module):
    """resnet_backbone.py:35-115: 1x1 -> 3x3(stride) -> 1x1 (x4), BN after each, residual add, ReLU."""

    expansion = 4

    def __init__(self, inplanes, planes, stride=1, downsample=None, groups=1, base_width=64, dilation=1,
                 norm_layer=None):
        super().__init__()
        width = int(planes * (base_width / 64.0)) * groups
        self.conv1 = conv1x1(inplanes, width)
        self.bn1 = BatchNorm2d(width)
        self.conv2 = conv3x3(width, width, stride, groups, dilation)
        self.bn2 = BatchNorm2d(width)
        self.conv3 = conv1x1(width, planes * self.expansion)
        self.bn3 = BatchNorm2d(planes * self.expansion)
        self.relu = ReLU()
        self.downsample = downsample
        self.stride = stride

    def forward(self, x):  # pragma: no cover - container
        raise RuntimeError("Bottleneck is part of a HIP model; call the top-level model")


def run_bottleneck(ctx, b, x):
    # conv1 is recorded before the downsample conv: in the reversed tape it delivers the last
    # contribution to x.grad (after the decoder's skip concat and the downsample branch), so it can
    # run the previous block's residual BN backward pass 1 in its epilogue (ops._dgrad_fused_res).
    # A stride-2 downsample data gradient that initialises x.grad writes zeros on the parity
    # classes it does not reach.
    a1 = ops.conv_bn(ctx, x, b.conv1._pc, b.bn1)
    yd = sd = None
    if b.downsample is not None:
        yd, sd = ops.conv(ctx, x, b.downsample[0]._pc, stats=True)
    a2 = ops.conv_bn(ctx, a1, b.conv2._pc, b.bn2, lazy=True)  # conv3 applies bn2-ReLU on load
    y3, s3 = ops.conv(ctx, a2, b.conv3._pc, stats=True)
    if b.downsample is not None:
        return ops.bn(ctx, y3, s3, b.bn3, relu=True, res_bn=(yd, sd, b.downsample[1]))
    return ops.bn(ctx, y3, s3, b.bn3, relu=True, res=x)


class ResNet(nn.Module):
    """resnet_backbone.py:118-201"""

    def __init__(self, block, layers, num_classes=1000):
        super().__init__()
        self.inplanes = 64
        self.conv1 = Conv2d(3, 64, 7, stride=2, padding=3, bias=False)
        self.bn1 = BatchNorm2d(64)
        self.relu = ReLU()
        self.maxpool = MaxPool2d(3, 2, 0, ceil_mode=True)
        self.layer1 = self._make_layer(block, 64, layers[0])
        self.layer2 = self._make_layer(block, 128, layers[1], stride=2)
        self.layer3 = self._make_layer(block, 256, layers[2], stride=2)
        self.layer4 = self._make_layer(block, 512, layers[3], stride=2)
        self.avgpool = AdaptiveAvgPool2d(7)
        self.fc = Linear(512 * block.expansion, num_classes)  # consumes RNG like the reference, then dropped
        for m in self.modules():
            if isinstance(m, Conv2d):
                n = m.kernel_size[0] * m.kernel_size[1] * m.out_channels
                m.weight.data.normal_(0, math.sqrt(2.0 / n))
            elif isinstance(m, BatchNorm2d):
                m.weight.data.fill_(1)
                m.bias.data.zero_()

    def _make_layer(self, block, planes, blocks, stride=1):
        downsample = None
        if stride != 1 or self.inplanes != planes * block.expansion:
            downsample = Seq(Conv2d(self.inplanes, planes * block.expansion, 1, stride=stride, bias=False),
                             BatchNorm2d(planes * block.expansion))
        layers = [block(self.inplanes, planes, stride, downsample)]
        self.inplanes = planes * block.expansion
        for _ in range(1, blocks):
            layers.append(block(self.inplanes, planes))
        return Seq(*layers)

    def forward(self, x):  # pragma: no cover - container
        raise RuntimeError("ResNet is part of a HIP model; call the top-level model")


def run_resnet(ctx, r, x):
    """resnet_backbone.py:182-201 -> [feat1, ..., feat5] Nodes"""
    ops.tap_mark(ctx, "stem")
    if ctx.dt == DT_BF16 and ops.STEM_FAST:
        y, st = ops.stem_conv(ctx, x, r.conv1)
    else:
        xin = ops.pack_input(ctx, x, 8)
        y, st = ops.conv(ctx, xin, r.conv1._pc, stats=True)
    feat1 = ops.bn(ctx, y, st, r.bn1, relu=True)
    h = ops.maxpool(ctx, feat1, r.maxpool.kernel_size, r.maxpool.stride, r.maxpool.ceil_mode)
    feats = [feat1]
    for name, layer in (("layer1", r.layer1), ("layer2", r.layer2), ("layer3", r.layer3), ("layer4", r.layer4)):
        ops.flush_point(ctx, name)
        for i in range(len(layer)):
            ops.tap_mark(ctx, f"{name}.{i}")
            h = run_bottleneck(ctx, layer[i], h)
        feats.append(h)
    return feats


def resnet50(**kwargs):
    """resnet_backbone.py:205-217 (avgpool/fc removed)."""
    model = ResNet(Bottleneck, [3, 4, 6, 3], **kwargs)
    del model.avgpool
    del model.fc
    return model
