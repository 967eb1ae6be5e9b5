"""``multitask_unet`` (reference: model/unet_multitask.py:13-139): the unet_resnet50 body with a
1-channel segmentation head and a classification head GAP(feat5) -> FC 2048->512 -> ReLU ->
Dropout(0.5) -> FC 512->3; ``MultiTaskLoss`` = seg BCE (or Lovasz) + w * CE, fused HIP kernels."""
import torch
import torch.nn as nn

from unetseg_hip import losses, ops
from unetseg_hip.plan import Dyn
from unetseg_hip.nn import AdaptiveAvgPool2d, Conv2d, Dropout, Flatten, HipModel, Linear, ReLU, Seq, Upsample

from .resnet_backbone import resnet50, run_resnet
from .unet_resnet import run_resnet_decoder, unetUp  # noqa: F401  (same block as the reference's copy)


class MultiTaskUNet(HipModel):
    """unet_multitask.py:31-106"""

    def __init__(self, num_seg_classes=1, num_cls_classes=3, backbone="resnet50"):
        super().__init__()
        self.num_seg_classes = num_seg_classes
        self.num_cls_classes = num_cls_classes
        if backbone != "resnet50":
            raise ValueError(f"Unsupported backbone: {backbone}")
        self.encoder = resnet50()
        in_filters = [192, 512, 1024, 3072]
        out_filters = [64, 128, 256, 512]
        self.up_concat4 = unetUp(in_filters[3], out_filters[3])
        self.up_concat3 = unetUp(in_filters[2], out_filters[2])
        self.up_concat2 = unetUp(in_filters[1], out_filters[1])
        self.up_concat1 = unetUp(in_filters[0], out_filters[0])
        self.up_conv = Seq(Upsample(scale_factor=2, align_corners=True),
                           Conv2d(out_filters[0], out_filters[0], 3, padding=1), ReLU(),
                           Conv2d(out_filters[0], out_filters[0], 3, padding=1), ReLU())
        self.seg_head = Conv2d(out_filters[0], num_seg_classes, 1)
        self.cls_head = Seq(AdaptiveAvgPool2d(1), Flatten(), Linear(2048, 512), ReLU(), Dropout(0.5),
                            Linear(512, num_cls_classes))
        #: explicit [B, 512] keep-mask for the dropout (parity tests); None -> hash RNG per step
        self.dropout_mask = None
        self._drop_step = 0
        self._finalize()

    def _next_drop_seed(self):
        self._drop_step += 1
        return 0x5EED0000 + self._drop_step

    def _run(self, ctx, x):
        if self.num_seg_classes > 2:
            raise NotImplementedError("HIP seg head supports num_seg_classes <= 2")
        self._pack_weights(ctx, ctx.tape is not None)
        feats = run_resnet(ctx, self.encoder, x)
        ops.tap_mark(ctx, "cls_head")
        # the dropout seed advances every step (a step plan re-evaluates it per replay)
        seed = Dyn(self._next_drop_seed(), self._next_drop_seed)
        cls, cls_holder, _ = ops.cls_head(ctx, feats[4], self.cls_head, self.dropout_mask, seed=seed)
        u = run_resnet_decoder(ctx, self, feats, head=self.seg_head)
        seg, seg_holder = ops.pw_head(ctx, u, self.seg_head)
        ops.tap_mark(ctx, "end")
        ctx.out_holders = [seg_holder, cls_holder]
        return seg, cls


class MultiTaskLoss(nn.Module):
    """unet_multitask.py:109-139: total = seg_loss(seg.squeeze(1), y.float()) + w * CE(cls, c).
    seg_loss_fn None / nn.BCEWithLogitsLoss -> fused BCE kernel; lovasz_hinge_loss -> Lovasz kernel."""

    def __init__(self, seg_loss_fn=None, cls_loss_weight=1.0):
        super().__init__()
        self.seg_loss_fn = seg_loss_fn or nn.BCEWithLogitsLoss()
        self.cls_loss_weight = cls_loss_weight

    def forward(self, seg_logits, cls_logits, seg_targets, cls_targets):
        fn = self.seg_loss_fn
        if isinstance(fn, nn.BCEWithLogitsLoss):
            if fn.pos_weight is not None or fn.weight is not None or fn.reduction != "mean":
                raise NotImplementedError("only the reference's default BCEWithLogitsLoss() is on the hot path")
            kind = "bce"
        elif getattr(fn, "__name__", "") == "lovasz_hinge_loss":
            kind = "lovasz_hinge"
        else:
            raise NotImplementedError(f"unsupported seg loss {fn}")
        return losses.multitask_loss(seg_logits, cls_logits, seg_targets, cls_targets, self.cls_loss_weight, kind)
