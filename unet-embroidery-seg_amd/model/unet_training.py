"""Losses, init and LR schedule (reference: model/unet_training.py).

Binary losses run on the fused HIP kernels; ``weights_init``/``get_lr_scheduler``/
``set_optimizer_lr`` are host logic restated from the reference.
"""
import math
from functools import partial

import torch

from unetseg_hip import losses


def weights_init(net, init_type="normal", init_gain=0.02):
    """unet_training.py:94-113: Conv* weights N(0, gain), BatchNorm2d gamma N(1, 0.02), beta 0.
    Visits modules in nn.Module.apply order so the torch RNG stream matches the reference's."""

    def init_func(m):
        classname = m.__class__.__name__
        if hasattr(m, "weight") and classname.find("Conv") != -1:
            if init_type == "normal":
                torch.nn.init.normal_(m.weight.data, 0.0, init_gain)
            elif init_type == "xavier":
                torch.nn.init.xavier_normal_(m.weight.data, gain=init_gain)
            elif init_type == "kaiming":
                torch.nn.init.kaiming_normal_(m.weight.data, a=0, mode="fan_in")
            elif init_type == "orthogonal":
                torch.nn.init.orthogonal_(m.weight.data, gain=init_gain)
            else:
                raise NotImplementedError("initialization method [%s] is not implemented" % init_type)
        elif classname.find("BatchNorm2d") != -1:
            torch.nn.init.normal_(m.weight.data, 1.0, 0.02)
            torch.nn.init.constant_(m.bias.data, 0.0)

    print("initialize network with %s type" % init_type)
    with torch.no_grad():
        net.apply(init_func)


def get_lr_scheduler(lr_decay_type, lr, min_lr, total_iters, warmup_iters_ratio=0.05, warmup_lr_ratio=0.1,
                     no_aug_iter_ratio=0.05, step_num=10):
    """unet_training.py:116-189 (YOLOX warm-cos per epoch, or step decay)."""

    def yolox_warm_cos_lr(lr, min_lr, total_iters, warmup_total_iters, warmup_lr_start, no_aug_iter, iters):
        if iters <= warmup_total_iters:
            lr = (lr - warmup_lr_start) * pow(iters / float(warmup_total_iters), 2) + warmup_lr_start
        elif iters >= total_iters - no_aug_iter:
            lr = min_lr
        else:
            lr = min_lr + 0.5 * (lr - min_lr) * (
                1.0 + math.cos(math.pi * (iters - warmup_total_iters) / (total_iters - warmup_total_iters - no_aug_iter)))
        return lr

    def step_lr(lr, decay_rate, step_size, iters):
        if step_size < 1:
            raise ValueError("step_size must above 1.")
        return lr * decay_rate ** (iters // step_size)

    if lr_decay_type == "cos":
        warmup_total_iters = min(max(warmup_iters_ratio * total_iters, 1), 3)
        warmup_lr_start = max(warmup_lr_ratio * lr, 1e-6)
        no_aug_iter = min(max(no_aug_iter_ratio * total_iters, 1), 15)
        return partial(yolox_warm_cos_lr, lr, min_lr, total_iters, warmup_total_iters, warmup_lr_start, no_aug_iter)
    decay_rate = (min_lr / lr) ** (1 / (step_num - 1))
    step_size = total_iters / step_num
    return partial(step_lr, lr, decay_rate, step_size)


def set_optimizer_lr(optimizer, lr_scheduler_func, epoch):
    """unet_training.py:192-199"""
    lr = lr_scheduler_func(epoch)
    for param_group in optimizer.param_groups:
        param_group["lr"] = lr


def bce_with_logits_loss(logits, targets, pos_weight=None):
    """unet_training.py:205-216 on the fused HIP kernel.  logits (N,H,W) or (N,1,H,W)."""
    lg = logits.unsqueeze(1) if logits.dim() == 3 else logits
    return losses._SegLossFn.apply(lg, targets, "bce", pos_weight)


def lovasz_hinge_loss(logits, labels, ignore_index=None, per_image=False):
    """unet_training.py:253-280 (always the per-image mean) on the fused HIP kernel; with
    ignore_index each image's loss runs over its valid pixels only (unet_training.py:268-274).
    A 1-D input is what binary_segmentation_loss hands over after masking (utils/train_and_eval.py:
    172-180): the reference then loops over single pixels, i.e. a per-pixel hinge mean."""
    lg = logits
    if lg.dim() == 1:
        return losses._SegLossFn.apply(lg.view(1, 1, 1, -1), labels.view(1, 1, -1), "lovasz_hinge", None,
                                       2 ** 62)  # no pixel is ignored: the masked kernel's flat path
    if lg.dim() == 2:
        lg, labels = lg.unsqueeze(0), labels.unsqueeze(0)
    if lg.dim() == 3:
        lg = lg.unsqueeze(1)
    if ignore_index is not None:
        return losses._SegLossFn.apply(lg, labels, "lovasz_image_masked", None, int(ignore_index))
    return losses._SegLossFn.apply(lg, labels, "lovasz_hinge", None)


def CE_Loss(inputs, target, cls_weights, num_classes=21):  # noqa: N802 - reference name
    """unet_training.py:9-24: weighted cross entropy, ignore_index = num_classes (fused HIP kernel)"""
    return losses.ce_loss(inputs, target, cls_weights, num_classes)


def Focal_Loss(inputs, target, cls_weights, num_classes=21, alpha=0.5, gamma=2):  # noqa: N802
    """unet_training.py:32-59: -(1-pt)^gamma * alpha * log pt over every pixel (fused HIP kernel)"""
    return losses.focal_loss(inputs, target, cls_weights, num_classes, alpha, gamma)


def Dice_loss(inputs, target, beta=1, smooth=1e-5):  # noqa: N802
    """unet_training.py:67-91: 1 - mean_c F-beta score of softmax vs the one-hot target (fused HIP kernel)"""
    return losses.dice_loss(inputs, target, beta, smooth)
