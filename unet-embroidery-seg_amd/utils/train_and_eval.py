"""Training / evaluation loops (reference: utils/train_and_eval.py:20-513): binary
(train_one_epoch_binary / evaluate_binary), multiclass (train_one_epoch / evaluate and the four
confusion-matrix metrics) and multitask.

Same signatures, return values and metric definitions as the reference; the losses and the
confusion counts run on fused HIP kernels.  The reference prints every iteration's ``loss.item()``
(a host sync that drains the launch queue each step); here the progress line carries the same
columns but shows the PREVIOUS iteration's loss, read from a pinned copy whose event has completed
while the current step is already queued (``_LaggedLoss``), so the GPU never idles for the print;
the epoch's loss sums accumulate on the device (the same fp64 sum of the same fp32 values) and are
read once per epoch.
"""
import time

import torch
from torch.amp import autocast

from unetseg_hip import losses
from utils.utils import get_lr


class LogColor:
    GREEN = "\033[1;32m"
    YELLOW = "\033[1;33m"
    RED = "\033[1;31m"
    RESET = "\033[0m"
    BLUE = "\033[1;34m"


class _LaggedLoss:
    """the previous step's scalar loss on the host without draining the queue: push() enqueues a
    non-blocking copy of this step's loss into a pinned buffer (two, alternating) and returns the
    value of the step before it, whose copy is complete by the time the current step is queued"""

    def __init__(self):
        self.bufs = None
        self.pending = None
        self.i = 0

    def push(self, loss):
        t = loss.detach().float().reshape(())
        if not t.is_cuda:
            return float(t)
        if self.bufs is None:
            self.bufs = [torch.empty((), dtype=torch.float32, pin_memory=True) for _ in range(2)]
        buf = self.bufs[self.i]
        self.i ^= 1
        buf.copy_(t, non_blocking=True)
        ev = torch.cuda.Event()
        ev.record()
        prev, self.pending = self.pending, (buf, ev)
        if prev is None:
            return None
        prev[1].synchronize()
        return float(prev[0])

    def flush(self):
        if self.pending is None:
            return None
        self.pending[1].synchronize()
        v = float(self.pending[0])
        self.pending = None
        return v


def _progress(epoch, train_epoch, it, n, gpu_used, lv, lr, size, header):
    """the reference's column-aligned progress line (train_and_eval.py:233-257, 373-401); lv: the
    loss printed (the previous iteration's; the epoch's first iteration prints its own at the end)"""
    if header:
        print(f"{LogColor.GREEN}Epoch{LogColor.RESET}{' ' * 12}{LogColor.YELLOW}data_num{LogColor.RESET}{' ' * 12}"
              f"{LogColor.YELLOW}GPU Mem{LogColor.RESET}{' ' * 12}{LogColor.YELLOW}Loss{LogColor.RESET}{' ' * 12}"
              f"{LogColor.YELLOW}LR{LogColor.RESET}{' ' * 12}{LogColor.YELLOW}Image_size{LogColor.RESET}{' ' * 12}")
    if lv is None:
        return
    e, b, g, ls, r = f"{epoch + 1}/{train_epoch}", f"{it}/{n}", f"{gpu_used:.2f} MB", f"{lv:.8f}", f"{lr:.8f}"
    print(f"\r{e}{' ' * (len('Epoch') + 12 - len(e))}{b}{' ' * (len('data_num') + 12 - len(b))}"
          f"{g}{' ' * (len('GPU Mem') + 12 - len(g))}{ls}{' ' * (len('Loss') + 12 - len(ls))}"
          f"{r}{' ' * (len('LR') + 12 - len(r))}{size}", end="", flush=True)


def _binary_logits_from_two_class(output: torch.Tensor) -> torch.Tensor:
    """train_and_eval.py:106-113"""
    if output.dim() != 4 or output.size(1) != 2:
        raise ValueError(f"Expected output shape (N,2,H,W), got {tuple(output.shape)}")
    return output[:, 1, :, :] - output[:, 0, :, :]


def _binary_confusion_from_pred(pred: torch.Tensor, target: torch.Tensor, ignore_index=None):
    """train_and_eval.py:116-137 (pred already thresholded; helper kept for API parity)"""
    if ignore_index is not None:
        valid = target != ignore_index
        pred, target = pred[valid], target[valid]
    pf, tf = pred == 1, target == 1
    tp = torch.logical_and(pf, tf).sum().item()
    fp = torch.logical_and(pf, ~tf).sum().item()
    fn = torch.logical_and(~pf, tf).sum().item()
    tn = torch.logical_and(~pf, ~tf).sum().item()
    return tp, fp, fn, tn


def binary_segmentation_metrics(tp: float, fp: float, fn: float, tn: float, eps: float = 1e-7):
    """train_and_eval.py:140-152"""
    precision = tp / (tp + fp + eps)
    recall = tp / (tp + fn + eps)
    dice = (2.0 * tp) / (2.0 * tp + fp + fn + eps)
    iou = tp / (tp + fp + fn + eps)
    accuracy = (tp + tn) / (tp + tn + fp + fn + eps)
    return {"Dice": float(dice), "IoU": float(iou), "Precision": float(precision), "Recall": float(recall),
            "Accuracy": float(accuracy)}


def binary_segmentation_loss(outputs, targets, loss_name: str, pos_weight=None, ignore_index=None):
    """train_and_eval.py:155-182 -> fused HIP kernel (2-class difference fused)."""
    return losses.binary_segmentation_loss(outputs, targets, loss_name, pos_weight, ignore_index)


def train_one_epoch_binary(model, optimizer, train_loader, device, loss_name: str, pos_weight, gpu_used, scaler, epoch,
                           train_epoch, ignore_index=None, max_batches=None):
    """train_and_eval.py:185-263"""
    epoch_loss = torch.zeros((), dtype=torch.float64, device=device)
    lag = _LaggedLoss()
    seen_batches = 0
    model_train = model.train().to(device)
    n_batches = len(train_loader)
    for iteration, batch in enumerate(train_loader):
        imgs, pngs = batch[0], batch[1]
        imgs = imgs.to(device, non_blocking=True)
        pngs = pngs.to(device, non_blocking=True)
        optimizer.zero_grad()
        if scaler is None:
            outputs = model_train(imgs)
            loss = binary_segmentation_loss(outputs, pngs, loss_name, pos_weight, ignore_index)
            loss.backward()
            optimizer.step()
        else:
            with autocast(device_type=device.type, enabled=True):
                outputs = model_train(imgs)
                loss = binary_segmentation_loss(outputs, pngs, loss_name, pos_weight, ignore_index)
            scaler.scale(loss).backward()
            scaler.step(optimizer)
            scaler.update()
        epoch_loss += loss.detach().double()
        seen_batches += 1
        _progress(epoch, train_epoch, iteration, n_batches, gpu_used, lag.push(loss), get_lr(optimizer), imgs.shape[2],
                  iteration == 0)
        if max_batches is not None and seen_batches >= max_batches:
            break
    if seen_batches:  # an empty loader returns 0 like the reference (nothing to report)
        _progress(epoch, train_epoch, seen_batches, n_batches, gpu_used, lag.flush(), get_lr(optimizer), imgs.shape[2],
                  False)
    print(f"{LogColor.GREEN}")
    time.sleep(0.2)
    return float(epoch_loss.item()) / max(seen_batches, 1)


def evaluate_binary(model, val_loader, device, loss_name: str, pos_weight, ignore_index=None, max_batches=None):
    """train_and_eval.py:266-305: eval-mode fp32 forward, global tp/fp/fn/tn, metrics with eps 1e-7."""
    model_eval = model.eval().to(device)
    total_loss = torch.zeros((), dtype=torch.float64, device=device)
    conf = torch.zeros(4, dtype=torch.int64, device=device)
    seen_batches = 0
    with torch.no_grad():
        for batch in val_loader:
            imgs, pngs = batch[0].to(device), batch[1].to(device)
            outputs = model_eval(imgs)
            loss = binary_segmentation_loss(outputs, pngs, loss_name, pos_weight, ignore_index)
            total_loss += loss
            losses.binary_confusion(outputs, pngs, conf, ignore_index)
            seen_batches += 1
            if max_batches is not None and seen_batches >= max_batches:
                break
    tp, fp, fn, tn = (float(v) for v in conf.tolist())
    metrics = binary_segmentation_metrics(tp, fp, fn, tn)
    metrics["Loss"] = float(total_loss.item() / max(seen_batches, 1))
    return metrics


def train_one_epoch_multitask(model, optimizer, train_loader, device, criterion, scaler, amp=True, max_batches=None,
                              hook=None):
    """train.py:225-250 (the reference keeps this loop inline): autocast fwd, fused BCE/Lovasz + CE,
    scaled backward, step.  Loss sums and the cls-accuracy counters stay on the device; one host read
    at the end of the epoch.  Returns (loss, seg_loss, cls_loss, cls_acc%) averaged like the reference
    (sums / len(train_loader))."""
    model.train()
    sums = torch.zeros(3, dtype=torch.float64, device=device)
    correct = torch.zeros((), dtype=torch.int64, device=device)
    total = 0
    for batch_idx, batch in enumerate(train_loader):
        if max_batches and batch_idx >= max_batches:
            break
        images, seg_targets, _, cls_targets = batch
        images, seg_targets, cls_targets = images.to(device), seg_targets.to(device), cls_targets.to(device)
        with autocast(device_type=device.type, enabled=amp and device.type == "cuda"):
            seg_logits, cls_logits = model(images)
            loss, seg_loss, cls_loss = criterion(seg_logits, cls_logits, seg_targets, cls_targets)
        optimizer.zero_grad()
        if scaler is not None:
            scaler.scale(loss).backward()
            scaler.step(optimizer)
            scaler.update()
        else:
            loss.backward()
            optimizer.step()
        sums += torch.stack([loss.detach(), seg_loss.detach(), cls_loss.detach()]).double()
        correct += cls_logits.detach().argmax(1).eq(cls_targets).sum()
        total += cls_targets.size(0)
        if hook is not None:
            hook(batch_idx)
    n = max(len(train_loader), 1)
    l, sl, cl = (float(v) / n for v in sums.tolist())  # the epoch's one host read ...
    losses.raise_if_soft_targets(device)  # ... and the check of the no-sync soft-label flag
    return l, sl, cl, 100.0 * float(correct.item()) / max(total, 1)


def evaluate_multitask(model, loader, device, criterion, max_batches=None):
    """train.py:294-355 / val.py:73-110: eval-mode forward; seg IoU = I/(U+1e-6), Dice = 2I/(|P|+|T|+1e-6)
    with P = sigmoid(seg) > 0.5 (fused confusion kernel, u64 counts on the device); cls accuracy %."""
    model.eval()
    sums = torch.zeros(3, dtype=torch.float64, device=device)
    conf = torch.zeros(4, dtype=torch.int64, device=device)
    correct = torch.zeros((), dtype=torch.int64, device=device)
    total = 0
    with torch.no_grad():
        for batch_idx, batch in enumerate(loader):
            if max_batches and batch_idx >= max_batches:
                break
            images, seg_targets, _, cls_targets = batch
            images, seg_targets, cls_targets = images.to(device), seg_targets.to(device), cls_targets.to(device)
            seg_logits, cls_logits = model(images)
            loss, seg_loss, cls_loss = criterion(seg_logits, cls_logits, seg_targets, cls_targets)
            sums += torch.stack([loss, seg_loss, cls_loss]).double()
            losses.binary_confusion(seg_logits, seg_targets, conf)
            correct += cls_logits.argmax(1).eq(cls_targets).sum()
            total += cls_targets.size(0)
    tp, fp, fn, _tn = (float(v) for v in conf.tolist())
    losses.raise_if_soft_targets(device)
    n = max(len(loader), 1)
    l, sl, cl = (float(v) / n for v in sums.tolist())
    return {"Loss": l, "Seg Loss": sl, "Cls Loss": cl, "IoU": tp / (tp + fp + fn + 1e-6),
            "Dice": 2 * tp / ((tp + fp) + (tp + fn) + 1e-6), "Cls Acc": 100.0 * float(correct.item()) / max(total, 1)}


# ------------------------------------------------------------------------------------------------
# multiclass task (train_and_eval.py:20-103, 308-513): metrics from one fused confusion histogram
# per batch (device, u64), losses on the fused CE / Focal / Dice kernels
# ------------------------------------------------------------------------------------------------
def _mc_hist(output, target):
    return losses.mc_confusion(output, target).cpu().numpy()


def pixel_accuracy(output, target):
    """train_and_eval.py:20-26 (correct / all pixels)"""
    return losses.mc_metrics_from_hist(_mc_hist(output, target))["Pixel Accuracy"]


def mean_accuracy(output, target, num_classes):
    """train_and_eval.py:28-59 (classes present in the target)"""
    return losses.mc_metrics_from_hist(_mc_hist(output, target))["Mean Accuracy"]


def mean_iou(output, target, num_classes):
    """train_and_eval.py:63-81 (classes present in the target)"""
    return losses.mc_metrics_from_hist(_mc_hist(output, target))["Mean IoU"]


def frequency_weighted_iou(output, target, num_classes):
    """train_and_eval.py:85-103"""
    return losses.mc_metrics_from_hist(_mc_hist(output, target))["Frequency Weighted IoU"]


def _mc_loss(outputs, pngs, labels, weights, num_classes, dice_loss, focal_loss):
    from model.unet_training import CE_Loss, Dice_loss, Focal_Loss
    if focal_loss:
        loss = Focal_Loss(outputs, pngs, weights, num_classes=num_classes)
    else:
        loss = CE_Loss(outputs, pngs, weights, num_classes=num_classes)
    if dice_loss:
        loss = loss + Dice_loss(outputs, labels)
    return loss


def train_one_epoch(model, optimizer, train_loader, device, dice_loss, focal_loss, gpu_used, num_classes, scaler,
                    epoch, train_epoch):
    """train_and_eval.py:308-409: CE or Focal (+ Dice) with unit class weights; returns the mean loss"""
    import numpy as np
    cls_weights = np.ones([num_classes], np.float32)
    epoch_loss = torch.zeros((), dtype=torch.float64, device=device)
    lag = _LaggedLoss()
    model_train = model.train().to(device)
    weights = torch.tensor(cls_weights).to(device)
    n_batches = len(train_loader)
    for iteration, batch in enumerate(train_loader):
        imgs, pngs, labels = batch[0].to(device), batch[1].to(device), batch[2].to(device)
        optimizer.zero_grad()
        if scaler is None:
            outputs = model_train(imgs)
            loss = _mc_loss(outputs, pngs, labels, weights, num_classes, dice_loss, focal_loss)
            loss.backward()
            optimizer.step()
        else:
            with autocast(device_type=device.type, enabled=True):
                outputs = model_train(imgs)
                loss = _mc_loss(outputs, pngs, labels, weights, num_classes, dice_loss, focal_loss)
            scaler.scale(loss).backward()
            scaler.step(optimizer)
            scaler.update()
        epoch_loss += loss.detach().double()
        _progress(epoch, train_epoch, iteration, n_batches, gpu_used, lag.push(loss), get_lr(optimizer), imgs.shape[2],
                  iteration == 0)
    if n_batches:
        _progress(epoch, train_epoch, n_batches, n_batches, gpu_used, lag.flush(), get_lr(optimizer), imgs.shape[2],
                  False)
    print(f"{LogColor.GREEN}")
    return float(epoch_loss.item()) / max(n_batches, 1)


def evaluate(model, val_loader, device, dice_loss, focal_loss, num_classes):
    """train_and_eval.py:411-513: per-batch metrics averaged over batches, as the reference does"""
    import numpy as np
    weights = torch.tensor(np.ones([num_classes], np.float32)).to(device)
    model_eval = model.eval().to(device)
    hists, loss_sum = [], torch.zeros((), dtype=torch.float64, device=device)
    with torch.no_grad():
        for batch in val_loader:
            imgs, pngs, labels = batch[0].to(device), batch[1].to(device), batch[2].to(device)
            outputs = model_eval(imgs)
            loss_sum += _mc_loss(outputs, pngs, labels, weights, num_classes, dice_loss, focal_loss).double()
            hists.append(losses.mc_confusion(outputs, pngs))
    n = max(len(val_loader), 1)
    keys = ("Pixel Accuracy", "Mean Accuracy", "Mean IoU", "Frequency Weighted IoU")
    tot = dict.fromkeys(keys, 0.0)
    for h in hists:  # one device->host copy per batch histogram, after the loop
        m = losses.mc_metrics_from_hist(h.cpu().numpy())
        for k in keys:
            tot[k] += m[k]
    metrics = {k: tot[k] / n for k in keys}
    metrics["Loss"] = float(loss_sum.item()) / n
    return metrics
