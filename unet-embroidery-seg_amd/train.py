"""Training entry point on the HIP path (reference: train.py:48-600).

Same command line, same `create_model` / `get_optimizer_and_lr` helpers and the same per-epoch
flow: set the warm-cos LR, train (binary: utils.train_and_eval.train_one_epoch_binary; multitask:
the fused seg+cls loop), validate, keep best/last `state_dict`s, write the metric history and a
summary.  Tasks: binary, multiclass (CE / Focal (+ Dice), Mean-IoU model selection) and
multitask.  Differences, all deliberate:
  * the model, losses, metrics and Adam run on hand-written HIP kernels (no CPU fallback);
  * a real `--data-path` reads the HF parquet layout with utils/hf_dataloader.py: DataLoader
    workers decode and draw the augmentation, the pixel work runs on the GPU (DeviceLoader);
    `--data-path synthetic` (the default here: no dataset ships offline) uses the seeded
    synthetic embroidery-like generator;
  * launched under torchrun (WORLD_SIZE > 1) it trains data-parallel over RCCL: rank r takes every
    W-th image, gradients are bucket-averaged during backward (unetseg_hip.ddp.GradBuckets);
  * the test-split visual export (utils/vis_export.py) needs an HF dataset, as the reference's does;
    plots (matplotlib) are out of scope.
"""
from __future__ import annotations

import argparse
import csv
import datetime
import json
import os
import sys
import time

_HERE = os.path.dirname(os.path.abspath(__file__))
if _HERE not in sys.path:
    sys.path.insert(0, _HERE)

import numpy as np  # noqa: E402
import torch  # noqa: E402
import torch.distributed as dist  # noqa: E402
from torch.utils.data import DataLoader  # noqa: E402

from model.model_factory import SUPPORTED_MODELS, build_model, load_weights_flexible  # noqa: E402
from model.unet_multitask import MultiTaskLoss  # noqa: E402
from model.unet_training import get_lr_scheduler, lovasz_hinge_loss, set_optimizer_lr, weights_init  # noqa: E402
from unetseg_hip.arena import FusedAdam  # noqa: E402
from unetseg_hip.ddp import GradBuckets, init_from_env, local_device  # noqa: E402
from utils.hf_dataloader import DeviceLoader, HFUnetDataset, make_collate  # noqa: E402
from utils.vis_export import export_binary_visuals  # noqa: E402
from utils.synthetic import SyntheticSegDataset, collate  # noqa: E402
from utils.train_and_eval import (  # noqa: E402
    evaluate,
    evaluate_binary,
    evaluate_multitask,
    train_one_epoch,
    train_one_epoch_binary,
    train_one_epoch_multitask,
)
from utils.utils import seed_everything, worker_init_fn  # noqa: E402


def create_model(model_name, num_classes, weights, num_seg_classes=1, num_cls_classes=3):
    """train.py:48-59"""
    if model_name == "multitask_unet":
        model = build_model(model_name, num_classes=num_classes, num_seg_classes=num_seg_classes,
                            num_cls_classes=num_cls_classes)
    else:
        model = build_model(model_name, num_classes=num_classes)
    weights_init(model)
    if weights:
        load_weights_flexible(model, weights)
    return model


def get_optimizer_and_lr(model, batch_size, train_epoch, momentum, weight_decay):
    """train.py:62-78: Adam(lr clamped to 1e-4, betas (momentum, 0.999), coupled wd) + warm-cos per epoch.
    The optimizer is FusedAdam: one HIP launch over the model's flat parameter arena, same update."""
    init_lr, min_lr, nbs = 1e-4, 1e-6, 16
    lim_max = lim_min = 1e-4
    init_fit = min(max(batch_size / nbs * init_lr, lim_min), lim_max)
    min_fit = min(max(batch_size / nbs * min_lr, lim_min * 1e-2), lim_max * 1e-2)
    optimizer = FusedAdam(model, lr=init_fit, betas=(momentum, 0.999), weight_decay=weight_decay)
    return optimizer, get_lr_scheduler("cos", init_fit, min_fit, train_epoch)


def _datasets(args, num_classes, rank, world):
    size = [args.input_size, args.input_size]
    cls = args.task == "multitask"
    if args.data_path != "synthetic":  # train.py:115-137
        task = "binary" if args.task == "multitask" else args.task
        mk = lambda split, aug: HFUnetDataset(args.data_path, size, num_classes, augmentation=aug,  # noqa: E731
                                              split=split, config=args.data_config, task=task,
                                              cache_dir=args.cache_dir, return_cls_label=cls)
        return mk("train", True), mk("validation", False), lambda: mk("test", False)
    if args.task == "multiclass":
        raise ValueError("the synthetic set is binary; the multiclass task needs a real --data-path")
    mk = lambda n, seed: SyntheticSegDataset(n, size, num_classes, seed=seed, return_cls_label=cls)  # noqa: E731
    return mk(args.synthetic_train, 1234), mk(args.synthetic_val, 777_000), lambda: mk(args.synthetic_val, 888_000)


class _SeededWorkerInit:
    """worker_init_fn(worker_id, seed) as a picklable callable (train.py:149)"""

    def __init__(self, seed):
        self.seed = seed

    def __call__(self, worker_id):
        worker_init_fn(worker_id, self.seed)


def _loader(ds, args, shuffle, rank, world, device, workers=None):
    sampler = None
    if world > 1:
        sampler = torch.utils.data.distributed.DistributedSampler(ds, world, rank, shuffle=shuffle, seed=args.seed)
        shuffle = False
    workers = args.workers if workers is None else workers
    hf = isinstance(ds, HFUnetDataset)
    dl = DataLoader(ds, batch_size=args.batch_size, shuffle=shuffle, sampler=sampler, num_workers=workers,
                    pin_memory=True, drop_last=False, collate_fn=make_collate(ds) if hf else collate,
                    worker_init_fn=_SeededWorkerInit(args.seed) if workers else None)
    # the fp32 one-hot seg_labels are read by the multiclass Dice term only
    return DeviceLoader(dl, device, onehot=args.task == "multiclass") if hf else dl


def _pos_weight_auto(train_ds, args, device):
    """train.py:190-203: neg/pos over evenly spaced training samples (labels of the augmented items)"""
    n = min(args.pos_weight_samples, len(train_ds))
    pos = neg = 0
    for i in np.linspace(0, len(train_ds) - 1, n, dtype=int):
        png = train_ds.get(int(i), device)[1] if isinstance(train_ds, HFUnetDataset) else train_ds[int(i)][1]
        pos += int((png == 1).sum())
        neg += int((png == 0).sum())
    if pos > 0:
        return torch.tensor([neg / pos], dtype=torch.float32, device=device)
    return None


def train(args):
    rank, world, local = init_from_env("nccl")
    seed_everything(args.seed)
    num_classes = args.num_classes + 1 if args.task == "multiclass" else 2  # train.py:83-92
    device = torch.device("cuda", local_device(local)) if world > 1 else torch.device(args.device)
    if device.type != "cuda" or not torch.cuda.is_available():
        raise RuntimeError("the HIP training path needs a GPU (no CPU fallback)")
    if device.index is None:
        device = torch.device("cuda", torch.cuda.current_device())
    torch.cuda.set_device(device)
    exp_folder = os.path.join(args.out_dir, datetime.datetime.now().strftime("exp_%Y%m%d_%H%M%S"))
    weights_folder = os.path.join(exp_folder, "weights")
    if rank == 0:
        os.makedirs(weights_folder, exist_ok=True)
        with open(os.path.join(exp_folder, "config.json"), "w", encoding="utf-8") as f:
            json.dump(vars(args), f, ensure_ascii=False, indent=2)

    train_ds, val_ds, make_test_ds = _datasets(args, num_classes, rank, world)
    train_loader = _loader(train_ds, args, True, rank, world, device)
    val_loader = _loader(val_ds, args, False, 0, 1, device)

    if args.task == "multitask":
        model = create_model(args.model, num_classes=1, weights=args.weights, num_seg_classes=1, num_cls_classes=3)
    else:
        model = create_model(args.model, num_classes=num_classes, weights=args.weights)
    model = model.to(device)
    buckets = GradBuckets(model) if world > 1 else None  # broadcasts rank 0's weights
    scaler = torch.amp.GradScaler(device.type, enabled=args.amp)
    optimizer, lr_fn = get_optimizer_and_lr(model, args.batch_size, args.epochs, args.momentum, args.weight_decay)

    pos_weight = None
    if args.task == "binary" and args.loss == "bce" and args.pos_weight:
        if args.pos_weight == "auto":
            pos_weight = _pos_weight_auto(train_ds, args, device)
        else:
            pos_weight = torch.tensor([float(args.pos_weight)], dtype=torch.float32, device=device)

    criterion = None
    if args.task == "multitask":
        seg_fn = lovasz_hinge_loss if args.loss == "lovasz_hinge" else torch.nn.BCEWithLogitsLoss()
        criterion = MultiTaskLoss(seg_loss_fn=seg_fn, cls_loss_weight=args.cls_loss_weight)

    mtb = args.max_train_batches or None
    mvb = args.max_val_batches or None
    best_score, best_epoch, best_metrics = -1.0, None, None
    best_path, last_path = os.path.join(weights_folder, "best.pth"), os.path.join(weights_folder, "last.pth")
    train_losses, val_losses, history = [], [], []
    t0 = time.time()
    for epoch in range(args.epochs):
        set_optimizer_lr(optimizer, lr_fn, epoch)
        if isinstance(train_loader.sampler, torch.utils.data.distributed.DistributedSampler):
            train_loader.sampler.set_epoch(epoch)
        if args.task == "multitask":
            loss, sl, cl, acc = train_one_epoch_multitask(model, optimizer, train_loader, device, criterion,
                                                          scaler if args.amp else None, args.amp, mtb)
            if rank == 0:
                print(f"Epoch {epoch + 1}/{args.epochs} - Loss: {loss:.4f} (Seg: {sl:.4f}, Cls: {cl:.4f}), "
                      f"Cls Acc: {acc:.2f}%")
        elif args.task == "binary":
            loss = train_one_epoch_binary(model, optimizer, train_loader, device, loss_name=args.loss,
                                          pos_weight=pos_weight, gpu_used=torch.cuda.memory_allocated() / 2**20,
                                          scaler=scaler if args.amp else None, epoch=epoch, train_epoch=args.epochs,
                                          ignore_index=None, max_batches=mtb)
        else:  # train.py:285-294
            loss = train_one_epoch(model, optimizer, train_loader, device, args.use_dice, args.loss == "focal",
                                   torch.cuda.memory_allocated() / 2**20, num_classes,
                                   scaler if args.amp else None, epoch, args.epochs)
        train_losses.append(loss)
        if buckets is not None:
            buckets.sync_buffers()  # BN running statistics: rank 0's (DDP broadcast_buffers semantics)
        if rank != 0:
            continue
        if args.task == "multitask":
            metrics = evaluate_multitask(model, val_loader, device, criterion, mvb)
            print(f"Val - IoU: {metrics['IoU']:.4f}, Dice: {metrics['Dice']:.4f}, Cls Acc: {metrics['Cls Acc']:.2f}%")
            score = float(metrics["IoU"])
        elif args.task == "binary":
            metrics = evaluate_binary(model, val_loader, device, loss_name=args.loss, pos_weight=pos_weight,
                                      ignore_index=None, max_batches=mvb)
            score = float(metrics["IoU"])
        else:
            metrics = evaluate(model, val_loader, device, args.use_dice, args.loss == "focal", num_classes)
            score = float(metrics["Mean IoU"])
        val_losses.append(metrics["Loss"])
        history.append(metrics)
        if score > best_score:
            best_score, best_epoch, best_metrics = score, epoch + 1, metrics
            torch.save(model.state_dict(), best_path)
            print(f"New best model saved with score: {best_score:.4f}")
        torch.save(model.state_dict(), last_path)

    if rank == 0:
        print(f"Training completed in {datetime.timedelta(seconds=int(time.time() - t0))}")
        test_metrics = None
        if os.path.exists(best_path):
            model.load_state_dict(torch.load(best_path, map_location=device, weights_only=True))
            try:
                test_ds = make_test_ds()
            except FileNotFoundError as e:  # the reference skips the test pass when the split is absent
                print(f"[test] skipped: {e}")
                test_ds = None
            test_loader = _loader(test_ds, args, False, 0, 1, device, max(0, args.workers // 2)) \
                if test_ds is not None else None
            mtest = args.max_test_batches or None
            if test_loader is None:
                pass
            elif args.task == "multitask":
                test_metrics = evaluate_multitask(model, test_loader, device, criterion, mtest)
            elif args.task == "multiclass":
                test_metrics = evaluate(model, test_loader, device, True, False, num_classes)
            else:
                test_metrics = evaluate_binary(model, test_loader, device, loss_name=args.loss, pos_weight=pos_weight,
                                               ignore_index=None, max_batches=mtest)
            with open(os.path.join(exp_folder, "test_metrics.json"), "w", encoding="utf-8") as f:
                json.dump(test_metrics, f, ensure_ascii=False, indent=2)
            # fixed-sample visual export of the test split (train.py:476-486; HF datasets only)
            if args.task in ("binary", "multitask") and args.export_vis and isinstance(test_ds, HFUnetDataset):
                try:
                    export_binary_visuals(model=model, hf_unet_dataset=test_ds, out_dir=os.path.join(exp_folder, "vis"),
                                          input_shape=[args.input_size] * 2, device=device, num_samples=args.vis_num,
                                          seed=args.vis_seed)
                except Exception as e:  # the reference reports and continues (train.py:487-488)
                    print(f"[WARN] Skip test evaluation: {e}")
        with open(os.path.join(exp_folder, "val_metrics_history.json"), "w", encoding="utf-8") as f:
            json.dump(history, f, ensure_ascii=False, indent=2)
        fields = ["epoch"] + [k for k in (history[0] if history else {})]
        with open(os.path.join(exp_folder, "val_metrics_history.csv"), "w", newline="", encoding="utf-8") as f:
            w = csv.DictWriter(f, fieldnames=fields)
            w.writeheader()
            for i, m in enumerate(history, start=1):
                w.writerow({"epoch": i, **m})
        with open(os.path.join(exp_folder, "summary.json"), "w", encoding="utf-8") as f:
            json.dump({"best_epoch": best_epoch, "best_score": float(best_score), "best_val_metrics": best_metrics,
                       "test_metrics": test_metrics, "best_model_path": best_path, "last_model_path": last_path,
                       "train_losses": train_losses, "val_losses": val_losses}, f, ensure_ascii=False, indent=2)
    if buckets is not None:
        dist.barrier()
        dist.destroy_process_group()
    return exp_folder


def parse_args(argv=None):
    """train.py:523-593 (same flags and defaults; data flags default to the synthetic set)."""
    p = argparse.ArgumentParser(description="U-Net training on the MI355X HIP path")
    p.add_argument("--weights", default="", help="pretrained state_dict (flexible load); '' = random init")
    p.add_argument("--data-path", default="synthetic")
    p.add_argument("--data-config", default="no-ai", choices=["full", "no-ai", "sam3"])
    p.add_argument("--task", default="binary", choices=["binary", "multiclass", "multitask"])
    p.add_argument("--model", default="unet_resnet50", choices=sorted(SUPPORTED_MODELS.keys()))
    p.add_argument("--cls-loss-weight", default=1.0, type=float)
    p.add_argument("--loss", default="lovasz_hinge", choices=["bce", "lovasz_hinge", "ce", "focal"])
    p.add_argument("--pos-weight", default="auto")
    p.add_argument("--pos-weight-samples", default=80, type=int)
    p.add_argument("--use-dice", action=argparse.BooleanOptionalAction, default=True)
    p.add_argument("--num-classes", default=4, type=int)
    p.add_argument("--device", default="cuda")
    p.add_argument("--batch-size", default=8, type=int)
    p.add_argument("--epochs", default=50, type=int)
    p.add_argument("--input-size", default=512, type=int)
    p.add_argument("--workers", default=4, type=int)
    p.add_argument("--lr", default=0.0001, type=float)
    p.add_argument("--momentum", default=0.9, type=float)
    p.add_argument("--wd", "--weight-decay", default=1e-4, type=float, dest="weight_decay")
    p.add_argument("--amp", action=argparse.BooleanOptionalAction, default=True)
    p.add_argument("--seed", default=11, type=int)
    p.add_argument("--cache-dir", default=".hf-cache/datasets")
    p.add_argument("--export-vis", action=argparse.BooleanOptionalAction, default=True)
    p.add_argument("--vis-num", default=8, type=int)
    p.add_argument("--vis-seed", default=0, type=int)
    p.add_argument("--max-train-batches", default=0, type=int)
    p.add_argument("--max-val-batches", default=0, type=int)
    p.add_argument("--max-test-batches", default=0, type=int)
    p.add_argument("--synthetic-train", default=64, type=int, help="synthetic training images")
    p.add_argument("--synthetic-val", default=16, type=int, help="synthetic val/test images")
    p.add_argument("--out-dir", default="logs")
    args = p.parse_args(argv)
    if args.pos_weight == "":
        args.pos_weight = None
    return args


if __name__ == "__main__":
    train(parse_args())
