"""Evaluation entry point on the HIP path (reference: val.py:22-155).

Loads a state_dict (weights_only) into the named model and reports the binary metrics
(evaluate_binary: Dice / IoU / Precision / Recall / Accuracy, eps 1e-7) or, for multitask, seg
IoU / Dice (eps 1e-6) plus overall and per-class classification accuracy, or for multiclass the
reference's `evaluate` (CE + Dice loss, pixel / mean accuracy, mean / frequency-weighted IoU).
Data: the HF parquet test split (utils/hf_dataloader.py, device augmentation) or the seeded
synthetic test split (`--data-path synthetic`, binary / multitask only).
"""
from __future__ import annotations

import argparse
import os
import sys

_HERE = os.path.dirname(os.path.abspath(__file__))
if _HERE not in sys.path:
    sys.path.insert(0, _HERE)

import torch  # noqa: E402
from torch.utils.data import DataLoader  # noqa: E402

from model.model_factory import SUPPORTED_MODELS, build_model  # noqa: E402
from unetseg_hip import losses  # noqa: E402
from utils.hf_dataloader import DeviceLoader, HFUnetDataset, make_collate  # noqa: E402
from utils.synthetic import SyntheticSegDataset, collate  # noqa: E402
from utils.train_and_eval import LogColor, evaluate, evaluate_binary  # noqa: E402

CLASS_NAMES = ["动物类", "植物类", "复合类"]  # val.py:84


def val(args):
    num_classes = args.num_classes + 1 if args.task == "multiclass" else 2  # val.py:22-27
    device = torch.device(args.device)
    input_shape = [args.input_size] * 2
    if args.data_path != "synthetic":  # val.py:31-56
        ds = HFUnetDataset(args.data_path, input_shape, num_classes, augmentation=False, split="test",
                           config=args.data_config, task="binary" if args.task == "multitask" else args.task,
                           cache_dir=args.cache_dir, return_cls_label=args.task == "multitask")
        print(f"Test samples: {len(ds)}")
        loader = DeviceLoader(DataLoader(ds, batch_size=args.batch_size, shuffle=False, num_workers=0,
                                         collate_fn=make_collate(ds)), device, onehot=args.task == "multiclass")
    else:
        if args.task == "multiclass":
            raise ValueError("the synthetic set is binary; the multiclass task needs a real --data-path")
        ds = SyntheticSegDataset(args.synthetic_test, input_shape, 2, seed=888_000,
                                 return_cls_label=args.task == "multitask")
        loader = DataLoader(ds, batch_size=args.batch_size, shuffle=False, num_workers=0, collate_fn=collate)
    if args.task == "multitask":
        model = build_model(args.model, num_classes=1, num_seg_classes=1, num_cls_classes=3)
    else:
        model = build_model(args.model, num_classes=num_classes)
    model.load_state_dict(torch.load(args.weights, map_location="cpu", weights_only=True))
    model.to(device)
    print(f"Model loaded from: {args.weights}")

    if args.task == "binary":
        m = evaluate_binary(model, loader, device, loss_name=args.loss, pos_weight=None, ignore_index=None)
        print(f"{LogColor.RED}Dice{LogColor.RESET}\t{LogColor.RED}IoU{LogColor.RESET}\t{LogColor.RED}Precision"
              f"{LogColor.RESET}\t{LogColor.RED}Recall{LogColor.RESET}\t{LogColor.RED}Accuracy{LogColor.RESET}")
        print(f"{m['Dice']:.4f}\t{m['IoU']:.4f}\t{m['Precision']:.4f}\t{m['Recall']:.4f}\t{m['Accuracy']:.4f}")
        return m
    if args.task == "multiclass":
        m = evaluate(model, loader, device, dice_loss=True, focal_loss=False, num_classes=num_classes)
        print(m)
        return m

    model.eval()
    conf = torch.zeros(4, dtype=torch.int64, device=device)
    per_cls = torch.zeros(3, 2, dtype=torch.int64, device=device)  # [class][correct, count]
    with torch.no_grad():
        for images, seg_t, _, cls_t in loader:
            images, seg_t, cls_t = images.to(device), seg_t.to(device), cls_t.to(device)
            seg_logits, cls_logits = model(images)
            losses.binary_confusion(seg_logits, seg_t, conf)
            pred = cls_logits.argmax(1)
            for c in range(3):
                sel = cls_t == c
                per_cls[c, 0] += (pred[sel] == c).sum()
                per_cls[c, 1] += sel.sum()
    tp, fp, fn, _ = (float(v) for v in conf.tolist())
    iou = tp / (tp + fp + fn + 1e-6)
    dice = 2 * tp / ((tp + fp) + (tp + fn) + 1e-6)
    pc = per_cls.tolist()
    acc = 100.0 * sum(c for c, _ in pc) / max(sum(n for _, n in pc), 1)
    print("=" * 50)
    print(f"Segmentation: IoU {iou:.4f}  Dice {dice:.4f}")
    print(f"Classification: overall accuracy {acc:.2f}%")
    for name, (c, n) in zip(CLASS_NAMES, pc):
        if n:
            print(f"    {name}: {100.0 * c / n:.2f}% ({n} samples)")
    print("=" * 50)
    return {"IoU": iou, "Dice": dice, "Cls Acc": acc}


def parse_args(argv=None):
    p = argparse.ArgumentParser(description="U-Net evaluation on the MI355X HIP path")
    p.add_argument("--data-path", default="./hf_datasets/merged_dataset_v2",
                   help="HF parquet dataset directory, or 'synthetic' (the seeded synthetic test split)")
    p.add_argument("--data-config", default="no-ai", choices=["full", "no-ai", "sam3"])
    p.add_argument("--weights", default="weights/unet_resnet_voc.pth")
    p.add_argument("--task", default="binary", choices=["binary", "multiclass", "multitask"])
    p.add_argument("--model", default="unet_resnet50", choices=sorted(SUPPORTED_MODELS.keys()))
    # val.py:176: ce / focal are accepted; the binary evaluation then refuses them as the reference's
    # binary_segmentation_loss does (ValueError "Unsupported loss_name")
    p.add_argument("--loss", default="lovasz_hinge", choices=["bce", "lovasz_hinge", "ce", "focal"])
    p.add_argument("--num-classes", default=4, type=int)
    p.add_argument("--device", default="cuda")
    p.add_argument("--input-size", default=512, type=int)
    p.add_argument("--batch-size", default=1, type=int)
    p.add_argument("--cache-dir", default=".hf-cache/datasets")
    p.add_argument("--synthetic-test", default=16, type=int)
    return p.parse_args(argv)


if __name__ == "__main__":
    val(parse_args())
