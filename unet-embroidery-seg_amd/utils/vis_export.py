"""Fixed-sample visual export of the binary / multitask test split (reference: utils/vis_export.py:1-97).

For ``num_samples`` indices drawn with ``random.Random(seed).sample`` (the reference's draw, so the
same seed picks the same samples), each test image is letterboxed exactly as the validation loader
does (HFUnetDataset.get: the device letterbox, bit-exact with PIL BICUBIC + paste), run through the
model on the HIP path, and saved as a 2x2 grid -- image / ground truth (red) / prediction (green) /
prediction overlaid at alpha 0.5 -- named ``{idx:04d}_{filename stem}_grid.png``, with the indices in
``indices.json``.  PIL only, as the reference.
"""
from __future__ import annotations

import json
import random
from pathlib import Path

import numpy as np
import torch
from PIL import Image


def _mask_to_rgb(mask01: np.ndarray, fg_color=(255, 0, 0)) -> np.ndarray:
    """vis_export.py:12-17"""
    out = np.zeros(mask01.shape + (3,), dtype=np.uint8)
    out[mask01 > 0] = np.array(fg_color, dtype=np.uint8)
    return out


def _make_grid(img_rgb: np.ndarray, gt01: np.ndarray, pred01: np.ndarray, alpha: float = 0.5) -> Image.Image:
    """vis_export.py:20-35: 2x2 image / gt / pred / overlay"""
    img = img_rgb.astype(np.uint8)
    pred_rgb = _mask_to_rgb(pred01, (0, 255, 0))
    overlay = (img.astype(np.float32) * (1 - alpha) + pred_rgb.astype(np.float32) * alpha).clip(0, 255).astype(np.uint8)
    h, w = img.shape[:2]
    canvas = Image.new("RGB", (w * 2, h * 2))
    canvas.paste(Image.fromarray(img), (0, 0))
    canvas.paste(Image.fromarray(_mask_to_rgb(gt01, (255, 0, 0))), (w, 0))
    canvas.paste(Image.fromarray(pred_rgb), (0, h))
    canvas.paste(Image.fromarray(overlay), (w, h))
    return canvas


@torch.no_grad()
def export_binary_visuals(model, hf_unet_dataset, out_dir: str, input_shape, device, num_samples: int = 8,
                          seed: int = 0):
    """vis_export.py:38-97.  hf_unet_dataset: an HFUnetDataset built with augmentation=False."""
    out_path = Path(out_dir)
    out_path.mkdir(parents=True, exist_ok=True)
    length = len(hf_unet_dataset)
    num_samples = min(num_samples, length)
    rng = random.Random(seed)
    indices = rng.sample(range(length), k=num_samples) if num_samples > 0 else []
    with (out_path / "indices.json").open("w", encoding="utf-8") as f:
        json.dump(indices, f, ensure_ascii=False, indent=2)
    model = model.eval().to(device)
    for idx in indices:
        jpg, png = hf_unet_dataset.get(idx, device)[:2]  # letterboxed image / 255 (fp32 [3,H,W]), labels
        # the reference displays the letterboxed uint8 image and feeds preprocess_input of it (/255):
        # jpg is exactly that division, so x255 recovers the uint8 pixels
        img_np = np.rint(np.transpose(jpg, (1, 2, 0)) * 255.0).astype(np.uint8)
        gt = (png > 0).astype(np.uint8)
        logits = model(torch.from_numpy(jpg[None]).float().to(device))
        pred = logits.argmax(dim=1).squeeze(0).cpu().numpy().astype(np.uint8)
        name = hf_unet_dataset._cell("filename", idx) or f"sample_{idx}"
        _make_grid(img_np, gt, pred, alpha=0.5).save(out_path / f"{idx:04d}_{Path(name).stem}_grid.png")
