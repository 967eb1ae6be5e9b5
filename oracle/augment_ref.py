"""TEST INFRASTRUCTURE ONLY (see oracle/__init__.py) -- CPU restatement of the reference's
augmentation (utils/hf_dataloader.py:67-105, 111-180, 183-213).

* The geometric part runs the reference's own PIL calls (Image.resize BICUBIC / NEAREST,
  FLIP_LEFT_RIGHT, paste on a (128,128,128) / 0 canvas) -- PIL is the library the reference uses,
  so this part is pinned by construction.
* The HSV jitter restates OpenCV's 8-bit RGB2HSV_b / HSV2RGB_b (color_hsv.simd.hpp, scalar path)
  and cv2.LUT in numpy.  cv2 is not installed here, so THIS PART IS PARITY UNPINNED: it follows the
  published OpenCV algorithm, not outputs of the reference.
"""
from __future__ import annotations

import numpy as np
from PIL import Image

HSV_SHIFT = 12
_SDIV = np.zeros(256, np.int64)
_HDIV = np.zeros(256, np.int64)
for _i in range(1, 256):
    _SDIV[_i] = int(np.rint((255 << HSV_SHIFT) / (1.0 * _i)))
    _HDIV[_i] = int(np.rint((180 << HSV_SHIFT) / (6.0 * _i)))


def rgb2hsv_u8(img):
    """cv2.cvtColor(img, COLOR_RGB2HSV) for uint8 RGB (hrange 180)"""
    r, g, b = (img[..., k].astype(np.int64) for k in range(3))
    v = np.maximum(np.maximum(b, g), r)
    vmin = np.minimum(np.minimum(b, g), r)
    diff = v - vmin
    vr = np.where(v == r, -1, 0)
    vg = np.where(v == g, -1, 0)
    s = (diff * _SDIV[v] + (1 << (HSV_SHIFT - 1))) >> HSV_SHIFT
    h = (vr & (g - b)) + (~vr & ((vg & (b - r + 2 * diff)) + ((~vg) & (r - g + 4 * diff))))
    h = (h * _HDIV[diff] + (1 << (HSV_SHIFT - 1))) >> HSV_SHIFT
    h = h + np.where(h < 0, 180, 0)
    return np.stack([np.clip(h, 0, 255), s, v], -1).astype(np.uint8)


def hsv2rgb_u8(hsv):
    """cv2.cvtColor(hsv, COLOR_HSV2RGB) for uint8 (float32 arithmetic, round half to even)"""
    f32 = np.float32
    h = hsv[..., 0].astype(f32)
    s = hsv[..., 1].astype(f32) * (f32(1.0) / f32(255.0))
    v = hsv[..., 2].astype(f32) * (f32(1.0) / f32(255.0))
    hscale = f32(6.0) / f32(180.0)
    hh = (h * hscale).astype(f32)
    hh = np.fmod(hh, f32(6.0)).astype(f32)
    sector = np.floor(hh).astype(np.int64)
    hh = (hh - sector.astype(f32)).astype(f32)
    bad = (sector < 0) | (sector >= 6)
    sector = np.where(bad, 0, sector)
    hh = np.where(bad, f32(0), hh).astype(f32)
    one = f32(1.0)
    tab = np.stack([v, (v * (one - s)).astype(f32), (v * (one - (s * hh).astype(f32))).astype(f32),
                    (v * (one - (s * (one - hh).astype(f32)).astype(f32))).astype(f32)], -1)
    sd = np.array([[1, 3, 0], [1, 0, 2], [3, 0, 1], [0, 2, 1], [0, 1, 3], [2, 1, 0]])
    idx = sd[sector]  # (..., 3): b, g, r tab indices
    b = np.take_along_axis(tab, idx[..., 0:1], -1)[..., 0]
    g = np.take_along_axis(tab, idx[..., 1:2], -1)[..., 0]
    r = np.take_along_axis(tab, idx[..., 2:3], -1)[..., 0]
    grey = s == 0
    b, g, r = (np.where(grey, v, c) for c in (b, g, r))
    out = np.stack([r, g, b], -1).astype(f32) * f32(255.0)
    return np.clip(np.rint(out.astype(f32)), 0, 255).astype(np.uint8)


def hsv_jitter(img, r):
    """hf_dataloader.py:165-178 (r = the 3 drawn factors)"""
    x = np.arange(0, 256, dtype=r.dtype)
    lut = [((x * r[0]) % 180).astype(np.uint8), np.clip(x * r[1], 0, 255).astype(np.uint8),
           np.clip(x * r[2], 0, 255).astype(np.uint8)]
    hsv = rgb2hsv_u8(img)
    hsv = np.stack([lut[k][hsv[..., k]] for k in range(3)], -1)
    return hsv2rgb_u8(hsv)


def random_params(iw, ih, w, h, rng=np.random, jitter=.3, hue=.1, sat=0.7, val=0.3):
    """the reference's draws, in its order (hf_dataloader.py:133-165): aspect jitter, scale, flip,
    paste offset, HSV factors"""
    def rand(a=0.0, b=1.0):
        return rng.rand() * (b - a) + a

    new_ar = iw / ih * rand(1 - jitter, 1 + jitter) / rand(1 - jitter, 1 + jitter)
    scale = rand(0.25, 2)
    if new_ar < 1:
        nh = int(scale * h)
        nw = int(nh * new_ar)
    else:
        nw = int(scale * w)
        nh = int(nw / new_ar)
    flip = rand() < .5
    dx = int(rand(0, w - nw))
    dy = int(rand(0, h - nh))
    r = rng.uniform(-1, 1, 3) * [hue, sat, val] + 1
    return dict(nw=nw, nh=nh, flip=bool(flip), dx=dx, dy=dy, r=r)


def val_params(iw, ih, w, h):
    """validation letterbox (hf_dataloader.py:118-131)"""
    scale = min(w / iw, h / ih)
    nw, nh = int(iw * scale), int(ih * scale)
    return dict(nw=nw, nh=nh, flip=False, dx=(w - nw) // 2, dy=(h - nh) // 2, r=None)


def augment(image, mask, w, h, p):
    """image / mask PIL (RGB / L) -> (uint8 HxWx3, uint8 HxW) exactly as get_random_data with params p"""
    img = image.resize((p["nw"], p["nh"]), Image.BICUBIC)
    lab = Image.fromarray(np.array(mask)).resize((p["nw"], p["nh"]), Image.NEAREST)
    if p["flip"]:
        img = img.transpose(Image.FLIP_LEFT_RIGHT)
        lab = lab.transpose(Image.FLIP_LEFT_RIGHT)
    new_image = Image.new("RGB", (w, h), (128, 128, 128))
    new_label = Image.new("L", (w, h), 0)
    new_image.paste(img, (p["dx"], p["dy"]))
    new_label.paste(lab, (p["dx"], p["dy"]))
    arr = np.array(new_image, np.uint8)
    if p["r"] is not None:
        arr = hsv_jitter(arr, p["r"])
    return arr, np.array(new_label, np.uint8)


def to_sample(arr, lab, num_classes, task):
    """hf_dataloader.py:78-91 + collate dtypes: (image fp32 [3,H,W], png int64 [H,W], onehot fp32)"""
    jpg = np.transpose(np.array(arr, np.float64) / 255.0, [2, 0, 1]).astype(np.float32)
    png = np.array(lab)
    if task == "binary":
        png = (png > 0).astype(np.uint8)
    png[png >= num_classes] = num_classes
    onehot = np.eye(num_classes + 1)[png.reshape(-1)].reshape(png.shape + (num_classes + 1,)).astype(np.float32)
    return jpg, png.astype(np.int64), onehot
