"""Host-side tables for the device augmentation (csrc/augment.hip) of utils/hf_dataloader.py.

The reference augments on the CPU (utils/hf_dataloader.py:111-180): PIL resize (BICUBIC image,
NEAREST mask), horizontal flip, paste on a grey / zero canvas, then an HSV jitter through cv2 LUTs.
Here the pixel work runs in HIP kernels and the host only builds small per-sample tables:

* PIL's separable BICUBIC resample (Pillow src/libImaging/Resample.c): per output coordinate a
  window [xmin, xmin + n) and float64 filter weights normalised to 22-bit fixed point; the kernels
  accumulate uint8 x int32 with the same rounding bias and clip, so the result is bit-exact with
  Image.resize(..., BICUBIC) (pinned against PIL itself by tests/test_augment_cpu.py);
* PIL's NEAREST scaling (Geometry.c ImagingScaleAffine): one source index per output coordinate;
* the three 256-entry LUTs of the HSV jitter, computed exactly as the reference's numpy code.
"""
from __future__ import annotations

import math

import numpy as np

PRECISION_BITS = 32 - 8 - 2
BICUBIC_SUPPORT = 2.0


def _bicubic(x):
    """Resample.c bicubic_filter (a = -0.5), elementwise on a float64 array"""
    a = -0.5
    x = np.abs(x)
    near = ((a + 2.0) * x - (a + 3.0)) * x * x + 1
    far = (((x - 5) * x + 8) * x - 4) * a
    return np.where(x < 1.0, near, np.where(x < 2.0, far, 0.0))


def bicubic_coeffs(in_size: int, out_size: int):
    """Resample.c precompute_coeffs + normalize_coeffs_8bpc: (bounds int32 [out][2] = (xmin, n),
    kk int32 [out][ksize], ksize).  Vectorised over output coordinates with the same float64
    operations; the normalising sum is a sequential cumsum, the C loop's order."""
    scale = filterscale = float(in_size) / out_size
    if filterscale < 1.0:
        filterscale = 1.0
    support = BICUBIC_SUPPORT * filterscale
    ksize = int(math.ceil(support)) * 2 + 1
    ss = 1.0 / filterscale
    center = (np.arange(out_size, dtype=np.float64) + 0.5) * scale
    lo = center - support + 0.5
    xmin = np.where(lo < 0, 0, np.trunc(lo)).astype(np.int64)  # (int) truncates, then clamps at 0
    xmax = np.minimum(np.trunc(center + support + 0.5).astype(np.int64), in_size) - xmin
    x = np.arange(ksize, dtype=np.int64)[None, :]
    kk = _bicubic((x + xmin[:, None] - center[:, None] + 0.5) * ss)
    kk = np.where(x < xmax[:, None], kk, 0.0)
    ww = np.cumsum(kk, axis=1)[:, -1]
    kk = np.where(ww[:, None] != 0.0, kk / np.where(ww == 0.0, 1.0, ww)[:, None], kk)
    scaled = kk * float(1 << PRECISION_BITS)
    fixed = np.trunc(np.where(kk < 0, -0.5 + scaled, 0.5 + scaled)).astype(np.int32)  # C casts truncate
    bounds = np.stack([xmin, xmax], 1).astype(np.int32)
    return bounds, fixed, ksize


def nearest_index(in_size: int, out_size: int):
    """Geometry.c ImagingScaleAffine: the source coordinate is ACCUMULATED in float64
    (xo = a/2; xo += a per output pixel, a = in/out) and truncated -- not a*(x+0.5), which differs
    in ~20% of size pairs (checked against Pillow by tests/test_augment_cpu.py).  cumsum is the
    same sequential float64 summation."""
    a = float(in_size) / out_size
    steps = np.full(out_size, a, dtype=np.float64)
    steps[0] = a * 0.5
    xo = np.cumsum(steps)
    idx = np.trunc(xo).astype(np.int64)
    return np.minimum(idx, in_size - 1).astype(np.int32)


def hsv_luts(r):
    """hf_dataloader.py:169-174: uint8 LUTs for hue (mod 180), saturation and value (clipped)"""
    x = np.arange(0, 256, dtype=np.asarray(r).dtype)
    lut_hue = ((x * r[0]) % 180).astype(np.uint8)
    lut_sat = np.clip(x * r[1], 0, 255).astype(np.uint8)
    lut_val = np.clip(x * r[2], 0, 255).astype(np.uint8)
    return np.stack([lut_hue, lut_sat, lut_val])


def resize_plan(iw, ih, nw, nh):
    """both passes of a BICUBIC resize of an (ih, iw) image to (nh, nw): horizontal tables, the
    source rows the vertical pass reads (ybox_first, ybox_last) and the vertical tables with bounds
    shifted to that row window, exactly as ImagingResampleInner arranges them"""
    bh, kh, ksh = bicubic_coeffs(iw, nw)
    bv, kv, ksv = bicubic_coeffs(ih, nh)
    y0 = int(bv[0, 0])
    y1 = int(bv[nh - 1, 0] + bv[nh - 1, 1])
    bv = bv.copy()
    bv[:, 0] -= y0
    return dict(bh=bh, kh=kh, ksh=ksh, bv=bv, kv=kv, ksv=ksv, ybox=(y0, y1))
