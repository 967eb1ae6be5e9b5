"""Synthetic HF-format parquet datasets for the loader tests (no dataset is available offline).

Layout and schema follow convert_and_upload.py:60-105 (``{root}/{config}/{split}/data.parquet``;
image / mask as HF Image structs {bytes, path}; label, filename, subset strings).  Images mix JPEG
and PNG, RGB / greyscale / palette modes and sizes, so every decode path of the reference's
``.convert("RGB")`` / ``.convert("L")`` is exercised.
"""
import io
import os

import numpy as np
from PIL import Image

LABELS = ["动物类12", "植物类3", "复合类7", "other1"]


def _encode(img, fmt):
    buf = io.BytesIO()
    img.save(buf, format=fmt, **({"quality": 90} if fmt == "JPEG" else {}))
    return buf.getvalue()


def make_image(rng, w, h, mode="RGB"):
    yy, xx = np.mgrid[0:h, 0:w]
    base = np.stack([(xx * 255 // max(w - 1, 1)), (yy * 255 // max(h - 1, 1)), ((xx + yy) * 7) % 256], -1)
    arr = np.clip(base + rng.integers(-40, 40, (h, w, 3)), 0, 255).astype(np.uint8)
    img = Image.fromarray(arr)
    return img.convert(mode) if mode != "RGB" else img


def make_mask(rng, w, h, values=(0, 1, 2, 3, 255), palette=False):
    m = np.zeros((h, w), np.uint8)
    for _ in range(3):
        cy, cx = rng.integers(0, h), rng.integers(0, w)
        ry, rx = rng.integers(2, max(3, h // 2)), rng.integers(2, max(3, w // 2))
        yy, xx = np.mgrid[0:h, 0:w]
        m[((yy - cy) / ry) ** 2 + ((xx - cx) / rx) ** 2 < 1] = rng.choice(values)
    img = Image.fromarray(m)
    if palette:
        img = img.convert("P")
        img.putpalette([v for i in range(256) for v in (i, i, i)])
    return img


def make_dataset(root, config="full", split="train", n=6, seed=0, sizes=None, embed=True, mask_sizes=None):
    """write a parquet split; returns its path.  sizes: list of (w, h)"""
    import pyarrow as pa
    import pyarrow.parquet as pq

    rng = np.random.default_rng(seed)
    sizes = sizes or [(int(rng.integers(24, 97)), int(rng.integers(24, 97))) for _ in range(n)]
    d = os.path.join(root, config, split)
    os.makedirs(d, exist_ok=True)
    images, masks, labels, names = [], [], [], []
    for i, (w, h) in enumerate(sizes):
        mode = "L" if i % 5 == 3 else "RGB"
        img = make_image(rng, w, h, mode)
        mw, mh = mask_sizes[i] if mask_sizes else (w, h)
        msk = make_mask(rng, mw, mh, palette=(i % 4 == 2))
        fmt = "JPEG" if i % 2 == 0 else "PNG"
        ib, mb = _encode(img, fmt), _encode(msk, "PNG")
        ipath, mpath = f"img_{i}.{fmt.lower()}", f"mask_{i}.png"
        if embed:
            images.append({"bytes": ib, "path": ipath})
            masks.append({"bytes": mb, "path": mpath})
        else:  # path-only cells (Dataset.to_parquet of path columns), relative to the config dir
            with open(os.path.join(root, config, ipath), "wb") as f:
                f.write(ib)
            with open(os.path.join(root, config, mpath), "wb") as f:
                f.write(mb)
            images.append({"bytes": None, "path": ipath})
            masks.append({"bytes": None, "path": mpath})
        labels.append(LABELS[i % len(LABELS)])
        names.append(f"sample_{i}")
    st = pa.struct([("bytes", pa.binary()), ("path", pa.string())])
    table = pa.table({"image": pa.array(images, st), "mask": pa.array(masks, st), "label": labels, "filename": names,
                      "subset": [config] * len(names)})
    path = os.path.join(d, "data.parquet")
    pq.write_table(table, path)
    return path
