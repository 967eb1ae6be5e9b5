"""HF parquet dataset with device augmentation (reference: utils/hf_dataloader.py:17-213).

Reference flow per sample, on CPU workers: decode -> get_random_data (PIL BICUBIC/NEAREST resize,
flip, paste, cv2 HSV jitter) -> /255, binarise / clamp the label, one-hot -> collate to tensors.

Here the split is at the pixel work:
  * ``HFUnetDataset.__getitem__`` (CPU, DataLoader workers) reads one parquet row, decodes the
    image / mask with PIL exactly as the reference (``.convert("RGB")`` / ``.convert("L")``) and
    draws the augmentation parameters with ``np.random`` in the reference's order
    (hf_dataloader.py:135-166), so a seeded run makes the same draws.  It returns a ``RawSample``.
  * ``hf_unet_dataset_collate(batch)`` -- the reference's one-argument collate_fn -- packs a list of
    ``RawSample`` (each carries its dataset's input_shape / num_classes / task) into one ``RawBatch``:
    the uint8 pixels back to back plus the per-sample descriptors and tables
    (utils/augment_tables.py).
  * ``RawBatch.to_device`` (main process) uploads the bytes and runs ``unetseg_augment_batch``
    (csrc/augment.hip): resize, flip, paste, HSV jitter, /255, label handling and one-hot for the
    whole batch, writing the collated ``(images, pngs, seg_labels[, cls_labels])`` the reference's
    collate returns, already on the GPU.  A ``RawBatch`` also unpacks like the reference's tuple
    (``imgs, pngs, labels = batch``: the device path runs on first access, and ``.to(device)`` on
    the results is then a no-op), so a reference training loop over
    ``DataLoader(ds, collate_fn=hf_unet_dataset_collate, pin_memory=True)`` runs unchanged.
    ``DeviceLoader`` wraps a DataLoader and does the device work one batch ahead on a side stream.
  * ``ds[i]`` is a ``RawSample``; unpacking it (``jpg, png, seg_labels = ds[i]``) gives the
    reference's item as numpy (one-sample device batch), as does ``ds.get(i)``.
The geometric part is bit-exact with Pillow; the HSV jitter follows OpenCV's 8-bit algorithm
(parity unpinned: cv2 is not installed here, see oracle/augment_ref.py).

Dataset layout (convert_and_upload.py:60-90): ``{data_dir}/{config}/{split}/data.parquet`` with
columns image / mask (HF Image structs: bytes + path), label, filename, subset.  The parquet files are
memory-mapped Arrow tables (as ``datasets.load_dataset`` keeps them); a row is materialised only in
``__getitem__``, so forked DataLoader workers share the mapping instead of copying Python objects.
"""
from __future__ import annotations

import glob
import io
import math
import os
from dataclasses import dataclass, field

import numpy as np
import torch
from PIL import Image

from utils import augment_tables as at

AUG_DESC = 20  # csrc/augment.hip descriptor width (int64)
(D_SRC, D_MSK, D_TMP, D_RSZ, D_IW, D_IH, D_NW, D_NH, D_DX, D_DY, D_FLIP, D_Y0, D_ROWS, D_KSH, D_KSV, D_TAB, D_HSV,
 D_MIW, D_MIH) = range(19)

_SPLIT_ALIASES = {"validation": ("validation", "val", "valid", "dev"), "train": ("train", "training"),
                  "test": ("test", "testing", "eval")}


def find_split_files(data_dir, config, split):
    """the parquet files ``load_dataset(f"{data_dir}/{config}", split=split)`` reads for a local
    directory (HF's default patterns: ``{split}/*.parquet``, ``{split}-*.parquet``,
    ``data/{split}-*.parquet``)"""
    root = os.path.join(data_dir, config)
    for name in _SPLIT_ALIASES.get(split, (split,)):
        for pat in (os.path.join(root, name, "*.parquet"), os.path.join(root, f"{name}-*.parquet"),
                    os.path.join(root, "data", f"{name}-*.parquet"), os.path.join(root, f"{name}.parquet")):
            files = sorted(glob.glob(pat))
            if files:
                return files
    raise FileNotFoundError(f"no parquet files for split '{split}' under {root}")


def _open_image(cell, base_dir):
    """an HF Image cell: {'bytes': ..., 'path': ...} (bytes win; else the path, relative to the data)"""
    if isinstance(cell, dict):
        data, path = cell.get("bytes"), cell.get("path")
    else:
        data, path = None, cell
    if data is not None:
        return Image.open(io.BytesIO(data))
    if path is None:
        raise ValueError("image cell has neither bytes nor path")
    if not os.path.isabs(path) and not os.path.exists(path):
        path = os.path.join(base_dir, path)
    return Image.open(path)


@dataclass
class RawSample:
    """one decoded sample and its drawn augmentation (picklable: crosses DataLoader workers), with the
    dataset settings the one-argument collate needs.  Unpacks as the reference's item
    ``(jpg, png, seg_labels[, cls_label])`` (numpy, through a one-sample device batch)."""
    image: np.ndarray  # uint8 [ih][iw][3]
    mask: np.ndarray  # uint8 [mh][mw]
    nw: int
    nh: int
    dx: int
    dy: int
    flip: bool
    r: np.ndarray | None  # HSV factors (training) or None (validation letterbox)
    cls_label: int | None = None
    input_shape: tuple | None = None
    num_classes: int | None = None
    task: str = "multiclass"

    def reference_item(self, device="cuda"):
        """hf_dataloader.py:67-105's return value: jpg fp32 [3,H,W], png int64 [H,W], seg_labels fp32
        [H,W,C+1] (numpy) [, cls_label int]"""
        if self.input_shape is None:
            raise TypeError("RawSample without dataset settings (input_shape / num_classes / task)")
        out = pack_batch([self], self.input_shape, self.num_classes, self.task).to_device(device)
        torch.cuda.synchronize()
        vals = [t[0].cpu().numpy() for t in out[:3]]
        return (*vals, int(out[3][0])) if len(out) == 4 else tuple(vals)

    def __iter__(self):
        return iter(self.reference_item())


class HFUnetDataset(torch.utils.data.Dataset):
    """hf_dataloader.py:17-105 (same constructor, same CLASS_TO_IDX, same draws)"""

    CLASS_TO_IDX = {"动物类": 0, "植物类": 1, "复合类": 2}

    def __init__(self, data_dir, input_shape, num_classes, augmentation=True, split="train", config="full",
                 task: str = "multiclass", cache_dir: str | None = None, return_cls_label: bool = False):
        import pyarrow.parquet as pq

        self.input_shape = input_shape
        self.num_classes = num_classes
        self.augmentation = augmentation
        self.task = task
        self.return_cls_label = return_cls_label
        self.files = find_split_files(data_dir, config, split)
        self.base_dir = os.path.join(data_dir, config)
        # memory-mapped Arrow tables (only the columns read); rows are decoded on access
        self._tables = []
        for f in self.files:
            names = pq.read_schema(f).names
            missing = {"image", "mask"} - set(names)
            if missing:
                raise ValueError(f"{f}: missing columns {sorted(missing)}")
            cols = [c for c in ("image", "mask", "label", "filename") if c in names]
            self._tables.append(pq.read_table(f, columns=cols, memory_map=True))
        self._starts = np.cumsum([0] + [t.num_rows for t in self._tables])
        self.length = int(self._starts[-1])

    def __len__(self):
        return self.length

    def _row(self, index):
        """(table, row) of a global index (negative indices as a list)"""
        if index < 0:
            index += self.length
        if not 0 <= index < self.length:
            raise IndexError(index)
        k = int(np.searchsorted(self._starts, index, side="right")) - 1
        return self._tables[k], int(index - self._starts[k])

    def _cell(self, column, index):
        t, r = self._row(index)
        if column not in t.column_names:
            return None
        return t.column(column)[r].as_py()

    @staticmethod
    def rand(a=0, b=1):
        """hf_dataloader.py:107-109"""
        return np.random.rand() * (b - a) + a

    def draw(self, iw, ih, jitter=.3, hue=.1, sat=0.7, val=0.3, random=True):
        """the parameters get_random_data (hf_dataloader.py:111-166) draws, in its order"""
        h, w = self.input_shape
        if not random:
            scale = min(w / iw, h / ih)
            nw, nh = int(iw * scale), int(ih * scale)
            return dict(nw=nw, nh=nh, dx=(w - nw) // 2, dy=(h - nh) // 2, flip=False, r=None)
        new_ar = iw / ih * self.rand(1 - jitter, 1 + jitter) / self.rand(1 - jitter, 1 + jitter)
        scale = self.rand(0.25, 2)
        if new_ar < 1:
            nh = int(scale * h)
            nw = int(nh * new_ar)
        else:
            nw = int(scale * w)
            nh = int(nw / new_ar)
        if nw <= 0 or nh <= 0:  # PIL's resize refuses an empty size, so does the reference
            raise ValueError(f"height and width must be > 0 (drew {nw}x{nh})")
        flip = self.rand() < .5
        dx = int(self.rand(0, w - nw))
        dy = int(self.rand(0, h - nh))
        r = np.random.uniform(-1, 1, 3) * [hue, sat, val] + 1
        return dict(nw=nw, nh=nh, dx=dx, dy=dy, flip=bool(flip), r=r)

    def cls_label_of(self, index):
        """hf_dataloader.py:94-103"""
        name = self._cell("label", index) or "unknown"
        for cname, idx in self.CLASS_TO_IDX.items():
            if name.startswith(cname):
                return idx
        return 0

    def __getitem__(self, index) -> RawSample:
        jpg = _open_image(self._cell("image", index), self.base_dir).convert("RGB")
        png = _open_image(self._cell("mask", index), self.base_dir).convert("L")
        iw, ih = jpg.size
        p = self.draw(iw, ih, random=self.augmentation)
        return RawSample(image=np.asarray(jpg, np.uint8), mask=np.asarray(png, np.uint8),
                         cls_label=self.cls_label_of(index) if self.return_cls_label else None,
                         input_shape=tuple(int(v) for v in self.input_shape), num_classes=int(self.num_classes),
                         task=self.task, **p)

    def get(self, index, device="cuda"):
        """the reference's item (jpg fp32 [3,H,W], png int64 [H,W], seg_labels fp32 [H,W,C+1][, cls]) as
        numpy, produced through the device path (one-sample batch)"""
        return self[index].reference_item(device)


@dataclass
class RawBatch:
    """host side of one batch: packed pixels + descriptors (+ host-built tables, or the HSV factors
    the device builds them from), ready for unetseg_augment_batch(_dev).  The arrays are torch CPU
    tensors -- in a DataLoader worker they are allocated in shared memory, so the batch reaches the
    main process as file descriptors instead of ~15 MB of pickled bytes."""
    src: torch.Tensor  # uint8
    msk: torch.Tensor  # uint8
    desc: torch.Tensor  # int64 [B][AUG_DESC]
    tables: torch.Tensor | None  # int32 (host-built), or None: built on the device from hsv_r
    tmp_bytes: int
    rsz_bytes: int
    input_shape: tuple
    num_classes: int
    binary: bool
    cls_labels: np.ndarray | None = None
    hsv_r: torch.Tensor | None = None  # float64 [B][3] (device tables)
    n_tables: int = 0
    pinned: dict = field(default_factory=dict)
    _tensors: tuple | None = None

    @property
    def batch_size(self):
        return self.desc.shape[0]

    def pin(self):
        """page-lock the host arrays (once) so the uploads run asynchronously"""
        if not self.pinned:
            for k in ("src", "msk", "tables", "desc", "hsv_r"):
                v = getattr(self, k)
                if v is not None:
                    self.pinned[k] = (v if torch.is_tensor(v) else torch.from_numpy(v)).pin_memory()
        return self

    def pin_memory(self, device=None):
        """DataLoader(pin_memory=True) calls this on every batch (torch.utils.data._utils.pin_memory)"""
        return self.pin()

    # -- the reference collate's tuple (hf_dataloader.py:205-213): (images, pngs, seg_labels[, cls]) --
    def tensors(self, device=None):
        """the collated tensors on `device` (default: the current HIP device); computed once"""
        if self._tensors is None:
            dev = torch.device(device) if device is not None else torch.device("cuda", torch.cuda.current_device())
            self._tensors = self.to_device(dev)
        return self._tensors

    def __len__(self):
        return 4 if self.cls_labels is not None else 3

    def __iter__(self):
        return iter(self.tensors())

    def __getitem__(self, i):
        return self.tensors()[i]

    def to_device(self, device="cuda", stream=None, onehot=True):
        """run the device augmentation; returns (images, pngs, seg_labels[, cls_labels]) on `device`"""
        from unetseg_hip.lib import lib

        device = torch.device(device)
        if device.type != "cuda":
            raise RuntimeError("the device augmentation needs a GPU (no CPU fallback)")
        stream = stream or torch.cuda.current_stream(device)
        self.pin()
        B = self.batch_size
        H, W = int(self.input_shape[0]), int(self.input_shape[1])
        with torch.cuda.stream(stream):
            dev = {k: v.to(device, non_blocking=True) for k, v in self.pinned.items()}
            tmp = torch.empty(max(self.tmp_bytes, 1), dtype=torch.uint8, device=device)
            rsz = torch.empty(max(self.rsz_bytes, 1), dtype=torch.uint8, device=device)
            img = torch.empty(B, 3, H, W, dtype=torch.float32, device=device)
            png = torch.empty(B, H, W, dtype=torch.int64, device=device)
            seg = torch.empty(B, H, W, self.num_classes + 1, dtype=torch.float32, device=device) if onehot else None
        scratch = [tmp, rsz]
        if self.tables is None:
            # tables built on the device from the descriptors (unetseg_augment_batch_dev)
            with torch.cuda.stream(stream):
                tab = torch.empty(max(self.n_tables, 1), dtype=torch.int32, device=device)
            scratch.append(tab)
            lib.augment_batch_dev(self.pinned["desc"].data_ptr(), dev["desc"].data_ptr(), B, dev["hsv_r"].data_ptr(),
                                  tab.data_ptr(), self.n_tables, dev["src"].data_ptr(), self.src.numel(),
                                  dev["msk"].data_ptr(), self.msk.numel(), tmp.data_ptr(), self.tmp_bytes,
                                  rsz.data_ptr(), self.rsz_bytes, H, W, self.num_classes, int(self.binary),
                                  img.data_ptr(), png.data_ptr(), seg.data_ptr() if seg is not None else None,
                                  stream.cuda_stream)
        else:
            lib.augment_batch(self.pinned["desc"].data_ptr(), dev["desc"].data_ptr(), B,
                              self.pinned["tables"].data_ptr(), dev["tables"].data_ptr(), self.tables.numel(),
                              dev["src"].data_ptr(), self.src.numel(), dev["msk"].data_ptr(), self.msk.numel(),
                              tmp.data_ptr(), self.tmp_bytes, rsz.data_ptr(), self.rsz_bytes, H, W, self.num_classes,
                              int(self.binary), img.data_ptr(), png.data_ptr(),
                              seg.data_ptr() if seg is not None else None, stream.cuda_stream)
        # the scratch and the uploads must outlive the kernels queued on `stream`
        for t in list(dev.values()) + scratch:
            t.record_stream(stream)
        out = (img, png, seg)
        if self.cls_labels is not None:
            with torch.cuda.stream(stream):
                cls = torch.from_numpy(self.cls_labels).to(device, non_blocking=True)
            out = out + (cls,)
        return out


def _host_buffer(n, dtype):
    """a CPU tensor for a batch array: in shared memory inside a DataLoader worker (the batch then
    crosses to the main process as a file descriptor, not as pickled bytes)"""
    t = torch.empty(max(int(n), 1), dtype=dtype)
    if torch.utils.data.get_worker_info() is not None:
        t.share_memory_()
    return t


def _vertical_window(ih, nh):
    """resize_plan's ybox: the first and one-past-last source rows of the vertical BICUBIC pass,
    from bicubic_coeffs' bounds of output rows 0 and nh - 1 (the same float64 operations)"""
    scale = float(ih) / nh
    support = at.BICUBIC_SUPPORT * max(scale, 1.0)

    def bounds(i):
        center = (i + 0.5) * scale
        lo = center - support + 0.5
        xmin = 0 if lo < 0 else math.trunc(lo)
        return xmin, min(math.trunc(center + support + 0.5), ih) - xmin

    y0 = bounds(0)[0]
    xl, nl = bounds(nh - 1)
    return y0, xl + nl


def _ksize(in_size, out_size):
    """bicubic_coeffs' taps per output coordinate"""
    return int(math.ceil(at.BICUBIC_SUPPORT * max(float(in_size) / out_size, 1.0))) * 2 + 1


def pack_batch(samples, input_shape=None, num_classes=None, task=None, device_tables=True):
    """list[RawSample] -> RawBatch.  The settings default to the ones the samples carry
    (HFUnetDataset.__getitem__).  device_tables (default): the BICUBIC / NEAREST tables and HSV LUTs
    are built on the device from the descriptors (csrc/augment.hip aug_tables, bit-identical to
    utils/augment_tables.py); False builds them here (the reference builder the device one is tested
    against)."""
    if samples and input_shape is None:
        input_shape, num_classes, task = samples[0].input_shape, samples[0].num_classes, task or samples[0].task
    if input_shape is None or num_classes is None:
        raise TypeError("pack_batch needs input_shape / num_classes (or samples that carry them)")
    task = task or "multiclass"
    B = len(samples)
    desc = np.zeros((B, AUG_DESC), np.int64)
    hsv_r = np.ones((B, 3), np.float64)
    tabs = []
    src_off = msk_off = tmp_off = rsz_off = tab_off = 0
    for i, s in enumerate(samples):
        ih, iw = s.image.shape[:2]
        mh, mw = s.mask.shape[:2]
        hsv = s.r is not None
        if device_tables:
            ksh, ksv = _ksize(iw, s.nw), _ksize(ih, s.nh)
            y0, y1 = _vertical_window(ih, s.nh)
            tlen = 2 * s.nw + s.nw * ksh + 2 * s.nh + s.nh * ksv + s.nw + s.nh + (768 if hsv else 0)
            if hsv:
                hsv_r[i] = np.asarray(s.r, np.float64)
        else:
            bh, kh, ksh = at.bicubic_coeffs(iw, s.nw)
            bv, kv, ksv = at.bicubic_coeffs(ih, s.nh)
            y0 = int(bv[0, 0])
            y1 = int(bv[-1, 0] + bv[-1, 1])
            bv = bv.copy()
            bv[:, 0] -= y0  # ImagingResampleInner: the vertical pass reads the horizontal pass's rows
            parts = [bh.ravel(), kh.ravel(), bv.ravel(), kv.ravel(), at.nearest_index(mw, s.nw),
                     at.nearest_index(mh, s.nh)]
            if hsv:
                parts.append(at.hsv_luts(np.asarray(s.r)).astype(np.int32).ravel())
            t = np.concatenate([np.asarray(p, np.int32) for p in parts])
            tabs.append(t)
            tlen = t.size
        rows = y1 - y0
        desc[i, [D_SRC, D_MSK, D_TMP, D_RSZ, D_IW, D_IH, D_NW, D_NH, D_DX, D_DY, D_FLIP, D_Y0, D_ROWS, D_KSH, D_KSV,
                 D_TAB, D_HSV, D_MIW, D_MIH]] = [src_off, msk_off, tmp_off, rsz_off, iw, ih, s.nw, s.nh, s.dx, s.dy,
                                                 int(s.flip), y0, rows, ksh, ksv, tab_off, int(hsv), mw, mh]
        src_off += iw * ih * 3
        msk_off += mw * mh
        tmp_off += rows * s.nw * 3
        rsz_off += s.nh * s.nw * 3
        tab_off += tlen
    # the pixels straight into the batch buffers (one copy each)
    src, msk = _host_buffer(src_off, torch.uint8), _host_buffer(msk_off, torch.uint8)
    sv, mv = src.numpy(), msk.numpy()
    for i, s in enumerate(samples):
        a, m = np.ascontiguousarray(s.image, np.uint8).ravel(), np.ascontiguousarray(s.mask, np.uint8).ravel()
        sv[desc[i, D_SRC]:desc[i, D_SRC] + a.size] = a
        mv[desc[i, D_MSK]:desc[i, D_MSK] + m.size] = m
    cls = None
    if samples and samples[0].cls_label is not None:
        cls = np.array([s.cls_label for s in samples], np.int64)
    tables = torch.from_numpy(np.concatenate(tabs)) if tabs else None
    return RawBatch(src=src, msk=msk, desc=torch.from_numpy(desc), tables=tables, tmp_bytes=tmp_off,
                    rsz_bytes=rsz_off, input_shape=tuple(int(v) for v in input_shape), num_classes=num_classes,
                    binary=(task == "binary"), cls_labels=cls,
                    hsv_r=torch.from_numpy(hsv_r) if device_tables else None, n_tables=tab_off)


class _Collate:
    """picklable collate bound to the dataset's shape / classes / task"""

    def __init__(self, input_shape, num_classes, task):
        self.args = (input_shape, num_classes, task)

    def __call__(self, batch):
        return pack_batch(batch, *self.args)


def hf_unet_dataset_collate(batch, input_shape=None, num_classes=None, task=None):
    """hf_dataloader.py:183-213, the reference's one-argument collate_fn: the settings come from the
    samples (HFUnetDataset stores them in each RawSample) unless given.  Returns a RawBatch, which
    unpacks as the reference's ``(images, pngs, seg_labels[, cls_labels])`` on the current HIP device
    (``RawBatch.tensors``), or feeds ``DeviceLoader`` / ``RawBatch.to_device``."""
    return pack_batch(batch, input_shape, num_classes, task)


def make_collate(dataset: HFUnetDataset):
    return _Collate(tuple(dataset.input_shape), dataset.num_classes, dataset.task)


class DeviceLoader:
    """iterate a DataLoader of RawBatch as the reference's collated tensors on `device`; batch i+1 is
    uploaded and augmented on a side stream while the caller computes on batch i.  onehot=False skips
    the fp32 one-hot seg_labels (B x H x W x (C+1): 50 MB at 512^2, B=16, C=2) and yields None in its
    slot -- the binary and multitask loops never read it (utils/train_and_eval.py:203-207)."""

    def __init__(self, loader, device="cuda", onehot=True):
        self.loader, self.device, self.onehot = loader, torch.device(device), onehot
        self.sampler = getattr(loader, "sampler", None)
        self.dataset = getattr(loader, "dataset", None)

    def __len__(self):
        return len(self.loader)

    def __iter__(self):
        side = torch.cuda.Stream(self.device)
        pending = None
        for raw in self.loader:
            cur = raw.to_device(self.device, side, self.onehot)
            ev = torch.cuda.Event()
            ev.record(side)
            if pending is not None:
                yield self._ready(*pending)
            pending = (cur, ev)
        if pending is not None:
            yield self._ready(*pending)

    def _ready(self, tensors, ev):
        cs = torch.cuda.current_stream(self.device)
        cs.wait_event(ev)
        for t in tensors:
            if t is not None:
                t.record_stream(cs)
        return tensors
