"""CPU: the loader's host side (utils/hf_dataloader.py, utils/augment_tables.py) against Pillow and
the reference's draw order.

* the per-sample BICUBIC tables, run through an integer emulation of csrc/augment.hip's two passes,
  reproduce ``PIL.Image.resize(..., BICUBIC)`` bit-exactly; the NEAREST index tables reproduce
  ``resize(..., NEAREST)`` (PIL accumulates the source coordinate -- the a*(x+0.5) formula is wrong
  for ~20% of size pairs);
* HFUnetDataset reads the HF parquet layout (bytes-embedded and path-only cells), decodes like the
  reference and draws the augmentation with np.random in the reference's order
  (hf_dataloader.py:135-166), leaving np.random in the same state;
* pack_batch lays out descriptors / tables the kernel's host-side checks accept, and a corrupted
  descriptor is refused before any launch;
* the OpenCV HSV restatement (oracle/augment_ref.py, parity unpinned) is self-consistent.
"""
import ctypes
import os

import numpy as np
import pytest
from PIL import Image

from augment_data import make_dataset
from oracle import augment_ref
from utils import augment_tables as at
from utils.hf_dataloader import (AUG_DESC, D_KSH, D_NW, D_SRC, HFUnetDataset, hf_unet_dataset_collate, make_collate,
                                 pack_batch)


def _emulate(src, nw, nh):
    """csrc/augment.hip aug_hpass + aug_vpass in numpy integers"""
    ih, iw, _ = src.shape
    p = at.resize_plan(iw, ih, nw, nh)
    y0, y1 = p["ybox"]
    tmp = np.zeros((y1 - y0, nw, 3), np.int64)
    for xx in range(nw):
        xm, n = p["bh"][xx]
        acc = np.full((y1 - y0, 3), 1 << 21, np.int64)
        for x in range(n):
            acc += src[y0:y1, xm + x].astype(np.int64) * p["kh"][xx, x]
        tmp[:, xx] = np.clip(acc >> 22, 0, 255)
    out = np.zeros((nh, nw, 3), np.int64)
    for yy in range(nh):
        ym, n = p["bv"][yy]
        acc = np.full((nw, 3), 1 << 21, np.int64)
        for y in range(n):
            acc += tmp[ym + y] * p["kv"][yy, y]
        out[yy] = np.clip(acc >> 22, 0, 255)
    return out.astype(np.uint8)


def test_bicubic_tables_match_pillow():
    rng = np.random.default_rng(2)
    cases = [(64, 48, 64, 90), (64, 48, 33, 48), (1, 1, 5, 7), (7, 3, 1, 1), (300, 200, 1024, 683), (512, 384, 97, 71)]
    cases += [(int(rng.integers(1, 200)), int(rng.integers(1, 200)), int(rng.integers(1, 260)),
               int(rng.integers(1, 260))) for _ in range(60)]
    for iw, ih, nw, nh in cases:
        src = rng.integers(0, 256, (ih, iw, 3), dtype=np.uint8)
        ref = np.array(Image.fromarray(src).resize((nw, nh), Image.BICUBIC))
        np.testing.assert_array_equal(_emulate(src, nw, nh), ref, err_msg=str((iw, ih, nw, nh)))


def test_nearest_tables_match_pillow():
    rng = np.random.default_rng(3)
    for _ in range(300):
        iw, ih = int(rng.integers(1, 400)), int(rng.integers(1, 400))
        nw, nh = int(rng.integers(1, 500)), int(rng.integers(1, 500))
        m = rng.integers(0, 256, (ih, iw), dtype=np.uint8)
        ref = np.array(Image.fromarray(m).resize((nw, nh), Image.NEAREST))
        np.testing.assert_array_equal(m[at.nearest_index(ih, nh)][:, at.nearest_index(iw, nw)], ref)


def test_hsv_restatement_consistent():
    rng = np.random.default_rng(4)
    img = rng.integers(0, 256, (64, 64, 3), dtype=np.uint8)
    back = augment_ref.hsv2rgb_u8(augment_ref.rgb2hsv_u8(img))
    # 8-bit HSV quantises hue to 2 degrees: a round trip moves a channel by a few levels at most
    assert np.abs(back.astype(int) - img).max() <= 8
    grey = np.full((4, 4, 3), 128, np.uint8)
    assert (augment_ref.rgb2hsv_u8(grey)[..., :2] == 0).all()
    np.testing.assert_array_equal(augment_ref.hsv2rgb_u8(augment_ref.rgb2hsv_u8(grey)), grey)
    # identity LUTs on the factors r = 1 leave the HSV triple unchanged
    lut = at.hsv_luts(np.ones(3))
    np.testing.assert_array_equal(lut[1], np.arange(256))
    np.testing.assert_array_equal(lut[0][:180], np.arange(180))


@pytest.mark.parametrize("embed", [True, False])
def test_dataset_reads_parquet_and_draws_in_reference_order(tmp_path, embed):
    make_dataset(str(tmp_path), "full", "train", n=5, seed=1, embed=embed)
    ds = HFUnetDataset(str(tmp_path), [64, 64], 4, augmentation=True, split="train", config="full",
                       task="multiclass", return_cls_label=True)
    assert len(ds) == 5
    for i in range(5):
        np.random.seed(100 + i)
        s = ds[i]
        after = np.random.rand()
        # the same draws through the oracle's restatement of get_random_data's sequence
        np.random.seed(100 + i)
        p = augment_ref.random_params(s.image.shape[1], s.image.shape[0], 64, 64)
        assert (s.nw, s.nh, s.dx, s.dy, s.flip) == (p["nw"], p["nh"], p["dx"], p["dy"], p["flip"])
        np.testing.assert_array_equal(s.r, p["r"])
        assert np.random.rand() == after
        assert s.image.dtype == np.uint8 and s.image.ndim == 3 and s.mask.ndim == 2
    assert [ds.cls_label_of(i) for i in range(4)] == [0, 1, 2, 0]


def test_dataset_validation_letterbox(tmp_path):
    make_dataset(str(tmp_path), "no-ai", "validation", n=3, seed=2, sizes=[(80, 40), (30, 90), (64, 64)])
    ds = HFUnetDataset(str(tmp_path), [64, 64], 2, augmentation=False, split="validation", config="no-ai",
                       task="binary")
    state = np.random.get_state()[1].copy()
    got = [(s.nw, s.nh, s.dx, s.dy, s.flip, s.r) for s in (ds[i] for i in range(3))]
    assert got == [(64, 32, 0, 16, False, None), (21, 64, 21, 0, False, None), (64, 64, 0, 0, False, None)]
    np.testing.assert_array_equal(np.random.get_state()[1], state)  # validation draws nothing


def test_missing_split_raises(tmp_path):
    make_dataset(str(tmp_path), "full", "train", n=2)
    with pytest.raises(FileNotFoundError):
        HFUnetDataset(str(tmp_path), [64, 64], 2, split="test", config="full")


def test_pack_batch_layout(tmp_path):
    make_dataset(str(tmp_path), "full", "train", n=4, seed=5)
    ds = HFUnetDataset(str(tmp_path), [48, 40], 4, split="train", config="full", task="multiclass")
    np.random.seed(0)
    samples = [ds[i] for i in range(4)]
    b = make_collate(ds)(samples)
    assert b.desc.shape == (4, AUG_DESC) and b.input_shape == (48, 40) and not b.binary
    assert b.src.numel() == sum(s.image.size for s in samples)
    assert list(b.desc[:, D_NW]) == [s.nw for s in samples]
    assert b.desc[0, D_SRC] == 0 and b.desc[1, D_SRC] == samples[0].image.size
    np.testing.assert_array_equal(b.src[:samples[0].image.size].numpy(), samples[0].image.ravel())
    # the reference's one-argument collate_fn (hf_dataloader.py:183): settings ride on the samples
    b1 = hf_unet_dataset_collate(samples)
    assert b1.input_shape == (48, 40) and b1.num_classes == 4 and not b1.binary
    np.testing.assert_array_equal(b1.desc, b.desc)
    assert len(b1) == 3 and b1.batch_size == 4  # unpacks as (images, pngs, seg_labels)
    b2 = hf_unet_dataset_collate(samples, [48, 40], 4, "multiclass")
    np.testing.assert_array_equal(b2.desc, b.desc)
    # the host-built tables (the device builder's reference): same descriptors, same table length
    bh = pack_batch(samples, device_tables=False)
    np.testing.assert_array_equal(bh.desc, b.desc)
    assert b.tables is None and bh.tables.numel() == b.n_tables
    np.testing.assert_array_equal(b.hsv_r.numpy(), np.stack([s.r for s in samples]))


def test_device_table_descriptors_match_host_builder():
    """the descriptor fields the device-table path computes on the host (taps per axis, the vertical
    pass's source-row window) equal bicubic_coeffs' for random up- and down-scales"""
    from utils.hf_dataloader import _ksize, _vertical_window
    rng = np.random.default_rng(4)
    for _ in range(400):
        n_in = int(rng.integers(1, 1500))
        n_out = int(rng.integers(1, 1500))
        b, _, ks = at.bicubic_coeffs(n_in, n_out)
        assert _ksize(n_in, n_out) == ks, (n_in, n_out)
        assert _vertical_window(n_in, n_out) == (int(b[0, 0]), int(b[-1, 0] + b[-1, 1])), (n_in, n_out)


def test_reference_dataloader_contract(tmp_path):
    """DataLoader(ds, collate_fn=hf_unet_dataset_collate, pin_memory=True, num_workers=2) as
    train.py:140-162 builds it: the one-argument collate runs in the workers, the pinning hook is
    RawBatch.pin_memory, and a batch unpacks into 3 (binary / multiclass) or 4 (multitask) items."""
    from torch.utils.data import DataLoader
    make_dataset(str(tmp_path), "full", "train", n=5, seed=8)
    for cls_label, n_items in ((False, 3), (True, 4)):
        ds = HFUnetDataset(str(tmp_path), [32, 32], 2, split="train", config="full", task="binary",
                           return_cls_label=cls_label)
        dl = DataLoader(ds, batch_size=2, shuffle=False, num_workers=2, collate_fn=hf_unet_dataset_collate,
                        drop_last=False)
        batches = list(dl)
        assert [b.batch_size for b in batches] == [2, 2, 1]
        assert all(len(b) == n_items and b.binary and b.input_shape == (32, 32) for b in batches)
        assert callable(getattr(batches[0], "pin_memory", None))  # DataLoader(pin_memory=True)'s hook


def test_dataset_memory_mapped(tmp_path):
    """rows stay in the (memory-mapped) Arrow tables; nothing is materialised per row at
    construction"""
    make_dataset(str(tmp_path), "full", "train", n=6, seed=9)
    ds = HFUnetDataset(str(tmp_path), [32, 32], 2, split="train", config="full")
    assert len(ds) == 6 and not hasattr(ds, "images")
    assert all(t.num_rows > 0 for t in ds._tables)
    np.random.seed(3)
    s = ds[-1]
    assert s.input_shape == (32, 32) and s.num_classes == 2 and s.task == "multiclass"
    with pytest.raises(IndexError):
        ds[6]


def test_augment_rejects_bad_descriptor_before_launch(tmp_path):
    from unetseg_hip import lib

    if not os.path.exists(lib.LIB_PATH):
        pytest.skip("libunetseg_hip.so not built")
    make_dataset(str(tmp_path), "full", "train", n=2, seed=6)
    ds = HFUnetDataset(str(tmp_path), [32, 32], 2, split="train", config="full", task="binary")
    np.random.seed(1)
    s0, s1 = ds[0], ds[1]
    b = pack_batch([s0, s1], (32, 32), 2, "binary", device_tables=False)
    b.desc, b.tables, b.src, b.msk = b.desc.numpy(), b.tables.numpy(), b.src.numpy(), b.msk.numpy()
    raw = lib.load()
    fake = ctypes.c_void_p(16)  # never dereferenced: the host checks fail first

    def call(desc, tables, src_bytes):
        return raw.unetseg_augment_batch(desc.ctypes.data, fake, 2, tables.ctypes.data, fake, tables.size, fake,
                                         src_bytes, fake, b.msk.size, fake, b.tmp_bytes, fake, b.rsz_bytes, 32, 32,
                                         2, 1, fake, fake, None, None)

    # the device-table entry point validates the descriptors it builds the tables from
    bd = pack_batch([s0, s1], (32, 32), 2, "binary")
    dd = bd.desc.numpy()

    def call_dev(desc, src_bytes, n_tables=bd.n_tables):
        return raw.unetseg_augment_batch_dev(desc.ctypes.data, fake, 2, fake, fake, n_tables, fake, src_bytes, fake,
                                             bd.msk.numel(), fake, bd.tmp_bytes, fake, bd.rsz_bytes, 32, 32, 2, 1,
                                             fake, fake, None, None)

    assert call_dev(dd, bd.src.numel() - 1) != 0 and b"image range" in raw.unetseg_last_error()
    assert call_dev(dd, bd.src.numel(), bd.n_tables - 1) != 0 and b"table range" in raw.unetseg_last_error()
    d2 = dd.copy()
    d2[0, D_KSH] += 2  # taps that do not match the sizes
    assert call_dev(d2, bd.src.numel()) != 0 and b"kernel sizes" in raw.unetseg_last_error()

    assert call(b.desc, b.tables, b.src.size - 1) != 0  # image range
    assert b"image range" in raw.unetseg_last_error()
    bad = b.tables.copy()
    bad[0] = 10_000  # first horizontal window starts outside the image
    assert call(b.desc, bad, b.src.size) != 0
    assert b"horizontal table" in raw.unetseg_last_error()
    d = b.desc.copy()
    d[1, D_NW] = 0
    assert call(d, b.tables, b.src.size) != 0
