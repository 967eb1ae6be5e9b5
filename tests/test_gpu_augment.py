"""GPU: the device augmentation (csrc/augment.hip via utils/hf_dataloader.py) against the CPU
restatement of the reference's get_random_data + preprocessing + collate (oracle/augment_ref.py).

The geometric part (PIL BICUBIC / NEAREST, flip, paste) and everything after it is compared
bit-exactly: fp32 images, int64 labels, one-hot.  The HSV jitter is compared bit-exactly with the
oracle's OpenCV restatement, which is itself parity unpinned (cv2 is absent here).
"""
import numpy as np
import pytest
import torch
from PIL import Image

from augment_data import make_dataset
from oracle import augment_ref
from utils.hf_dataloader import DeviceLoader, HFUnetDataset, make_collate

pytestmark = pytest.mark.gpu


def _oracle_batch(ds, samples):
    h, w = ds.input_shape
    imgs, pngs, segs = [], [], []
    for s in samples:
        p = dict(nw=s.nw, nh=s.nh, dx=s.dx, dy=s.dy, flip=s.flip, r=s.r)
        arr, lab = augment_ref.augment(Image.fromarray(s.image), Image.fromarray(s.mask), w, h, p)
        jpg, png, oh = augment_ref.to_sample(arr, lab, ds.num_classes, ds.task)
        imgs.append(jpg)
        pngs.append(png)
        segs.append(oh)
    return np.stack(imgs), np.stack(pngs), np.stack(segs)


def _check(ds, samples, out):
    ri, rp, rs = _oracle_batch(ds, samples)
    torch.cuda.synchronize()
    gi, gp, gs = (t.cpu().numpy() for t in out[:3])
    assert gi.dtype == np.float32 and gp.dtype == np.int64 and gs.dtype == np.float32
    for b in range(len(samples)):
        bad = np.argwhere(gi[b] != ri[b])
        assert bad.size == 0, (b, bad[:5], gi[b][tuple(bad[0])], ri[b][tuple(bad[0])])
    np.testing.assert_array_equal(gp, rp)
    np.testing.assert_array_equal(gs, rs)


@pytest.mark.parametrize("task,nc,train,shape", [("binary", 2, True, (64, 64)), ("multiclass", 4, True, (48, 80)),
                                                  ("binary", 2, False, (64, 64)), ("multiclass", 4, False, (40, 56))])
def test_augment_matches_oracle(tmp_path, task, nc, train, shape):
    make_dataset(str(tmp_path), "full", "train", n=10, seed=11)
    ds = HFUnetDataset(str(tmp_path), list(shape), nc, augmentation=train, split="train", config="full", task=task,
                       return_cls_label=True)
    np.random.seed(7)
    samples = [ds[i] for i in range(len(ds))]
    out = make_collate(ds)(samples).to_device("cuda")
    _check(ds, samples, out)
    assert out[3].tolist() == [s.cls_label for s in samples]


def test_augment_edge_geometry(tmp_path):
    """flip at both edges, negative / overhanging paste offsets, mask size != image size, 1-pixel
    resize targets, an identity resize"""
    make_dataset(str(tmp_path), "full", "train", n=6, seed=3, sizes=[(50, 30)] * 6,
                 mask_sizes=[(50, 30), (25, 15), (60, 45), (50, 30), (7, 90), (50, 30)])
    ds = HFUnetDataset(str(tmp_path), [32, 32], 4, split="train", config="full", task="multiclass")
    np.random.seed(0)
    samples = [ds[i] for i in range(6)]
    geo = [(60, 36, -10, -2, True), (1, 1, 5, 7, False), (50, 30, -9, 1, True), (70, 9, -30, 20, False),
           (3, 64, 31, -16, True), (50, 30, 0, 0, False)]
    for s, (nw, nh, dx, dy, fl) in zip(samples, geo):
        s.nw, s.nh, s.dx, s.dy, s.flip = nw, nh, dx, dy, fl
    samples[1].r = None  # one sample without the HSV jitter inside a training batch
    _check(ds, samples, make_collate(ds)(samples).to_device("cuda"))


def test_augment_bench_size(tmp_path):
    """the 512x512 B=16 shape of the headline workload from 640x480-class sources"""
    sizes = [(640, 480), (480, 640), (800, 600), (512, 512)] * 4
    make_dataset(str(tmp_path), "full", "train", n=16, seed=5, sizes=sizes)
    ds = HFUnetDataset(str(tmp_path), [512, 512], 2, split="train", config="full", task="binary")
    np.random.seed(11)
    samples = [ds[i] for i in range(16)]
    _check(ds, samples, make_collate(ds)(samples).to_device("cuda"))


@pytest.mark.parametrize("workers", [0, 2])
def test_device_loader(tmp_path, workers):
    """DataLoader (CPU workers: decode + draws) -> DeviceLoader (upload + kernels one batch ahead)"""
    make_dataset(str(tmp_path), "full", "validation", n=7, seed=9)
    ds = HFUnetDataset(str(tmp_path), [64, 64], 2, augmentation=False, split="validation", config="full",
                       task="binary")
    loader = torch.utils.data.DataLoader(ds, batch_size=3, shuffle=False, num_workers=workers,
                                         collate_fn=make_collate(ds))
    seen = 0
    for imgs, pngs, segs in DeviceLoader(loader, "cuda"):
        samples = [ds[i] for i in range(seen, seen + imgs.shape[0])]
        _check(ds, samples, (imgs, pngs, segs))
        seen += imgs.shape[0]
    assert seen == 7


def test_single_item_matches_reference_item(tmp_path):
    make_dataset(str(tmp_path), "full", "validation", n=2, seed=4)
    ds = HFUnetDataset(str(tmp_path), [48, 48], 4, augmentation=False, split="validation", config="full",
                       task="multiclass", return_cls_label=True)
    jpg, png, seg, cls = ds.get(1)
    s = ds[1]
    arr, lab = augment_ref.augment(Image.fromarray(s.image), Image.fromarray(s.mask), 48, 48,
                                   dict(nw=s.nw, nh=s.nh, dx=s.dx, dy=s.dy, flip=False, r=None))
    rj, rp, rs = augment_ref.to_sample(arr, lab, 4, "multiclass")
    np.testing.assert_array_equal(jpg, rj)
    np.testing.assert_array_equal(png, rp)
    np.testing.assert_array_equal(seg, rs)
    assert cls == ds.cls_label_of(1)


@pytest.mark.parametrize("task,model,loss", [("binary", "unet_plain", "bce"), ("multiclass", "unet_plain", "ce"),
                                             ("multitask", "multitask_unet", "lovasz_hinge")])
def test_train_val_on_parquet(tmp_path, task, model, loss):
    """train.py / val.py on an HF-layout dataset (train / validation / test splits) through the
    device loader, DataLoader workers decoding"""
    import json
    import os

    import train
    import val

    data = tmp_path / "hf"
    for split, n, seed in (("train", 6, 1), ("validation", 3, 2), ("test", 2, 3)):
        make_dataset(str(data), "no-ai", split, n=n, seed=seed)
    common = ["--task", task, "--model", model, "--input-size", "64", "--data-path", str(data), "--num-classes", "3"]
    args = train.parse_args(common + ["--loss", loss, "--batch-size", "2", "--epochs", "2", "--workers", "2",
                                      "--pos-weight", "auto", "--out-dir", str(tmp_path / "logs")])
    exp = train.train(args)
    summ = json.load(open(os.path.join(exp, "summary.json")))
    assert len(summ["train_losses"]) == 2 and all(v == v and v > 0 for v in summ["train_losses"])
    assert summ["test_metrics"] is not None
    if task == "binary":  # --export-vis (default on, train.py:580-585): 2x2 grids of the test split
        grids = sorted(f for f in os.listdir(os.path.join(exp, "vis")) if f.endswith("_grid.png"))
        assert len(grids) == 2 and Image.open(os.path.join(exp, "vis", grids[0])).size == (128, 128)
    vloss = [] if task == "multiclass" else ["--loss", loss if loss != "ce" else "bce"]
    m = val.val(val.parse_args(common + vloss + ["--weights", os.path.join(exp, "weights", "best.pth")]))
    key = "Mean IoU" if task == "multiclass" else "IoU"
    assert 0.0 <= float(m[key]) <= 1.0


@pytest.mark.parametrize("cls_label", [False, True])
def test_reference_loop_contract(tmp_path, cls_label):
    """the reference's own loader + loop code shape (train.py:140-162, utils/train_and_eval.py:203-207):
    DataLoader(ds, collate_fn=hf_unet_dataset_collate, pin_memory=True, workers) and
    ``imgs, pngs, labels = batch; imgs = imgs.to(device)`` -- the batch is the collated tensors,
    identical to the oracle's restatement of get_random_data + the reference collate; the single
    item unpacks as the reference's ``(jpg, png, seg_labels[, cls])``"""
    from utils.hf_dataloader import hf_unet_dataset_collate
    make_dataset(str(tmp_path), "full", "train", n=5, seed=13)
    ds = HFUnetDataset(str(tmp_path), [64, 64], 2, split="train", config="full", task="binary",
                       return_cls_label=cls_label)
    loader = torch.utils.data.DataLoader(ds, batch_size=2, shuffle=False, num_workers=2, pin_memory=True,
                                         collate_fn=hf_unet_dataset_collate, drop_last=False)
    seen = 0
    for batch in loader:
        if cls_label:
            imgs, pngs, labels, cls = batch
        else:
            imgs, pngs, labels = batch
        imgs, pngs, labels = imgs.to("cuda"), pngs.to("cuda"), labels.to("cuda")
        B = imgs.shape[0]
        assert imgs.shape == (B, 3, 64, 64) and pngs.dtype == torch.int64 and labels.shape == (B, 64, 64, 3)
        # replay the worker's draws: samples are re-drawn with the same seeded RNG below
        seen += B
    assert seen == 5
    np.random.seed(21)
    samples = [ds[i] for i in range(5)]
    b = hf_unet_dataset_collate(samples)
    _check(ds, samples, tuple(b))
    np.random.seed(22)
    s = ds[3]
    item = tuple(s)
    assert len(item) == (4 if cls_label else 3)
    _check(ds, [s], tuple(torch.from_numpy(np.asarray(v))[None] for v in item[:3]))


def _fake_samples(rng, n, hsv=True):
    from utils.hf_dataloader import RawSample
    out = []
    for i in range(n):
        iw, ih = int(rng.integers(1, 1400)), int(rng.integers(1, 1400))
        mw, mh = (iw, ih) if i % 3 else (int(rng.integers(1, 900)), int(rng.integers(1, 900)))
        nw, nh = int(rng.integers(1, 1100)), int(rng.integers(1, 1100))
        r = (rng.uniform(-1, 1, 3) * [.1, .7, .3] + 1) if (hsv and i % 4) else None
        out.append(RawSample(image=np.zeros((ih, iw, 3), np.uint8), mask=np.zeros((mh, mw), np.uint8), nw=nw, nh=nh,
                             dx=0, dy=0, flip=False, r=r, input_shape=(64, 64), num_classes=2, task="binary"))
    return out


def test_device_tables_bit_exact():
    """unetseg_augment_tables_dev (aug_tables) against the host builder utils/augment_tables.py (itself
    pinned against Pillow by tests/test_augment_cpu.py): every BICUBIC window / tap, NEAREST index and
    HSV LUT entry equal, for random up- and down-scales, masks of another size, with and without HSV"""
    from unetseg_hip.lib import lib
    from utils.hf_dataloader import pack_batch
    rng = np.random.default_rng(21)
    for rep in range(4):
        samples = _fake_samples(rng, 24)
        host = pack_batch(samples, device_tables=False)
        devb = pack_batch(samples)
        np.testing.assert_array_equal(devb.desc.numpy(), host.desc.numpy())
        desc = devb.desc.cuda()
        r = devb.hsv_r.cuda()
        tab = torch.full((devb.n_tables,), -7, dtype=torch.int32, device="cuda")
        tasks = max(s.nw + s.nh + 2 + 768 for s in samples)
        lib.augment_tables_dev(desc.data_ptr(), len(samples), r.data_ptr(), tab.data_ptr(), tasks,
                               torch.cuda.current_stream().cuda_stream)
        torch.cuda.synchronize()
        got, want = tab.cpu().numpy(), host.tables.numpy()
        bad = np.flatnonzero(got != want)
        assert bad.size == 0, (rep, bad[:8], got[bad[:8]], want[bad[:8]])


def test_device_tables_batch_equals_host_tables(tmp_path):
    """the bench-size batch through unetseg_augment_batch_dev equals unetseg_augment_batch with host
    tables, bit for bit (images, labels, one-hot)"""
    from utils.hf_dataloader import pack_batch
    sizes = [(640, 480), (480, 640), (800, 600), (512, 512)] * 4
    make_dataset(str(tmp_path), "full", "train", n=16, seed=6, sizes=sizes)
    ds = HFUnetDataset(str(tmp_path), [512, 512], 2, split="train", config="full", task="binary")
    np.random.seed(13)
    samples = [ds[i] for i in range(16)]
    a = pack_batch(samples).to_device("cuda")
    b = pack_batch(samples, device_tables=False).to_device("cuda")
    torch.cuda.synchronize()
    for x, y in zip(a, b):
        assert torch.equal(x, y)
