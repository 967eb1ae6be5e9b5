"""Seeded synthetic embroidery-like batches: the HF dataset is not available offline.

image float32 [B,3,S,S] in [0,1): 0.5 + low-frequency noise + coloured filled ellipses;
mask  int64   [B,S,S] in {0,1}: union of 1-4 random ellipses (~30 % foreground);
cls   int64   [B] in {0,1,2}.
"""
import numpy as np
import torch


def make_batch(batch, size, seed, with_cls=False):
    rng = np.random.default_rng(seed)
    yy, xx = np.mgrid[0:size, 0:size].astype(np.float32)
    imgs = np.empty((batch, 3, size, size), np.float32)
    masks = np.zeros((batch, size, size), np.int64)
    for b in range(batch):
        coarse = rng.random((3, 8, 8), dtype=np.float32)
        rep = int(np.ceil(size / 8))
        low = np.kron(coarse, np.ones((rep, rep), np.float32))[:, :size, :size]
        img = 0.35 + 0.3 * low
        for _ in range(int(rng.integers(1, 5))):
            cy, cx = rng.random(2) * size
            ry, rx = (0.08 + 0.22 * rng.random(2)) * size
            ell = ((yy - cy) / ry) ** 2 + ((xx - cx) / rx) ** 2 < 1.0
            masks[b][ell] = 1
            color = rng.random(3).astype(np.float32)
            img[:, ell] = 0.5 * img[:, ell] + 0.5 * color[:, None]
        img += 0.05 * rng.standard_normal(img.shape, dtype=np.float32)
        imgs[b] = np.clip(img, 0.0, 0.999)
    x, y = torch.from_numpy(imgs), torch.from_numpy(masks)
    if with_cls:
        return x, y, torch.from_numpy(rng.integers(0, 3, batch).astype(np.int64))
    return x, y


class SyntheticSegDataset(torch.utils.data.Dataset):
    """Drop-in for HFUnetDataset's item contract (utils/hf_dataloader.py:67-105): (jpg, png, seg_labels[, cls])."""

    def __init__(self, length, input_shape, num_classes=2, seed=1234, return_cls_label=False):
        self.length, self.size, self.num_classes = length, int(input_shape[0]), num_classes
        self.seed, self.return_cls_label = seed, return_cls_label

    def __len__(self):
        return self.length

    def __getitem__(self, i):
        out = make_batch(1, self.size, self.seed + i, with_cls=True)
        x, y, c = out[0][0].numpy(), out[1][0].numpy(), int(out[2][0])
        seg = np.eye(self.num_classes + 1, dtype=np.float32)[y.reshape(-1)].reshape(self.size, self.size, -1)
        return (x, y, seg, c) if self.return_cls_label else (x, y, seg)


def collate(batch):
    """hf_unet_dataset_collate (utils/hf_dataloader.py:183-213)"""
    cols = list(zip(*batch))
    x = torch.from_numpy(np.stack(cols[0])).float()
    y = torch.from_numpy(np.stack(cols[1])).long()
    s = torch.from_numpy(np.stack(cols[2])).float()
    if len(cols) == 4:
        return x, y, s, torch.tensor(cols[3], dtype=torch.long)
    return x, y, s
