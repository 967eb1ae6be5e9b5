"""DeviceLoader throughput on a synthetic HF-layout parquet set.

    python tools/loader_bench.py [--n 256] [--batch 16] [--size 512] [--workers 4 8 16] [--out FILE]

Writes a parquet dataset of JPEG images / PNG masks (640x480-class sources, the layout of the
reference's convert_and_upload.py) under $TMPDIR, then times, per worker count, full passes of
DataLoader(num_workers=W, collate_fn=hf_unet_dataset_collate) -> DeviceLoader (upload + device
augmentation one batch ahead): images/s delivered on the GPU, with the training-mode draws
(resize, flip, paste, HSV).  One warm-up pass per setting.  Prints one JSON object.
"""
import argparse
import json
import os
import sys
import tempfile
import time

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
for p in (REPO, os.path.join(REPO, "unet-embroidery-seg_amd"), os.path.join(REPO, "tests")):
    sys.path.insert(0, p)

import torch  # noqa: E402


def _cpu_quota():
    """CPUs this process may use per the cgroup quota (the GPU box grants a share of a larger host:
    more workers than this share contend with the main process and the pinning thread)"""
    try:
        q, per = open("/sys/fs/cgroup/cpu.max").read().split()[:2]
        return None if q == "max" else round(int(q) / int(per), 2)
    except (OSError, ValueError):
        return None


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--n", type=int, default=256)
    ap.add_argument("--batch", type=int, default=16)
    ap.add_argument("--size", type=int, default=512)
    ap.add_argument("--workers", type=int, nargs="+", default=[4, 8, 16])
    ap.add_argument("--passes", type=int, default=2)
    ap.add_argument("--out", default=None)
    a = ap.parse_args()
    from augment_data import make_dataset
    from utils.hf_dataloader import DeviceLoader, HFUnetDataset, hf_unet_dataset_collate

    root = tempfile.mkdtemp(prefix="loader_bench_")
    sizes = [(640, 480), (480, 640), (800, 600), (512, 512)] * (a.n // 4 + 1)
    t0 = time.perf_counter()
    make_dataset(root, "full", "train", n=a.n, seed=1, sizes=sizes[:a.n])
    t_make = time.perf_counter() - t0
    ds = HFUnetDataset(root, [a.size, a.size], 2, split="train", config="full", task="binary")
    res = {"dataset": f"{a.n} synthetic images (JPEG and PNG, 640x480-class) + PNG masks, parquet (convert_and_upload layout)",
           "batch": a.batch, "input_size": a.size, "task": "binary", "augmentation": True,
           "host_cpus_affinity": len(os.sched_getaffinity(0)), "cpu_quota": _cpu_quota(),
           "make_dataset_s": round(t_make, 1), "runs": []}
    for w in a.workers:
        for onehot in (False, True):
            # pin_memory=True as the reference's train.py:140-150 (RawBatch.pin_memory runs in the
            # DataLoader's pinning thread, off the main thread)
            dl = torch.utils.data.DataLoader(ds, batch_size=a.batch, shuffle=True, num_workers=w,
                                             collate_fn=hf_unet_dataset_collate, drop_last=True,
                                             persistent_workers=w > 0, pin_memory=True)
            loader = DeviceLoader(dl, "cuda", onehot=onehot)
            times = []
            for p in range(a.passes + 1):
                torch.cuda.synchronize()
                t0 = time.perf_counter()
                n = 0
                for imgs, pngs, segs in loader:
                    n += imgs.shape[0]
                torch.cuda.synchronize()
                if p > 0:
                    times.append((n, time.perf_counter() - t0))
            n = sum(x for x, _ in times)
            t = sum(y for _, y in times)
            res["runs"].append({"workers": w, "onehot": onehot, "images_per_s": round(n / t, 1),
                                "ms_per_batch": round(1e3 * t / (n / a.batch), 2)})
            print(res["runs"][-1], file=sys.stderr, flush=True)
            del dl, loader
    line = json.dumps(res)
    print(line)
    if a.out:
        open(a.out, "w").write(line + "\n")


if __name__ == "__main__":
    main()
