"""Helpers (reference: utils/utils.py:42-72)."""
import random

import numpy as np
import torch


def get_lr(optimizer):
    for param_group in optimizer.param_groups:
        return param_group["lr"]


def seed_everything(seed=11):
    random.seed(seed)
    np.random.seed(seed)
    torch.manual_seed(seed)
    torch.cuda.manual_seed(seed)
    torch.cuda.manual_seed_all(seed)
    torch.backends.cudnn.deterministic = True
    torch.backends.cudnn.benchmark = False


def worker_init_fn(worker_id, seed=0):
    worker_seed = worker_id + seed
    random.seed(worker_seed)
    np.random.seed(worker_seed)
    torch.manual_seed(worker_seed)


def preprocess_input(image):
    image /= 255.0
    return image


def cvtColor(image):
    """utils/utils.py:11-16: anything but a 3-channel image is converted to RGB"""
    if len(np.shape(image)) == 3 and np.shape(image)[2] == 3:
        return image
    return image.convert("RGB")


def letterbox_params(iw, ih, w, h):
    """resize_image's geometry (utils/utils.py:22-34): (nw, nh, dx, dy) of the centred paste"""
    scale = min(w / iw, h / ih)
    nw, nh = int(iw * scale), int(ih * scale)
    return nw, nh, (w - nw) // 2, (h - nh) // 2
