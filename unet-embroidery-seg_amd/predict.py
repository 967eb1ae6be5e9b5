"""Single-image / folder inference on the HIP path (reference: predict.py:32-175).

Per image, as the reference: RGB conversion, 480x480 letterbox (PIL BICUBIC resize onto a
(128,128,128) canvas), /255, eval-mode forward, softmax, crop of the letterbox window, bilinear
resize to the original size, argmax, palette colours, optional 0.3 / 0.7 blend with the original,
``<name>_mask.png`` in ``run/predict/expN``.  Here the letterbox runs in the loader's augmentation
kernels (csrc/augment.hip, bit-exact with PIL; its /255 equals the reference's float32 division for
every byte value), the model on the HIP kernels, and softmax + crop + resize + argmax is one kernel
(unetseg_softmax_resize_argmax).  The reference resizes with cv2.INTER_LINEAR (half-pixel centres,
edge clamp) and blends with cv2.addWeighted; cv2 is absent here, so the label map follows that
published rule (parity unpinned, see tests/test_gpu_predict.py) and the blend is
round-half-even of 0.3 a + 0.7 b in float32.
"""
from __future__ import annotations

import argparse
import colorsys
import os
import sys
import time
from pathlib import Path

_HERE = os.path.dirname(os.path.abspath(__file__))
if _HERE not in sys.path:
    sys.path.insert(0, _HERE)

import numpy as np  # noqa: E402
import torch  # noqa: E402
from PIL import Image  # noqa: E402

from model.model_factory import SUPPORTED_MODELS, build_model  # noqa: E402
from unetseg_hip.lib import lib  # noqa: E402
from utils.hf_dataloader import RawSample, pack_batch  # noqa: E402
from utils.utils import cvtColor, letterbox_params  # noqa: E402

INPUT_SHAPE = (480, 480)  # predict.py:55
VOC_COLORS = [(0, 0, 0), (128, 0, 0), (0, 128, 0), (128, 128, 0), (0, 0, 128), (128, 0, 128), (0, 128, 128),
              (128, 128, 128), (64, 0, 0), (192, 0, 0), (64, 128, 0), (192, 128, 0), (64, 0, 128), (192, 0, 128),
              (64, 128, 128), (192, 128, 128), (0, 64, 0), (128, 64, 0), (0, 192, 0), (128, 192, 0), (0, 64, 128),
              (128, 64, 128)]


def time_synchronized():
    """predict.py:16-30"""
    if torch.cuda.is_available():
        torch.cuda.synchronize()
    return time.time()


def colors_for(num_classes):
    """predict.py:62-70"""
    if num_classes <= 21:
        return VOC_COLORS
    hsv = [(x / num_classes, 1., 1.) for x in range(num_classes)]
    return [(int(r * 255), int(g * 255), int(b * 255)) for r, g, b in (colorsys.hsv_to_rgb(*t) for t in hsv)]


def load_model(model_name, model_path, num_classes, device):
    """predict.py:32-38 (weights_only load)"""
    net = build_model(model_name, num_classes=num_classes)
    net.load_state_dict(torch.load(model_path, map_location="cpu", weights_only=True))
    net.eval()
    net.to(device)
    return net


def letterbox(image, device):
    """resize_image + preprocess_input on the device: fp32 [1,3,480,480] and (nw, nh)"""
    iw, ih = image.size
    nw, nh, dx, dy = letterbox_params(iw, ih, INPUT_SHAPE[1], INPUT_SHAPE[0])
    s = RawSample(image=np.asarray(image, np.uint8), mask=np.zeros((1, 1), np.uint8), nw=nw, nh=nh, dx=dx, dy=dy,
                  flip=False, r=None)
    x = pack_batch([s], INPUT_SHAPE, 1, "binary").to_device(device, onehot=False)[0]
    return x, nw, nh


def predict_labels(model, image, device):
    """predict.py:72-93: the argmax label map int32 [H][W] at the image's original size"""
    x, nw, nh = letterbox(image, device)
    with torch.no_grad():
        pr = model(x)[0].float().contiguous()
    C, H, W = pr.shape
    ow, oh = image.size
    labels = torch.empty(oh, ow, dtype=torch.int32, device=device)
    lib.softmax_resize_argmax(pr.data_ptr(), C, H, W, (INPUT_SHAPE[0] - nh) // 2, (INPUT_SHAPE[1] - nw) // 2, nh, nw,
                              oh, ow, labels.data_ptr(), torch.cuda.current_stream(device).cuda_stream)
    return labels.cpu().numpy()


def blend(old, seg, alpha=0.7):
    """cv2.addWeighted(old, 1 - alpha, seg, alpha, 0) for uint8 (float32 arithmetic, round half even)"""
    f = np.float32
    v = old.astype(f) * f(1 - alpha) + seg.astype(f) * f(alpha)
    return np.clip(np.rint(v), 0, 255).astype(np.uint8)


def detect_image(file_path, model, num_classes, exp_folder, mix_type=True, device=None):
    """predict.py:41-109"""
    try:
        image = Image.open(file_path)
    except (FileNotFoundError, IOError) as e:
        print(f"Error opening image: {e}")
        return None
    device = device or torch.device("cuda")
    image = cvtColor(image)
    old_img = image.copy()
    pr = predict_labels(model, image, device)
    oh, ow = pr.shape
    seg_img = np.reshape(np.array(colors_for(num_classes), np.uint8)[np.reshape(pr, [-1])], [oh, ow, -1])
    out = Image.fromarray(blend(np.array(old_img), seg_img)) if mix_type else Image.fromarray(np.uint8(seg_img))
    save_path = os.path.join(exp_folder, os.path.splitext(os.path.basename(file_path))[0] + "_mask.png")
    out.save(save_path)
    print(f"Mask saved at: {save_path}")
    return save_path


def create_val_exp_folder(root="run"):
    """utils/create_exp_folder.py:33-56: run/predict/expN (first free N >= 1)"""
    base = os.path.join(root, "predict")
    os.makedirs(os.path.join(base, "exp"), exist_ok=True)
    n = 1
    while os.path.exists(os.path.join(base, f"exp{n}")):
        n += 1
    path = os.path.join(base, f"exp{n}")
    os.mkdir(path)
    return path


def predict(args):
    """predict.py:112-145"""
    exp_folder = create_val_exp_folder(args.out_dir)
    num_classes = args.num_classes + 1
    assert os.path.exists(args.weights), f"weights {args.weights} not found."
    if not torch.cuda.is_available():
        raise RuntimeError("the HIP inference path needs a GPU (no CPU fallback)")
    device = torch.device("cuda")
    model = load_model(args.model, args.weights, num_classes, device)
    if os.path.isdir(args.data_path):
        files = [str(p) for p in Path(args.data_path).rglob("*") if p.suffix in [".jpg", ".png", ".jpeg"]]
    elif os.path.isfile(args.data_path):
        files = [args.data_path]
    else:
        raise ValueError(f"Unsupported input path: {args.data_path}")
    t0 = time_synchronized()
    saved = [detect_image(f, model, num_classes, exp_folder, mix_type=args.mix_type, device=device)
             for f in files if f.endswith((".jpg", ".png", ".jpeg"))]
    print(f"inference time for: {time_synchronized() - t0}")
    return saved


def parse_args(argv=None):
    """predict.py:148-175"""
    p = argparse.ArgumentParser(description="U-Net predict on the MI355X HIP path")
    p.add_argument("--data_path", default="VOCdevkit/VOC2012/JPEGImages/2007_000129.jpg")
    p.add_argument("--weights", default="run/train/exp10/weights/best_model_20.pth")
    p.add_argument("--num-classes", default=20, type=int)
    p.add_argument("--model", default="unet_resnet50", choices=sorted(SUPPORTED_MODELS.keys()))
    p.add_argument("--mix_type", default=True, action="store_true")
    p.add_argument("--out-dir", default="run")
    return p.parse_args(argv)


if __name__ == "__main__":
    predict(parse_args())
