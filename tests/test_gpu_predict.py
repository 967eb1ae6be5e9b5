"""GPU: predict.py (reference predict.py:41-145) against the CPU oracle.

The oracle does what the reference does per image: PIL letterbox to 480x480 (utils/utils.py:22-34),
/255 in float32, eval-mode fp32 forward (oracle/ref_cpu.py on the same hash weights), softmax,
crop of the letterbox window, bilinear resize to the original size with half-pixel centres and edge
clamp (cv2.INTER_LINEAR's rule; cv2 itself is absent, so that step is parity unpinned) and argmax.
Labels must agree wherever the oracle's top-2 probability margin exceeds 1e-3 (fp32 conv
reassociation moves probabilities by ~1e-5) and on >= 99.9 % of all pixels.
"""
import os

import numpy as np
import pytest
import torch
import torch.nn.functional as F
from PIL import Image

pytestmark = pytest.mark.gpu


def _oracle_labels(name, params, buffers, image):
    from oracle import ref_cpu
    from utils.utils import letterbox_params

    iw, ih = image.size
    nw, nh, dx, dy = letterbox_params(iw, ih, 480, 480)
    canvas = Image.new("RGB", (480, 480), (128, 128, 128))
    canvas.paste(image.resize((nw, nh), Image.BICUBIC), (dx, dy))
    x = torch.from_numpy(np.transpose(np.array(canvas, np.float32) / 255.0, (2, 0, 1))[None].copy())
    with torch.no_grad():
        pr = ref_cpu.forward(name, params, buffers, x, train=False)[0]
    pr = torch.softmax(pr, 0)[:, dy:dy + nh, dx:dx + nw]
    pr = F.interpolate(pr[None], size=(ih, iw), mode="bilinear", align_corners=False)[0]
    top2 = pr.topk(2, 0).values
    return pr.argmax(0).numpy(), (top2[0] - top2[1]).numpy(), x


@pytest.mark.parametrize("size", [(640, 427), (300, 512)])
def test_predict_labels_match_oracle(tmp_path, size):
    import predict
    from augment_data import make_image
    from model.model_factory import build_model
    from oracle import ref_cpu
    from oracle.weights import make_torch_state

    torch.set_num_threads(16)
    name, nc = "unet_resnet50", 3
    state = make_torch_state(ref_cpu.model_spec(name, num_classes=nc))
    wpath = tmp_path / "w.pth"
    torch.save(state, wpath)
    model = predict.load_model(name, str(wpath), nc, torch.device("cuda"))
    image = make_image(np.random.default_rng(size[0]), *size)
    got = predict.predict_labels(model, image, torch.device("cuda"))
    params, buffers = ref_cpu.split_state(build_model(name, num_classes=nc).state_dict() | state)
    ref, margin, x_ref = _oracle_labels(name, params, buffers, image)
    # the device letterbox is the PIL one, bit for bit
    x_dev, _, _ = predict.letterbox(image, torch.device("cuda"))
    np.testing.assert_array_equal(x_dev.cpu().numpy(), x_ref.numpy())
    assert got.shape == ref.shape == (size[1], size[0])
    sure = margin > 1e-3
    assert (got[sure] == ref[sure]).all(), int((got[sure] != ref[sure]).sum())
    assert (got == ref).mean() >= 0.999
    assert len(np.unique(ref)) > 1  # a non-degenerate label map


def test_predict_cli_writes_masks(tmp_path):
    import predict
    from augment_data import make_image
    from model.model_factory import build_model

    m = build_model("unet_plain", num_classes=3)
    wpath = tmp_path / "w.pth"
    torch.save(m.state_dict(), wpath)
    img_dir = tmp_path / "imgs"
    img_dir.mkdir()
    rng = np.random.default_rng(0)
    make_image(rng, 96, 64).save(img_dir / "a.jpg")
    make_image(rng, 50, 80, "L").save(img_dir / "b.png")
    (img_dir / "notes.txt").write_text("skip me")
    args = predict.parse_args(["--data_path", str(img_dir), "--weights", str(wpath), "--num-classes", "2",
                               "--model", "unet_plain", "--out-dir", str(tmp_path / "run")])
    saved = predict.predict(args)
    assert sorted(os.path.basename(p) for p in saved) == ["a_mask.png", "b_mask.png"]
    for p, (w, h) in zip(sorted(saved), [(96, 64), (50, 80)]):
        out = Image.open(p)
        assert out.size == (w, h) and out.mode == "RGB"
