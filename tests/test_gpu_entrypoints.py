"""GPU: the drop-in entry points (train.py / val.py / utils.train_and_eval) and the mIoU criterion.

* train.py binary and multitask runs (tiny synthetic sets) complete, write the reference's
  artefacts (best/last state_dicts, metric history, summary) and val.py reloads the checkpoint;
* mIoU parity: eval-mode fp32 forward of unet_resnet50 on the same hash weights on a
  fixed synthetic set of 64 images at 512x512; the binary IoU from the HIP confusion kernel must be
  within 1e-4 of the CPU oracle's.
"""
import json
import os

import pytest
import torch

pytestmark = pytest.mark.gpu
DEV = "cuda"


@pytest.fixture(scope="module", autouse=True)
def _need_gpu():
    if not torch.cuda.is_available():
        pytest.skip("no GPU")


@pytest.mark.parametrize("task,model,loss", [("binary", "unet_plain", "lovasz_hinge"),
                                             ("binary", "unet_resnet50", "bce"),
                                             ("multitask", "multitask_unet", "bce")])
def test_train_and_val_entrypoints(tmp_path, task, model, loss):
    import train
    import val

    args = train.parse_args(["--task", task, "--model", model, "--loss", loss, "--input-size", "64", "--batch-size",
                             "2", "--epochs", "2", "--synthetic-train", "4", "--synthetic-val", "2", "--workers", "0",
                             "--out-dir", str(tmp_path)])
    exp = train.train(args)
    summ = json.load(open(os.path.join(exp, "summary.json")))
    assert summ["best_epoch"] in (1, 2)
    assert len(summ["train_losses"]) == 2 and all(l == l and l > 0 for l in summ["train_losses"])  # noqa: E741
    assert os.path.exists(os.path.join(exp, "weights", "last.pth"))
    hist = json.load(open(os.path.join(exp, "val_metrics_history.json")))
    assert len(hist) == 2 and 0.0 <= hist[-1]["IoU"] <= 1.0
    vargs = val.parse_args(["--weights", os.path.join(exp, "weights", "best.pth"), "--task", task, "--model", model,
                            "--input-size", "64", "--data-path", "synthetic", "--synthetic-test", "2"])
    m = val.val(vargs)
    assert 0.0 <= m["IoU"] <= 1.0


def test_miou_parity_unet_resnet50_512():
    from model.model_factory import build_model
    from oracle import ref_cpu
    from oracle.weights import make_torch_state
    from unetseg_hip import losses
    from utils.synthetic import make_batch
    from utils.train_and_eval import binary_segmentation_metrics

    torch.set_num_threads(16)
    state = make_torch_state(ref_cpu.model_spec("unet_resnet50", num_classes=2))
    params, buffers = ref_cpu.split_state(state)
    m = build_model("unet_resnet50", num_classes=2)
    m.load_state_dict(state)
    m = m.to(DEV).eval()
    m.compute_dtype = "fp32"
    conf = torch.zeros(4, dtype=torch.int64, device=DEV)
    rconf = [0, 0, 0, 0]
    nflip = 0
    for i in range(8):  # 64 images, 8 per batch
        x, y = make_batch(8, 512, seed=50_000 + i)
        with torch.no_grad():
            o = m(x.to(DEV))
            losses.binary_confusion(o, y.to(DEV), conf)
            ro = ref_cpu.forward("unet_resnet50", params, buffers, x, train=False)
        rconf = [a + b for a, b in zip(rconf, ref_cpu.binary_confusion(ro, y))]
        nflip += int(((ro[:, 1] - ro[:, 0]).abs() < 1e-4).sum())
        # 1e-3 per pixel, relative once |logit| > 1 (these hash-weight logits reach ~13 at 512^2)
        err = ((o.cpu() - ro).abs() / ro.abs().clamp(min=1.0)).max()
        assert err < 1e-3, err
    hip = binary_segmentation_metrics(*[float(v) for v in conf.tolist()])
    ref = binary_segmentation_metrics(*[float(v) for v in rconf])
    assert abs(hip["IoU"] - ref["IoU"]) < 1e-4, (hip, ref, nflip)
