"""CPU: host-side logic of the drop-in surface (no GPU): CLI defaults mirror the reference's
train.py:523-593, the factory's errors, and the no-fallback rule (a CPU forward raises)."""
import pytest
import torch


def test_train_cli_defaults_match_reference():
    import train

    a = train.parse_args([])
    assert (a.task, a.model, a.loss, a.batch_size, a.epochs, a.input_size) == ("binary", "unet_resnet50",
                                                                               "lovasz_hinge", 8, 50, 512)
    assert (a.momentum, a.weight_decay, a.amp, a.seed, a.cls_loss_weight) == (0.9, 1e-4, True, 11, 1.0)
    assert train.parse_args(["--pos-weight", ""]).pos_weight is None


def test_val_cli_defaults_match_reference():
    """val.py:158-187: every flag of the reference with its default (ce / focal accepted by --loss)"""
    import val

    a = val.parse_args([])
    assert (a.data_path, a.data_config, a.weights, a.task, a.model, a.loss) == (
        "./hf_datasets/merged_dataset_v2", "no-ai", "weights/unet_resnet_voc.pth", "binary", "unet_resnet50",
        "lovasz_hinge")
    assert (a.num_classes, a.input_size, a.cache_dir, a.device) == (4, 512, ".hf-cache/datasets", "cuda")
    for loss in ("bce", "lovasz_hinge", "ce", "focal"):
        assert val.parse_args(["--loss", loss]).loss == loss


def test_train_export_vis_default_matches_reference():
    import train

    assert train.parse_args([]).export_vis is True  # train.py:580-585
    assert train.parse_args(["--no-export-vis"]).export_vis is False


def test_optimizer_and_schedule_match_reference():
    """get_optimizer_and_lr: lr clamps to 1e-4 for any batch size; warm-cos epoch 0 = 1e-5."""
    import train
    from model.model_factory import build_model

    m = build_model("unet_plain", num_classes=2)
    for bs in (2, 8, 16, 64):
        opt, lr_fn = train.get_optimizer_and_lr(m, bs, 50, 0.9, 1e-4)
        assert opt.param_groups[0]["lr"] == pytest.approx(1e-4)
        assert opt.param_groups[0]["betas"] == (0.9, 0.999)
        assert lr_fn(0) == pytest.approx(1e-5)


def test_factory_errors_and_no_cpu_fallback():
    from model.model_factory import SUPPORTED_MODELS, build_model

    with pytest.raises(ValueError):
        build_model("no_such_model", num_classes=2)
    assert {"unet_resnet50", "unet_plain", "attention_unet", "multitask_unet"} <= set(SUPPORTED_MODELS)
    m = build_model("unet_plain", num_classes=2)
    with pytest.raises(RuntimeError):
        m(torch.zeros(1, 3, 32, 32))


def test_train_refuses_cpu_and_real_data():
    import train

    with pytest.raises((RuntimeError, NotImplementedError)):
        train.train(train.parse_args(["--device", "cpu", "--epochs", "1"]))


def test_binary_epoch_empty_loader_returns_zero(capsys):
    """an empty train loader returns 0 like the reference (utils/train_and_eval.py:
    185-263 divides by max(seen, 1)) instead of reading the image size of a batch that never came"""
    import contextlib
    import io

    import torch
    from model.model_factory import build_model
    from utils.train_and_eval import train_one_epoch_binary
    with contextlib.redirect_stdout(io.StringIO()):
        m = build_model("unet_plain", 2)
    opt = torch.optim.Adam(m.parameters(), lr=1e-4)
    out = train_one_epoch_binary(m, opt, [], torch.device("cpu"), "bce", None, False, None, 0, 1)
    assert out == 0.0
