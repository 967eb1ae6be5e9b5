"""CPU: the reference's initial weights, bit for bit.

``train.create_model`` (reference train.py:48-59) = ``build_model`` + ``weights_init``
(model/unet_training.py:94-113) after ``seed_everything(11)`` (utils/utils.py:50-57).  The HIP models
keep the reference's module tree, parameter registration and constructor RNG consumption (conv /
linear default inits, the ResNet's own normal_ init, then weights_init's normal_ draws), so under
the same seed every state_dict entry must be bitwise identical.  tests/golden/init_seed11.npz holds
the sha256 of every entry's bytes as produced by the reference itself (oracle/gen_golden.py init).
"""
import contextlib
import hashlib
import io
import os

import numpy as np
import pytest
import torch

CASES = [("unet_plain", dict(num_classes=2)), ("unet_resnet50", dict(num_classes=2)),
         ("attention_unet", dict(num_classes=2)),
         ("multitask_unet", dict(num_classes=1, num_seg_classes=1, num_cls_classes=3)),
         ("dualdense_unet", dict(num_classes=2)), ("dualdense_unet", dict(num_classes=5))]


@pytest.mark.parametrize("name,kw", CASES, ids=[f"{n}_c{k['num_classes']}" for n, k in CASES])
def test_create_model_seed11_bit_exact(golden_dir, name, kw):
    from model.model_factory import build_model
    from model.unet_training import weights_init
    d = np.load(os.path.join(golden_dir, "init_seed11.npz"))
    tag = f"{name}_c{kw['num_classes']}"
    torch.manual_seed(11)
    with contextlib.redirect_stdout(io.StringIO()):
        m = build_model(name, **kw)
        weights_init(m)
    sd = m.state_dict()
    keys = list(d[tag + "::keys"])
    assert list(sd.keys()) == keys
    bad = []
    for k, digest, head in zip(keys, d[tag + "::sha256"], d[tag + "::head"]):
        a = sd[k].detach().contiguous().numpy()
        if hashlib.sha256(a.tobytes()).hexdigest() != digest:
            bad.append((k, a.reshape(-1)[:4], head[:4]))
    assert not bad, f"{len(bad)} entries differ, first: {bad[:3]}"


def test_train_create_model_matches(golden_dir):
    """train.create_model (the reference entry point, same name and arguments) gives the same init"""
    import train
    d = np.load(os.path.join(golden_dir, "init_seed11.npz"))
    torch.manual_seed(11)
    with contextlib.redirect_stdout(io.StringIO()):
        m = train.create_model("unet_resnet50", 2, "")
    sd = m.state_dict()
    for k, digest in zip(d["unet_resnet50_c2::keys"], d["unet_resnet50_c2::sha256"]):
        assert hashlib.sha256(sd[k].detach().contiguous().numpy().tobytes()).hexdigest() == digest, k
