"""TEST INFRASTRUCTURE ONLY (see oracle/__init__.py) — golden-vector generator.

Run in the survey/build container only (the reference does not exist on the GPU box):

    PYTHONDONTWRITEBYTECODE=1 python oracle/gen_golden.py

It imports the reference read-only from /root/reference (model/*, utils/train_and_eval.py;
train.py is NOT imported: it needs cv2, so its ten lines of optimizer construction,
train.py:62-78, are restated here) and writes small .npz fixtures under tests/golden/.
The fixtures are data (inputs + the reference's outputs); no reference source travels.
"""
from __future__ import annotations

import os
import sys

import numpy as np
import torch

HERE = os.path.dirname(os.path.abspath(__file__))
REPO = os.path.dirname(HERE)
REF = os.environ.get("UNETSEG_REFERENCE", "/root/reference")
OUT = os.path.join(REPO, "tests", "golden")
sys.path.insert(0, REPO)

from oracle.weights import make_torch_state  # noqa: E402


def synth(b, s, seed):
    """Small seeded inputs: smooth image in [0,1) + blob mask (≈30 % foreground)."""
    g = torch.Generator().manual_seed(seed)
    img = torch.rand(b, 3, s, s, generator=g)
    img = 0.5 * img + 0.5 * torch.nn.functional.avg_pool2d(img, 5, 1, 2)
    yy, xx = torch.meshgrid(torch.arange(s), torch.arange(s), indexing="ij")
    mask = torch.zeros(b, s, s, dtype=torch.int64)
    for i in range(b):
        for _ in range(3):
            c = torch.rand(2, generator=g) * s
            r = (0.15 + 0.2 * torch.rand(2, generator=g)) * s
            mask[i] |= ((((yy - c[0]) / r[0]) ** 2 + ((xx - c[1]) / r[1]) ** 2) < 1).long()
    return img.float(), mask


def ref_model(name, **kw):
    from model.model_factory import build_model

    return build_model(name, **kw)


def load_hash(model):
    spec = [(k, tuple(v.shape)) for k, v in model.state_dict().items()]
    model.load_state_dict(make_torch_state(spec))
    return spec


def main():
    sys.path.insert(0, REF)
    sys.dont_write_bytecode = True
    from model.unet_training import get_lr_scheduler, lovasz_hinge_loss
    from model.unet_multitask import MultiTaskLoss
    from utils.train_and_eval import (_binary_confusion_from_pred, binary_segmentation_loss,
                                      binary_segmentation_metrics)

    os.makedirs(OUT, exist_ok=True)
    torch.set_num_threads(8)
    cases = [("unet_plain", 128, 2), ("unet_resnet50", 64, 2), ("attention_unet", 64, 2), ("multitask_unet", 64, 2)]
    for name, s, b in cases:
        torch.manual_seed(0)
        kw = dict(num_classes=1, num_seg_classes=1, num_cls_classes=3) if name == "multitask_unet" else dict(num_classes=2)
        m = ref_model(name, **kw)
        spec = load_hash(m)
        x, y = synth(b, s, seed=1000 + s)
        rec = {"x": x.numpy(), "y": y.numpy(),
               "spec_names": np.array([n for n, _ in spec]),
               "spec_shapes": np.array([",".join(map(str, sh)) for _, sh in spec])}
        m.train()
        if name == "multitask_unet":
            drop = (torch.Generator().manual_seed(7), )
            mask = (torch.rand(b, 512, generator=drop[0]) >= 0.5).float()
            m.cls_head[4].register_forward_hook(lambda mod, inp, out: inp[0] * mask * 2.0)
            cls_t = torch.tensor([0, 2][:b])
            seg, cls = m(x)
            crit = MultiTaskLoss(seg_loss_fn=torch.nn.BCEWithLogitsLoss(), cls_loss_weight=1.0)
            loss, sl, cl = crit(seg, cls, y, cls_t)
            loss.backward()
            rec.update(dropout_mask=mask.numpy(), cls_t=cls_t.numpy(), seg=seg.detach().numpy(),
                       cls=cls.detach().numpy(), loss=np.array([loss.item(), sl.item(), cl.item()]))
        else:
            out = m(x)
            loss = binary_segmentation_loss(out, y, "lovasz_hinge")
            loss.backward()
            with torch.no_grad():
                bce = binary_segmentation_loss(out, y, "bce")
                bce_pw = binary_segmentation_loss(out, y, "bce", pos_weight=torch.tensor([2.5]))
            rec.update(out=out.detach().numpy(), loss=np.array([loss.item(), bce.item(), bce_pw.item()]))
        # gradients: L2 norm of every param grad + full grads of a few small tensors
        gnames, gnorms = [], []
        for k, p in m.named_parameters():
            gnames.append(k)
            gnorms.append(float(p.grad.double().norm()))
        rec["grad_names"] = np.array(gnames)
        rec["grad_norms"] = np.array(gnorms)
        last = [k for k, _ in m.named_parameters()][-2:]
        first_bn = [k for k in gnames if k.endswith(".weight") and m.state_dict()[k].dim() == 1][:1]
        for k in last + first_bn:
            rec["grad::" + k] = dict(m.named_parameters())[k].grad.numpy()
        # running stats after one train forward (first BN)
        sd = m.state_dict()
        rm_keys = [k for k in sd if k.endswith("running_mean")][:2]
        for k in rm_keys:
            rec["state::" + k] = sd[k].numpy()
            rec["state::" + k.replace("running_mean", "running_var")] = sd[k.replace("running_mean", "running_var")].numpy()
        # eval-mode (running stats) fp32 output
        m.eval()
        with torch.no_grad():
            o = m(x)
            rec["eval_out"] = (o[0] if isinstance(o, tuple) else o).numpy()
            if name != "multitask_unet":
                tp, fp, fn, tn = _binary_confusion_from_pred(o.argmax(1), y)
                rec["eval_conf"] = np.array([tp, fp, fn, tn], dtype=np.int64)
        # CPU-autocast-bf16 train-mode output (reference default CPU semantics)
        if name in ("unet_plain", "unet_resnet50"):
            m2 = ref_model(name, **kw)
            load_hash(m2)
            m2.train()
            with torch.no_grad(), torch.autocast("cpu", dtype=torch.bfloat16):
                rec["out_bf16"] = m2(x).float().numpy()
        np.savez_compressed(os.path.join(OUT, f"model_{name}.npz"), **rec)
        print("wrote", name, {k: v.shape for k, v in rec.items() if not k.startswith("grad::")} if False else "")

    # ---- loss fixtures ------------------------------------------------------------------
    g = torch.Generator().manual_seed(3)
    logits = torch.randn(3, 40, 48, generator=g) * 2.0
    labels = (torch.rand(3, 40, 48, generator=g) < 0.35).float()
    lg = logits.clone().requires_grad_(True)
    lv = lovasz_hinge_loss(lg, labels)
    lv.backward()
    tied = logits.to(torch.bfloat16).float()
    tied = torch.round(tied * 4) / 4                              # heavy ties
    lv_t = lovasz_hinge_loss(tied, labels)
    two = torch.randn(3, 2, 40, 48, generator=g)
    tgt = (torch.rand(3, 40, 48, generator=g) < 0.4).long()
    twog = two.clone().requires_grad_(True)
    bce = binary_segmentation_loss(twog, tgt, "bce", pos_weight=torch.tensor([1.7]))
    bce.backward()
    empty = lovasz_hinge_loss(torch.zeros(0, 4, 4), torch.zeros(0, 4, 4))
    np.savez_compressed(os.path.join(OUT, "losses.npz"), logits=logits.numpy(), labels=labels.numpy(),
                        lovasz=np.array([lv.item()]), lovasz_grad=lg.grad.numpy(),
                        tied=tied.numpy(), lovasz_tied=np.array([lv_t.item()]),
                        two=two.numpy(), tgt=tgt.numpy(), bce_pw=np.array([bce.item()]),
                        bce_grad=twog.grad.numpy(), empty=np.array([float(empty)]))

    # ---- metric fixture -----------------------------------------------------------------
    outs = torch.randn(4, 2, 33, 35, generator=g)
    outs[0, :, :4, :4] = 0.0                                     # argmax ties -> class 0
    tg = (torch.rand(4, 33, 35, generator=g) < 0.3).long()
    conf = _binary_confusion_from_pred(outs.argmax(1), tg)
    met = binary_segmentation_metrics(*conf)
    np.savez_compressed(os.path.join(OUT, "metrics.npz"), outs=outs.numpy(), tg=tg.numpy(),
                        conf=np.array(conf, dtype=np.int64),
                        met=np.array([met[k] for k in ("Dice", "IoU", "Precision", "Recall", "Accuracy")]))

    # ---- LR schedule + Adam trajectory (train.py:62-78 restated; model/unet_training.py) -
    for E in (1, 5, 10, 50, 100, 300):
        f = get_lr_scheduler("cos", 1e-4, 1e-6, E)
        np.save(os.path.join(OUT, f"lr_cos_E{E}.npy"), np.array([f(e) for e in range(E)]))
    torch.manual_seed(0)
    m = ref_model("unet_plain", num_classes=2)
    load_hash(m)
    x, y = synth(2, 64, seed=55)
    opt = torch.optim.Adam(m.parameters(), 1e-4, betas=(0.9, 0.999), weight_decay=1e-4)
    sched = get_lr_scheduler("cos", 1e-4, 1e-6, 5)
    traj = []
    m.train()
    for ep in range(5):
        for pg in opt.param_groups:
            pg["lr"] = sched(ep)
        opt.zero_grad()
        loss = binary_segmentation_loss(m(x), y, "lovasz_hinge")
        loss.backward()
        opt.step()
        traj.append(loss.item())
    fin = {k: v.numpy() for k, v in m.state_dict().items() if k in ("outc.weight", "outc.bias", "inc.net.0.weight")}
    np.savez_compressed(os.path.join(OUT, "trajectory_unet_plain.npz"), x=x.numpy(), y=y.numpy(),
                        loss=np.array(traj), **{"final::" + k: v for k, v in fin.items()})
    print("golden fixtures written to", OUT)


def gen_init():
    """init_seed11.npz: the reference's create_model init (train.py:48-59 = build_model +
    weights_init, model/unet_training.py:94-113) under torch.manual_seed(11) (train.py seeds 11 via
    seed_everything, utils/utils.py:50-57).  Per state_dict entry: sha256 of the float32/int64
    bytes (bit-exact pin without shipping 176 MB) plus the first 8 values."""
    import hashlib

    sys.path.insert(0, REF)
    sys.dont_write_bytecode = True
    from model.model_factory import build_model
    from model.unet_training import weights_init

    rec = {}
    for name, kw in [("unet_plain", dict(num_classes=2)), ("unet_resnet50", dict(num_classes=2)),
                     ("attention_unet", dict(num_classes=2)),
                     ("multitask_unet", dict(num_classes=1, num_seg_classes=1, num_cls_classes=3)),
                     ("dualdense_unet", dict(num_classes=2)), ("dualdense_unet", dict(num_classes=5))]:
        torch.manual_seed(11)
        m = build_model(name, **kw)
        weights_init(m)
        tag = f"{name}_c{kw['num_classes']}"
        keys, digests, heads = [], [], []
        for k, v in m.state_dict().items():
            a = v.detach().contiguous().numpy()
            keys.append(k)
            digests.append(hashlib.sha256(a.tobytes()).hexdigest())
            h = np.zeros(8, dtype=np.float64)
            flat = a.reshape(-1)[:8].astype(np.float64)
            h[:flat.size] = flat
            heads.append(h)
        rec[tag + "::keys"] = np.array(keys)
        rec[tag + "::sha256"] = np.array(digests)
        rec[tag + "::head"] = np.stack(heads)
    np.savez_compressed(os.path.join(OUT, "init_seed11.npz"), **rec)
    print("wrote init_seed11.npz")


def gen_loop():
    """loop_unet_plain.npz: the reference's own train_one_epoch_binary (utils/train_and_eval.py:185-263,
    fp32: scaler None) for 3 epochs of 2 batches with the warm-cos LR (set_optimizer_lr per epoch) and
    Adam (train.py:62-78), then evaluate_binary (:266-305) on a validation list."""
    sys.path.insert(0, REF)
    sys.dont_write_bytecode = True
    import contextlib
    import io

    from model.unet_training import get_lr_scheduler, set_optimizer_lr
    from utils.train_and_eval import evaluate_binary, train_one_epoch_binary

    torch.set_num_threads(8)
    torch.manual_seed(0)
    m = ref_model("unet_plain", num_classes=2)
    load_hash(m)
    batches = []
    for i in range(2):
        x, y = synth(2, 64, seed=700 + i)
        batches.append((x, y, torch.zeros(1)))
    vx, vy = synth(2, 64, seed=777)
    val = [(vx, vy, torch.zeros(1))]
    opt = torch.optim.Adam(m.parameters(), 1e-4, betas=(0.9, 0.999), weight_decay=1e-4)
    sched = get_lr_scheduler("cos", 1e-4, 1e-6, 3)
    losses_ep = []
    dev = torch.device("cpu")
    with contextlib.redirect_stdout(io.StringIO()):
        for ep in range(3):
            set_optimizer_lr(opt, sched, ep)
            losses_ep.append(train_one_epoch_binary(m, opt, batches, dev, "lovasz_hinge", None, 0.0, None, ep, 3))
        met = evaluate_binary(m, val, dev, "lovasz_hinge", None)
    fin = {k: v.numpy() for k, v in m.state_dict().items() if k in ("outc.weight", "outc.bias", "up4.conv.net.3.weight")}
    rec = {"x%d" % i: b[0].numpy() for i, b in enumerate(batches)}
    rec.update({"y%d" % i: b[1].numpy() for i, b in enumerate(batches)})
    rec.update(vx=vx.numpy(), vy=vy.numpy(), epoch_loss=np.array(losses_ep),
               metrics=np.array([met[k] for k in ("Dice", "IoU", "Precision", "Recall", "Accuracy", "Loss")]))
    rec.update({"final::" + k: v for k, v in fin.items()})
    np.savez_compressed(os.path.join(OUT, "loop_unet_plain.npz"), **rec)
    print("wrote loop_unet_plain.npz", losses_ep, met)


def gen_multiclass():
    """multiclass.npz: the reference's CE_Loss / Focal_Loss / Dice_loss (values + logit gradients;
    class weights, the ignore label num_classes, a non-matching size that triggers their logit
    interpolation) and the four multiclass metrics (utils/train_and_eval.py:20-103)."""
    sys.path.insert(0, REF)
    sys.dont_write_bytecode = True
    from model.unet_training import CE_Loss, Dice_loss, Focal_Loss
    from utils.train_and_eval import frequency_weighted_iou, mean_accuracy, mean_iou, pixel_accuracy

    g = torch.Generator().manual_seed(21)
    rec = {}
    for tag, (n, c, h, w, ht, wt) in {"a": (2, 5, 24, 20, 24, 20), "b": (3, 21, 16, 16, 16, 16),
                                      "r": (2, 4, 12, 10, 24, 20)}.items():
        logits = torch.randn(n, c, h, w, generator=g) * 2
        tgt = torch.randint(0, c + 1, (n, ht, wt), generator=g)  # c = ignore label (num_classes)
        onehot = torch.eye(c + 1)[tgt.reshape(-1)].reshape(n, ht, wt, c + 1)
        cw = (0.5 + torch.rand(c, generator=g)).float()
        rec[f"{tag}_logits"], rec[f"{tag}_tgt"], rec[f"{tag}_onehot"], rec[f"{tag}_cw"] = (
            logits.numpy(), tgt.numpy(), onehot.numpy(), cw.numpy())
        for name, fn in {"ce": lambda x: CE_Loss(x, tgt, cw, num_classes=c),
                         "ce1": lambda x: CE_Loss(x, tgt, torch.ones(c), num_classes=c),
                         "focal": lambda x: Focal_Loss(x, tgt, cw, num_classes=c),
                         "dice": lambda x: Dice_loss(x, onehot)}.items():
            x = logits.clone().requires_grad_(True)
            v = fn(x)
            v.backward()
            rec[f"{tag}_{name}"] = np.array([v.item()])
            rec[f"{tag}_{name}_grad"] = x.grad.numpy()
        if (h, w) == (ht, wt):
            rec[f"{tag}_metrics"] = np.array([pixel_accuracy(logits, tgt), mean_accuracy(logits, tgt, c),
                                              mean_iou(logits, tgt, c), frequency_weighted_iou(logits, tgt, c)])
    np.savez_compressed(os.path.join(OUT, "multiclass.npz"), **rec)
    print("wrote multiclass.npz")


def gen_ignore():
    """ignore.npz: binary_segmentation_loss / lovasz_hinge_loss / confusion with ignore_index (255)
    (utils/train_and_eval.py:116-182, model/unet_training.py:253-280)."""
    sys.path.insert(0, REF)
    sys.dont_write_bytecode = True
    from model.unet_training import lovasz_hinge_loss
    from utils.train_and_eval import _binary_confusion_from_pred, binary_segmentation_loss

    g = torch.Generator().manual_seed(31)
    two = torch.randn(3, 2, 20, 24, generator=g) * 2
    tgt = (torch.rand(3, 20, 24, generator=g) < 0.4).long()
    tgt[torch.rand(3, 20, 24, generator=g) < 0.2] = 255
    tgt[2] = 255  # one image entirely ignored
    rec = {"two": two.numpy(), "tgt": tgt.numpy()}
    for name in ("bce", "lovasz_hinge"):
        x = two.clone().requires_grad_(True)
        v = binary_segmentation_loss(x, tgt, name, pos_weight=torch.tensor([1.3]) if name == "bce" else None,
                                     ignore_index=255)
        v.backward()
        rec[f"{name}"] = np.array([v.item()])
        rec[f"{name}_grad"] = x.grad.numpy()
    z = (two[:, 1] - two[:, 0]).clone().requires_grad_(True)
    v = lovasz_hinge_loss(z, tgt, ignore_index=255)
    v.backward()
    rec["lovasz_direct"] = np.array([v.item()])
    rec["lovasz_direct_grad"] = z.grad.numpy()
    rec["conf"] = np.array(_binary_confusion_from_pred(two.argmax(1), tgt, ignore_index=255), dtype=np.int64)
    np.savez_compressed(os.path.join(OUT, "ignore.npz"), **rec)
    print("wrote ignore.npz", rec["bce"], rec["lovasz_hinge"], rec["lovasz_direct"], rec["conf"])


def gen_models2():
    """model_dualdense_unet.npz and odd-size fixtures (unet_plain / attention_unet / dualdense at 72x88:
    the pad-then-cat and interpolate branches), hash weights, train mode fp32: logits, loss, grad norms."""
    sys.path.insert(0, REF)
    sys.dont_write_bytecode = True
    from utils.train_and_eval import binary_segmentation_loss

    torch.set_num_threads(8)
    for name, s, b, tag in [("dualdense_unet", 64, 2, "model_dualdense_unet"),
                            ("unet_plain", (72, 88), 2, "odd_unet_plain"),
                            ("attention_unet", (72, 88), 2, "odd_attention_unet"),
                            ("dualdense_unet", (72, 88), 1, "odd_dualdense_unet")]:
        torch.manual_seed(0)
        m = ref_model(name, num_classes=2)
        spec = load_hash(m)
        hh, ww = (s, s) if isinstance(s, int) else s
        x, y = synth(b, max(hh, ww), seed=2000 + hh)
        x, y = x[:, :, :hh, :ww].contiguous(), y[:, :hh, :ww].contiguous()
        m.train()
        out = m(x)
        loss = binary_segmentation_loss(out, y, "lovasz_hinge")
        loss.backward()
        rec = {"x": x.numpy(), "y": y.numpy(), "out": out.detach().numpy(), "loss": np.array([loss.item()]),
               "grad_names": np.array([k for k, _ in m.named_parameters()]),
               "grad_norms": np.array([float(p.grad.double().norm()) for _, p in m.named_parameters()])}
        m.eval()
        with torch.no_grad():
            rec["eval_out"] = m(x).numpy()
        np.savez_compressed(os.path.join(OUT, f"{tag}.npz"), **rec)
        print("wrote", tag, loss.item())


if __name__ == "__main__":
    which = sys.argv[1:] or ["main"]
    for w in which:
        {"main": main, "init": gen_init, "loop": gen_loop, "multiclass": gen_multiclass, "ignore": gen_ignore,
         "models2": gen_models2}[w]()
