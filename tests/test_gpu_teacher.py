"""GPU: every gradient of the benchmarked bf16 training step, held individually at full size.

One bench step (create_model init, bf16 kernels, a created HIP stream, weight gradients on the side
stream, concat weight gradients held back to layer4, FusedAdam(overlap=True): Adam + weight re-pack
per bucket during backward) of each GPU configuration -- C2 unet_resnet50 B=16 (Lovasz, and BCE),
C4 attention_unet B=8, C5 multitask_unet B=8, all 512x512 -- runs with tests/teacher_tap.Recorder
installed as ops.TAP.  Each block of the model (ResNet stem, each bottleneck, each decoder block,
the heads: ``ops.tap_mark`` in the model code) is then rebuilt in float64 from the tensors the HIP
path stored, and its backward is run from HIP's own incoming gradient (teacher forcing, see
teacher_tap.py), so no error is amplified across blocks.  Held per tensor:

* every parameter gradient (fp32): relative L2 <= PARAM_REL against the float64 rebuild with bf16
  rounding where the path stores a gradient (``emu``), or <= NOISE_K x the distance between that
  rebuild run in float32 and in float64 where fp32 accumulation is ill-conditioned; the analytically
  zero psi conv bias gradients absolutely, at <= ZERO_U x the L2 norm of their summands;
* every block input's gradient contribution (bf16-stored): relative L2 <= INPUT_REL;
* every op's forward output against float64 on the stored inputs: relative L2 <= FWD_REL (bf16
  rounding of the stored output is ~1.1e-3 rms);
* the loss gradient against the oracle's loss in float64 on HIP's logits: <= LOSS_REL;
* the overlapped Adam update against torch.optim.Adam's formula on the pre-step state.

Reference: model/resnet_backbone.py:80-115, model/unet_resnet.py:25-42,80-104,
model/unet_attention.py:30-89, model/unet_multitask.py:73-139, model/unet_training.py:219-280.
"""
import contextlib
import io
import json
import os
import time

import pytest
import torch

from teacher_tap import Recorder, check_segment, rel_l2

pytestmark = pytest.mark.gpu
DEV = "cuda"

PARAM_REL = 1e-3
#: ... or NOISE_K x the float32 rebuild's own distance from the float64 one, where fp32 accumulation
#: itself is ill-conditioned (per-channel sums with heavy cancellation: a BN bias whose incoming
#: gradient is nearly mean-free).  Round 4 measured every such tensor at <= 1.33x its noise floor
#: (C5 layer1.0.downsample.0.weight), so 3x leaves room for the draw of the noise and no more.
NOISE_K = 3.0
#: conv biases in front of a train-mode BN (the attention gates' psi conv, model/unet_attention.py:24-25):
#: the exact gradient is 0 (BN removes the mean), so a relative bound is vacuous (the float64 value is
#: ~1e-17).  Held absolutely: |hip - float64| <= ZERO_U x ||d loss / d psi||_2, the L2 norm of the
#: gradient's summands (the psi path is fp32: the BN backward's per-pixel terms carry fp32 cancellation
#: noise, summed over N/8 - N pixels).  Measured (round 5, C4): |hip - float64| / ||terms||_2 <= 2.8e-6
#: (~47 fp32 units); ZERO_U = 2^-12 leaves ~90x, while a 1 % error of the summands -- random signs:
#: 1e-2 x ||terms||_2, one sign: up to 1e-2 x ||terms||_1 (200-500x the L2 norm here) -- lands 40x to
#: 10^4x above it.  The L1 / L2 norms and the ratio are in the report (`zero_abs`).  (Round 4 and early
#: round 5 held it at <= 4x the float32 rebuild's absolute deviation: not a bound on anything the HIP
#: path does differently -- it failed after an fp64 reduction-order change in the BN finalize, with
#: that deviation exactly 0 in one block.)
ZERO_U = 2.0 ** -12
ZERO_GRAD = ("attn.psi.0.bias",)
INPUT_REL = 1e-2
FWD_REL = 5e-3
LOSS_REL = 1e-4
ADAM_REL = 1e-3

CONFIGS = {
    "c2_lovasz": ("unet_resnet50", 16, "lovasz_hinge", 22),
    "c2_bce": ("unet_resnet50", 16, "bce", 22),
    "c4_attention": ("attention_unet", 8, "lovasz_hinge", 10),
    "c5_multitask": ("multitask_unet", 8, "bce", 23),
}


@pytest.fixture(scope="module", autouse=True)
def _need_gpu():
    if not torch.cuda.is_available():
        pytest.skip("no GPU")
    from unetseg_hip import load
    load()


@contextlib.contextmanager
def _torch_exact():
    prev = (torch.backends.cudnn.enabled, torch.backends.cuda.matmul.allow_tf32)
    torch.backends.cudnn.enabled = False
    torch.backends.cuda.matmul.allow_tf32 = False
    try:
        yield
    finally:
        torch.backends.cudnn.enabled, torch.backends.cuda.matmul.allow_tf32 = prev


def _bench_step(name, batch, loss_name):
    """bench.py's model, optimizer and step; returns (model, opt, step fn, batches)"""
    from model.model_factory import create_model
    from unetseg_hip.arena import FusedAdam
    from unetseg_hip.losses import binary_segmentation_loss, multitask_loss
    from utils.synthetic import make_batch

    torch.manual_seed(11)
    kw = dict(num_classes=1) if name == "multitask_unet" else dict(num_classes=2)
    with contextlib.redirect_stdout(io.StringIO()):
        model = create_model(name, weights="", **kw).to(DEV).train()
    model.compute_dtype = "bf16"
    opt = FusedAdam(model, lr=1e-4, betas=(0.9, 0.999), weight_decay=1e-4, overlap=True, bucket_mb=8.0)
    batches = []
    for i in range(2):
        x, y, c = make_batch(batch, 512, seed=1234 + i, with_cls=True)
        batches.append((x.to(DEV), y.to(DEV), c.to(DEV)))
    multitask = name == "multitask_unet"

    def step(i):
        x, y, c = batches[i]
        opt.zero_grad()
        with torch.autocast("cuda", dtype=torch.bfloat16):
            if multitask:
                seg, cls = model(x)
                loss = multitask_loss(seg, cls, y, c, 1.0, loss_name)[0]
            else:
                loss = binary_segmentation_loss(model(x), y, loss_name)
        loss.backward()
        opt.step()
        return loss

    return model, opt, step, batches


def _adam_ref(w0, g, m0, v0, step, lr, b1=0.9, b2=0.999, eps=1e-8, wd=1e-4):
    """torch.optim.Adam (coupled weight decay, train.py:62-78) in float64"""
    w0, g, m0, v0 = (t.double() for t in (w0, g, m0, v0))
    g = g + wd * w0
    m = b1 * m0 + (1 - b1) * g
    v = b2 * v0 + (1 - b2) * g * g
    bc1, bc2 = 1 - b1 ** step, 1 - b2 ** step
    return w0 - (lr / bc1) * m / ((v.sqrt() / bc2 ** 0.5) + eps)


def _loss_check(name, loss_name, rec, batch):
    from oracle import ref_cpu
    _, y, c = batch
    outs = rec.outputs()
    # Lovasz in fp32 -- the kernel's key precision: the sort order (hence the per-pixel gradient) of
    # near-equal hinge errors follows the fp32 keys; BCE / CE in float64
    dt = torch.float32 if loss_name == "lovasz_hinge" else torch.float64
    leaves = [t.to(dt).requires_grad_(True) for _, t in outs]
    if name == "multitask_unet":
        total = ref_cpu.multitask_loss(leaves[1], leaves[0], y, c, 1.0, loss_name)[0]
        # outputs are recorded in op order: cls head (after the encoder) before the seg head
    else:
        total = ref_cpu.binary_segmentation_loss(leaves[0], y, loss_name)
    total.backward()
    return [rel_l2(rec.holder_grads[o], leaf.grad) for (o, _), leaf in zip(outs, leaves)]


def _run(tag):
    name, batch, loss_name, nseg = CONFIGS[tag]
    from unetseg_hip import ops

    t0 = time.time()
    stream = torch.cuda.Stream(DEV)
    prev_stream = torch.cuda.current_stream(DEV)
    torch.cuda.set_stream(stream)
    try:
        model, opt, step, batches = _bench_step(name, batch, loss_name)
        step(0)  # warm: the checked step's forward reads the weights the overlapped Adam re-packed
        torch.cuda.synchronize()
        w0, m0, v0 = model._flat.clone(), opt._m.clone(), opt._v.clone()
        rec = Recorder()
        ops.TAP = rec
        try:
            loss = step(1)
        finally:
            ops.TAP = None
        torch.cuda.synchronize()
    finally:
        torch.cuda.set_stream(prev_stream)
    t_step = time.time() - t0
    assert rec.done and len(rec.segments()) == nseg, [n for _, n in rec.segments()]
    names = {id(p): n for n, p in model.named_parameters()}

    def weights(p):
        off, n = model.flat_slice(p)
        return w0[off:off + n].view(p.shape)

    def hip_grad(p):
        return p.grad

    # the overlapped update: every parameter moved by Adam from the pre-step state and the final grads
    exp = _adam_ref(w0, model._flat_grad, m0, v0, opt._step, opt.param_groups[0]["lr"])
    adam_rel = rel_l2(model._flat.double() - w0.double(), exp - w0.double())
    with _torch_exact():
        loss_rel = _loss_check(name, loss_name, rec, batches[1])
    report = {"config": tag, "model": name, "batch": batch, "loss": loss_name, "hip_loss": float(loss.item()),
              "adam_update_rel": adam_rel, "loss_grad_rel": loss_rel, "segments": {}}
    bad = []
    t1 = time.time()
    refs = {}
    zabs = {}  # segment -> {ZERO_GRAD parameter: (|hip - float64|, (L1, L2) of its summands)}
    for mode, emu, dt in (("emu", True, torch.float64), ("emu32", True, torch.float32), ("f64", False, torch.float64)):
        for k, sname in rec.segments():
            with _torch_exact():
                r = check_segment(rec, k, weights, hip_grad, emu=emu, dt=dt)
            seg = report["segments"].setdefault(sname, {})
            if mode == "emu32":
                # accumulation-noise floor: the same rebuild in float32 against the float64 one
                for p, _, ref in r["params"]:
                    seg["emu"]["noise"][names[id(p)]] = rel_l2(ref, refs[id(p)])
                continue
            if emu:
                for p, _, ref in r["params"]:
                    if names[id(p)].endswith(ZERO_GRAD):
                        zabs.setdefault(sname, {})[names[id(p)]] = (
                            float((hip_grad(p).double() - ref.double()).norm()), r["bias_l1"].get(id(p)))
            pr = sorted(((rel, names[id(p)]) for p, rel, _ in r["params"]), reverse=True)
            ir = [rel for _, rel in r["inputs"]]
            fr = sorted(((rel, kind) for kind, rel in r["fwd"]), reverse=True)
            seg[mode] = {"param_max": pr[0][0] if pr else 0.0, "param_worst": pr[0][1] if pr else None,
                         "n_params": len(pr), "input_max": max(ir) if ir else 0.0, "n_inputs": len(ir),
                         "fwd_max": fr[0][0] if fr else 0.0, "params": {n: rel for rel, n in pr}, "noise": {}}
            if emu:
                for p, _, ref in r["params"]:
                    refs[id(p)] = ref
                bad += [(sname, "input", rel) for rel in ir if not rel <= INPUT_REL]
                bad += [(sname, f"fwd:{kind}", rel) for rel, kind in fr if not rel <= FWD_REL]
            del r
        torch.cuda.empty_cache()
    worst_ratio = (0.0, None)
    for sname, seg in report["segments"].items():
        e = seg["emu"]
        e["zero_abs"] = {}
        for n, rel in e["params"].items():
            if n.endswith(ZERO_GRAD):
                # analytically zero: the absolute error against the bf16 rounding of its summands
                err, norms = zabs[sname][n]
                l1, l2 = norms if norms else (None, None)
                e["zero_abs"][n] = {"abs_err": err, "summands_l1": l1, "summands_l2": l2,
                                    "allow": ZERO_U * l2 if l2 else None, "ratio": err / (ZERO_U * l2) if l2 else None}
                if l2 is None or not err <= ZERO_U * l2:
                    bad.append((sname, n, err, ZERO_U * l2 if l2 else None))
                continue
            else:
                allow = max(PARAM_REL, NOISE_K * e["noise"][n])
                if rel > PARAM_REL:
                    worst_ratio = max(worst_ratio, (rel / max(e["noise"][n], 1e-300), n))
            if not rel <= allow:
                bad.append((sname, n, rel, allow))
        e["allowance_max"] = max(max(PARAM_REL, NOISE_K * v) for k, v in e["noise"].items()
                                 if not k.endswith(ZERO_GRAD)) if e["noise"] else None
    report["worst_noise_ratio"] = {"ratio": worst_ratio[0], "param": worst_ratio[1], "noise_k": NOISE_K}
    t_check = time.time() - t1
    report["seconds"] = {"step": round(t_step, 1), "check": round(t_check, 1)}
    n_params = sum(s["emu"]["n_params"] for s in report["segments"].values())
    report["n_params_checked"] = n_params
    print(f"\n{tag}: {len(rec.segments())} blocks, {n_params} parameter tensors, step {t_step:.1f}s, "
          f"check {t_check:.1f}s; loss-grad rel {', '.join(f'{v:.2e}' for v in loss_rel)}; adam rel {adam_rel:.2e}")
    for sname, seg in report["segments"].items():
        line = "  ".join(f"{m}: param {v['param_max']:.2e} input {v['input_max']:.2e} fwd {v['fwd_max']:.2e}"
                         for m, v in seg.items() if m in ("emu", "f64"))
        print(f"  {sname:18s} {line}  (worst {seg['emu']['param_worst']})")
    out = os.environ.get("UNETSEG_TEACHER_OUT")
    if out:
        os.makedirs(out, exist_ok=True)
        with open(os.path.join(out, f"teacher_{tag}.json"), "w") as f:
            json.dump(report, f, indent=1)
    assert n_params == len(list(model.parameters())), "a parameter was not checked"
    assert all(v <= LOSS_REL for v in loss_rel), loss_rel
    assert adam_rel <= ADAM_REL, adam_rel
    assert not bad, bad[:12]


@pytest.mark.timeout(600)
@pytest.mark.parametrize("tag", list(CONFIGS))
def test_teacher_forced_step(tag):
    _run(tag)
