"""GPU: unet_resnet50 at the benchmark's full size (512x512), bf16 fast kernels, against the oracle
run in torch on the GPU.

Round 1 held the bf16 model path to "1.5x the reference's own CPU-bf16 error" at B=2, 64x64, where
the problem is ill-conditioned (BN batch statistics of 2x4x4 pixels at layer4) and that bound is
~1 logit.  These tests use well-conditioned full-size problems instead:

* eval mode (running statistics calibrated to the data, so no batch-statistic feedback), B=2;
* train mode at the benchmark batch, B=16 (BN statistics over >= 16x16x16 pixels per channel).

Three oracle runs on identical inputs and hash-filled weights (oracle/weights.py), all in torch on
the GPU with MIOpen disabled (torch's own im2col + rocBLAS GEMM convolutions; TF32 off):
  * ``f32``: the reference's fp32 semantics (oracle/ref_cpu.py, model/unet_resnet.py:80-104);
  * ``amp``: the same under torch.autocast(bf16) -- the reference's own AMP regime;
  * ``emu``: fp32 arithmetic with bf16 rounding exactly where the HIP path stores a tensor
    (ref_cpu.Ctx.bf16_storage).  HIP and ``emu`` differ only in accumulation order and the
    rounding flips it causes, so this is the strict check of the fast kernels at full size.
Measured (first run): bf16 storage alone moves the logits by ~2 % of their
range (amp vs f32: max 1.1-1.5, mean 0.13-0.14 on |logit| <= 5.4-6.7), and HIP vs emu is 0.2-0.36 of
that -- accumulation-order rounding flips (~1e-3 of the elements per layer, one ulp each) amplified
through ~70 layers, not a kernel error (a wrong tap, channel or concat slot is O(1) per element).
Bounds:
  * HIP vs emu: max and mean |d logit| <= EMU_FRAC x (amp vs f32);
  * HIP vs f32 no worse than AMP_FACTOR x the amp run's own error (max and mean |d logit|);
  * argmax decisions (the metric) agree wherever the fp32 margin exceeds twice HIP's logit error;
  * train: loss within 2x amp's deviation + 1e-3 relative; per-parameter gradient relative L2 error
    (median over tensors) no worse than AMP_FACTOR x amp's, and individually (<= AMP_FACTOR x
    amp's + 1e-3) for every tensor amp moves by < 5 % (measured: the decoder and heads, 0.7-10 %
    for both HIP and amp).  The encoder's gradients are ill-conditioned at this init: bf16
    rounding of the FORWARD activations alone (emu, fp32 backward) moves them by ~100 %, so no
    absolute bound is meaningful there -- they are held to fp32 parity at 64x64
    (test_gpu_models.py) and per kernel in test_gpu_configs.py;
  * BN running statistics after the step within 2 % of emu's.
"""
import contextlib
import io

import pytest
import torch

pytestmark = pytest.mark.gpu

DEV = "cuda"
EMU_FRAC = 0.45
AMP_FACTOR = 1.5
#: fp32 step at the benchmark size: every gradient tensor (encoder included) within this relative L2 of
#: the oracle's fp32 run, or 4x that run's own distance from float64 where that is larger
FP32_GRAD_REL = 2e-3


@pytest.fixture(scope="module", autouse=True)
def _need_gpu():
    if not torch.cuda.is_available():
        pytest.skip("no GPU")
    from unetseg_hip import load
    load()


@contextlib.contextmanager
def _torch_exact():
    """torch's native GPU convolutions (no MIOpen), no TF32"""
    prev = (torch.backends.cudnn.enabled, torch.backends.cudnn.allow_tf32, torch.backends.cuda.matmul.allow_tf32)
    torch.backends.cudnn.enabled = False
    torch.backends.cudnn.allow_tf32 = False
    torch.backends.cuda.matmul.allow_tf32 = False
    try:
        yield
    finally:
        (torch.backends.cudnn.enabled, torch.backends.cudnn.allow_tf32, torch.backends.cuda.matmul.allow_tf32) = prev


def _state(name="unet_resnet50"):
    from oracle import ref_cpu
    from oracle.weights import make_torch_state
    return make_torch_state(ref_cpu.model_spec(name, num_classes=2))


def _oracle(state):
    from oracle import ref_cpu
    params, buffers = ref_cpu.split_state(state)
    return ({k: v.to(DEV).detach().requires_grad_(True) for k, v in params.items()},
            {k: v.to(DEV) for k, v in buffers.items()})


def _calibrate(state, x):
    """running statistics := the batch statistics of x (one fp32 train-mode oracle pass with
    momentum 1), so that eval mode is well conditioned"""
    from oracle import ref_cpu
    params, buffers = _oracle(state)
    old = ref_cpu.BN_MOMENTUM
    ref_cpu.BN_MOMENTUM = 1.0
    try:
        with torch.no_grad(), _torch_exact():
            ref_cpu.forward("unet_resnet50", params, buffers, x, train=True)
    finally:
        ref_cpu.BN_MOMENTUM = old
    out = dict(state)
    for k, v in buffers.items():
        out[k] = v.cpu()
    return out


def _hip_model(state, train):
    from model.model_factory import build_model
    with contextlib.redirect_stdout(io.StringIO()):
        m = build_model("unet_resnet50", num_classes=2)
    m.load_state_dict(state)
    m = m.to(DEV).train(train)
    m.compute_dtype = "bf16"
    return m


def _err(a, b):
    d = (a.double() - b.double()).abs()
    return d.max().item(), d.mean().item()


def test_eval_forward_512_bf16():
    """eval-mode forward, 2 x 512^2, running statistics calibrated on a different batch"""
    from oracle import ref_cpu
    from utils.synthetic import make_batch
    xc, _ = make_batch(2, 512, seed=21)
    x, _ = make_batch(2, 512, seed=22)
    state = _calibrate(_state(), xc.to(DEV))
    m = _hip_model(state, train=False)
    with torch.no_grad():
        hip = m(x.to(DEV)).float()
    torch.cuda.synchronize()
    params, buffers = _oracle(state)
    xd = x.to(DEV)
    with torch.no_grad(), _torch_exact():
        f32 = ref_cpu.forward("unet_resnet50", params, buffers, xd, train=False)
        emu = ref_cpu.forward("unet_resnet50", params, buffers, xd, train=False, bf16_storage=True)
        with torch.autocast("cuda", dtype=torch.bfloat16):
            amp = ref_cpu.forward("unet_resnet50", params, buffers, xd, train=False).float()
    scale = f32.abs().max().item()
    e_emu, e_f32, e_amp = _err(hip, emu), _err(hip, f32), _err(amp, f32)
    print(f"\neval 512 B=2: max|logit| {scale:.3f}  hip-emu max/mean {e_emu[0]:.3e}/{e_emu[1]:.3e}  "
          f"hip-f32 {e_f32[0]:.3e}/{e_f32[1]:.3e}  amp-f32 {e_amp[0]:.3e}/{e_amp[1]:.3e}")
    assert e_emu[0] <= EMU_FRAC * e_amp[0] and e_emu[1] <= EMU_FRAC * e_amp[1], (e_emu, e_amp)
    assert e_f32[0] <= AMP_FACTOR * e_amp[0] and e_f32[1] <= AMP_FACTOR * e_amp[1], (e_f32, e_amp)
    # the metric: argmax (tie -> 0) decisions agree except where the fp32 margin is below the
    # HIP path's own logit error
    margin = (f32[:, 1] - f32[:, 0]).abs()
    flip = (hip.argmax(1) != f32.argmax(1)) & (margin > 2 * e_f32[0])
    assert int(flip.sum()) == 0


@pytest.mark.parametrize("loss_name", ["lovasz_hinge", "bce"])
def test_train_step_512_b16_bf16(loss_name):
    """train-mode fwd + loss + bwd at the benchmark configuration (B=16, 512^2): logits, loss,
    every parameter gradient and the BN running statistics, with the benchmark's Lovasz hinge and with
    BCE.  BCE is smooth (no sort-order discontinuity), yet the encoder's gradients move as much under
    bf16 storage as with Lovasz (measured: amp-vs-f32 median 1.06 for both): the ill-conditioning is
    the BN-ResNet backward at this init, not the loss; every tensor is held at full size in fp32 by
    test_train_step_512_b16_fp32_every_tensor."""
    from oracle import ref_cpu
    from unetseg_hip.losses import binary_segmentation_loss
    from utils.synthetic import make_batch
    x, y = make_batch(16, 512, seed=31)
    state = _state()
    m = _hip_model(state, train=True)
    for p in m.parameters():
        p.grad = None
    out = m(x.to(DEV))
    loss = binary_segmentation_loss(out, y.to(DEV), loss_name)
    loss.backward()
    torch.cuda.synchronize()
    hip_out = out.detach().float()
    hip_grads = {k: p.grad.detach().clone() for k, p in m.named_parameters()}
    hip_bufs = {k: b.detach().clone() for k, b in m.named_buffers()}
    runs = {}
    xd, yd = x.to(DEV), y.to(DEV)
    for tag, kw in (("f32", {}), ("amp", dict(autocast_bf16=True)), ("emu", dict(bf16_storage=True))):
        params, buffers = _oracle(state)
        with _torch_exact():
            l_, o_, g_ = ref_cpu.train_step("unet_resnet50", params, buffers, xd, yd, loss_name, **kw)
        runs[tag] = (l_.item(), o_.float(), g_, buffers)
        torch.cuda.empty_cache()
    f32 = runs["f32"]
    scale = f32[1].abs().max().item()
    e_emu, e_f32, e_amp = _err(hip_out, runs["emu"][1]), _err(hip_out, f32[1]), _err(runs["amp"][1], f32[1])

    def grad_rel(g):
        r = []
        for k, v in f32[2].items():
            n = v.double().norm().item()
            if n > 0:
                r.append((g[k].double() - v.double()).norm().item() / n)
        r.sort()
        return r[len(r) // 2], r[-1]

    gh, ga, ge = grad_rel(hip_grads), grad_rel(runs["amp"][2]), None
    ge = []
    for k, v in runs["emu"][2].items():
        n = v.double().norm().item()
        if n > 0:
            ge.append((hip_grads[k].double() - v.double()).norm().item() / n)
    ge.sort()
    print(f"\ntrain 512 B=16: max|logit| {scale:.3f}  hip-emu {e_emu[0]:.3e}/{e_emu[1]:.3e}  "
          f"hip-f32 {e_f32[0]:.3e}/{e_f32[1]:.3e}  amp-f32 {e_amp[0]:.3e}/{e_amp[1]:.3e}")
    print(f"loss hip {loss.item():.6f} f32 {f32[0]:.6f} amp {runs['amp'][0]:.6f} emu {runs['emu'][0]:.6f}")
    print(f"grad rel L2 (median/max): hip-f32 {gh[0]:.3e}/{gh[1]:.3e} amp-f32 {ga[0]:.3e}/{ga[1]:.3e} "
          f"hip-emu {ge[len(ge) // 2]:.3e}/{ge[-1]:.3e}")
    for k in ("final.weight", "final.bias", "up_conv.3.weight", "up_conv.1.weight", "up_concat1.conv2.weight",
              "up_concat4.conv1.weight", "resnet.layer4.2.conv3.weight", "resnet.layer1.0.conv1.weight",
              "resnet.conv1.weight", "resnet.bn1.weight"):
        v = f32[2][k].double()
        n = v.norm().item()
        print(f"  {k:32s} |g| {n:.3e} hip {(hip_grads[k].double() - v).norm().item() / n:.3e} "
              f"amp {(runs['amp'][2][k].double() - v).norm().item() / n:.3e} "
              f"emu {(runs['emu'][2][k].double() - v).norm().item() / n:.3e}")
    assert e_emu[0] <= EMU_FRAC * e_amp[0] and e_emu[1] <= EMU_FRAC * e_amp[1], (e_emu, e_amp)
    assert e_f32[0] <= AMP_FACTOR * e_amp[0] and e_f32[1] <= AMP_FACTOR * e_amp[1], (e_f32, e_amp)
    assert abs(loss.item() - f32[0]) <= 2 * abs(runs["amp"][0] - f32[0]) + 1e-3 * abs(f32[0])
    assert gh[0] <= AMP_FACTOR * ga[0], (gh, ga)
    # well-conditioned tensors (bf16 storage moves them by < 5 %: the decoder and heads) are
    # held individually
    well = 0
    for k, v in f32[2].items():
        v = v.double()
        n = v.norm().item()
        if n == 0:
            continue
        ra = (runs["amp"][2][k].double() - v).norm().item() / n
        if ra < 0.05:
            well += 1
            rh = (hip_grads[k].double() - v).norm().item() / n
            assert rh <= AMP_FACTOR * ra + 1e-3, (k, rh, ra)
    print(f"well-conditioned gradient tensors checked individually: {well}")
    assert well >= 10
    worst = sorted(((hip_grads[k].double() - v.double()).norm().item() / max(v.double().norm().item(), 1e-30), k)
                   for k, v in runs["emu"][2].items() if v.double().norm().item() > 0)
    print("hip-emu per tensor, worst 4: " + ", ".join(f"{k} {r:.3e}" for r, k in worst[-4:]))
    # BN running statistics after the step (bn_finalize over 16 x H x W pixels per channel)
    for k, v in runs["emu"][3].items():
        if k.endswith(("running_mean", "running_var")):
            hb = hip_bufs[k].double()
            assert (hb - v.double()).abs().max().item() <= 2e-2 * v.double().abs().max().item() + 1e-4, k
        elif k.endswith("num_batches_tracked"):
            assert int(hip_bufs[k]) == int(v)


def test_train_step_512_b16_fp32_every_tensor():
    """The HIP path in fp32 (compute_dtype="fp32": the same op graph, fused BN / ReLU backward
    epilogues, side-stream weight gradients, fused Lovasz) at the benchmark size, B=16, 512^2, against
    the oracle's fp32 and float64 runs in torch on the GPU: EVERY gradient tensor, the encoder's
    included, within FP32_GRAD_REL relative L2 of the fp32 oracle (or 4x the fp32 oracle's own
    distance from float64, where the problem's conditioning makes that larger); logits within 1e-3
    (north_star); loss 1e-5 relative; running statistics 1e-4.  The bf16 product kernels of every
    configuration this step runs are held per launch in tests/test_gpu_configs.py."""
    from oracle import ref_cpu
    from unetseg_hip.losses import binary_segmentation_loss
    from utils.synthetic import make_batch
    x, y = make_batch(16, 512, seed=37)
    xd, yd = x.to(DEV), y.to(DEV)
    state = _state()
    m = _hip_model(state, train=True)
    m.compute_dtype = "fp32"
    for p in m.parameters():
        p.grad = None
    out = m(xd)
    loss = binary_segmentation_loss(out, yd, "lovasz_hinge")
    loss.backward()
    torch.cuda.synchronize()
    hip_out = out.detach().float()
    hip_grads = {k: p.grad.detach().clone() for k, p in m.named_parameters()}
    hip_bufs = {k: b.detach().clone() for k, b in m.named_buffers()}
    hip_loss = loss.item()
    del m, out, loss
    torch.cuda.empty_cache()
    runs = {}
    for tag, dt in (("f32", torch.float32), ("f64", torch.float64)):
        params, buffers = _oracle(state)
        params = {k: v.detach().to(dt).requires_grad_(True) for k, v in params.items()}
        buffers = {k: (v.to(dt) if v.is_floating_point() else v) for k, v in buffers.items()}
        with _torch_exact():
            l_, o_, g_ = ref_cpu.train_step("unet_resnet50", params, buffers, xd.to(dt), yd, "lovasz_hinge")
        runs[tag] = (l_.item(), o_, g_, buffers)
        del params
        torch.cuda.empty_cache()
    f32, f64 = runs["f32"], runs["f64"]
    e_out = (hip_out.double() - f32[1].double()).abs().max().item()
    rows = []
    for k, v in f32[2].items():
        n = v.double().norm().item()
        if n == 0:
            continue
        r_hip = (hip_grads[k].double() - v.double()).norm().item() / n
        n64 = f64[2][k].norm().item()
        r_ref = (v.double() - f64[2][k]).norm().item() / max(n64, 1e-300)
        rows.append((r_hip, r_ref, k))
    rows.sort()
    print(f"\nfp32 512 B=16: max|logit| {f32[1].abs().max().item():.3f} hip-f32 max|d| {e_out:.3e} "
          f"loss hip {hip_loss:.7f} f32 {f32[0]:.7f} f64 {f64[0]:.7f}")
    print(f"grad rel L2 hip-f32: median {rows[len(rows) // 2][0]:.3e} max {rows[-1][0]:.3e} ({rows[-1][2]}); "
          f"f32-f64 max {max(r[1] for r in rows):.3e}")
    assert e_out < 1e-3, e_out
    assert abs(hip_loss - f32[0]) <= 1e-5 * abs(f32[0]) + 1e-6
    bad = [(k, rh, rr) for rh, rr, k in rows if rh > max(FP32_GRAD_REL, 4 * rr)]
    assert not bad, bad[:8]
    for k, v in f32[3].items():
        if k.endswith(("running_mean", "running_var")):
            hb, vb = hip_bufs[k].double(), v.double()
            assert (hb - vb).abs().max().item() <= 1e-4 * vb.abs().max().item() + 1e-6, k
