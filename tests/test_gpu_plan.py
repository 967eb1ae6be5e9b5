"""GPU: a replayed step plan (unetseg_hip/plan.py) is the eager training step, bit for bit.

Two identical models (create_model init under one seed, bf16, FusedAdam(overlap=True): per-bucket
Adam + weight re-pack on the side stream, as bench.py runs them) train on the same two batches in
turn.  Model A runs every step eagerly; model B runs one eager step, records the next (the recording
is itself a real eager step) and replays the rest.  After every step the flat parameters, gradients,
Adam moments, BN running statistics and the loss must be identical -- the plan issues exactly the
eager step's launches, in the same order, on the same streams, with the per-step values (Adam's step
count, the dropout seed, the input batch) re-evaluated.  Reference: the training loops
utils/train_and_eval.py:185-263 and train.py:225-264 whose steps the plan replays.
"""
import contextlib
import io

import pytest
import torch

pytestmark = pytest.mark.gpu
DEV = "cuda"


@pytest.fixture(scope="module", autouse=True)
def _need_gpu():
    if not torch.cuda.is_available():
        pytest.skip("no GPU")
    from unetseg_hip import load
    load()


def _setup(name, batch, size, loss_name, seed=11, overlap=True):
    from model.model_factory import create_model
    from unetseg_hip.arena import FusedAdam
    from unetseg_hip.losses import binary_segmentation_loss, multitask_loss

    torch.manual_seed(seed)
    kw = dict(num_classes=1) if name == "multitask_unet" else dict(num_classes=2)
    with contextlib.redirect_stdout(io.StringIO()):
        model = create_model(name, weights="", **kw).to(DEV).train()
    model.compute_dtype = "bf16"
    opt = FusedAdam(model, lr=1e-4, betas=(0.9, 0.999), weight_decay=1e-4, overlap=overlap, bucket_mb=8.0)
    multitask = name == "multitask_unet"

    def step(x, y, c):
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

    return model, opt, step


def _state(model, opt, loss):
    bufs = torch.cat([b.detach().double().reshape(-1) for b in model.buffers()])
    return (model._flat.clone(), model._flat_grad.clone(), opt._m.clone(), opt._v.clone(), bufs,
            loss.detach().clone(), opt._step)


@pytest.mark.timeout(300)
@pytest.mark.parametrize("name,batch,size,loss_name,overlap", [
    ("unet_resnet50", 2, 256, "lovasz_hinge", True),
    ("multitask_unet", 2, 256, "bce", True),
    ("attention_unet", 2, 128, "lovasz_hinge", True),
    # the whole-arena Adam on the compute stream (bench.py --overlap-adam 0): the step count and lr
    # must advance on every replay
    ("unet_resnet50", 2, 256, "lovasz_hinge", False),
    # the timed configurations at their bench sizes (BASELINE C2 / C4 / C5): the 512^2 conv
    # configurations, the plan's private pool with its stream-ordered reuse across three streams
    ("unet_resnet50", 16, 512, "lovasz_hinge", True),
    ("attention_unet", 8, 512, "lovasz_hinge", True),
    ("multitask_unet", 8, 512, "bce", True),
])
def test_plan_replay_bit_identical(name, batch, size, loss_name, overlap):
    from unetseg_hip.plan import StepPlan
    from utils.synthetic import make_batch

    stream = torch.cuda.Stream(DEV)
    prev = torch.cuda.current_stream(DEV)
    torch.cuda.set_stream(stream)
    try:
        data = []
        for i in range(2):
            x, y, c = make_batch(batch, size, seed=1234 + i, with_cls=True)
            data.append((x.to(DEV), y.to(DEV), c.to(DEV)))
        nsteps = 5
        ma, oa, sa = _setup(name, batch, size, loss_name, overlap=overlap)
        ref = []
        for i in range(nsteps):
            ref.append(_state(ma, oa, sa(*data[i % 2])))
        torch.cuda.synchronize()
        del ma, oa, sa
        torch.cuda.empty_cache()
        mb, ob, sb = _setup(name, batch, size, loss_name, overlap=overlap)
        got = [_state(mb, ob, sb(*data[0]))]
        # the recording runs on fresh copies of batch 1's tensors (replay rebases onto the real batches)
        rec_in = tuple(t.clone() for t in data[1])
        plan = StepPlan({"x": rec_in[0], "y": rec_in[1], "c": rec_in[2]})
        loss = plan.record(lambda: sb(*rec_in))
        got.append(_state(mb, ob, loss))
        for i in range(2, nsteps):
            x, y, c = data[i % 2]
            loss = plan.replay(x=x, y=y, c=c)
            got.append(_state(mb, ob, loss))
        torch.cuda.synchronize()
        st = plan.stats()
        print(f"\n{name}: plan {st}")
        assert st["torch_ops"] <= 12, st
        names = ("params", "grads", "adam m", "adam v", "BN buffers", "loss", "step")
        for i, (a, b) in enumerate(zip(ref, got)):
            for n, u, v in zip(names, a, b):
                if isinstance(u, torch.Tensor):
                    assert torch.equal(u, v), f"step {i}: {n} differ (max {((u.double() - v.double()).abs().max().item()):.3e})"
                else:
                    assert u == v, f"step {i}: {n} {u} != {v}"
    finally:
        torch.cuda.set_stream(prev)
