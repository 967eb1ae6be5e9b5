"""GPU: the data-parallel path with the real HipModel, two ranks sharing one MI355X.

The 8-GPU node is the driver's; here two processes both use cuda:0 and the gloo backend moves the
gradient buckets (UNETSEG_DIST_BACKEND=gloo, as in bench.py's N>1 rehearsal).  Everything else is
the production path: HipModel's tape, ``ops.OVERLAP`` (weight gradients on the side HIP stream),
``param_done`` ordering, ``GradBuckets._issue`` enqueuing each bucket's AVG all-reduce (and, with
the overlapped optimizer, that bucket's Adam + re-pack) on the comm stream after it waits for the
compute and weight-gradient streams, and the fused Adam over the flat arena.

Cases: unet_resnet50 fp32 64x64 B=2 (small), and the BASELINE multi-GPU steps at their per-GPU
workload in bf16 -- unet_resnet50 512x512 B=16 (C3) and multitask_unet 512x512 B=8 (C5, whose cls
head reports its four parameters to the buckets after the decoder's).  Two ranks at ~25 GB each.

Checked: after one DP step the arena gradient on both ranks equals the mean of the two
ranks' local (single-process) gradients, and the parameters after Adam are bitwise identical across
ranks and equal to a single-process Adam update with that mean gradient.  Also: buffers are
broadcast from rank 0 at wrap time and ``sync_buffers`` re-broadcasts them (running
statistics drift per rank between syncs).
"""
import os
import socket

import pytest
import torch

pytestmark = pytest.mark.gpu


def _free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    port = s.getsockname()[1]
    s.close()
    return port


def _worker(rank, world, port, model_name, q, dtype="fp32", batch=2, size=64, overlap=False, reduce="fp32"):
    import contextlib
    import io
    import sys

    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port), RANK=str(rank), WORLD_SIZE=str(world),
                      LOCAL_RANK=str(rank), UNETSEG_DIST_BACKEND="gloo")
    try:
        import torch.distributed as dist

        from model.model_factory import build_model
        from oracle import ref_cpu
        from oracle.weights import make_torch_state
        from unetseg_hip import ops
        from unetseg_hip.arena import FusedAdam
        from unetseg_hip.ddp import GradBuckets, init_from_env
        from unetseg_hip.losses import binary_segmentation_loss, multitask_loss
        from utils.synthetic import make_batch

        assert ops.OVERLAP
        init_from_env("nccl")
        dev = torch.device("cuda", 0)
        torch.cuda.set_stream(torch.cuda.Stream(dev))
        with contextlib.redirect_stdout(io.StringIO()):
            kw = dict(num_classes=1) if model_name == "multitask_unet" else dict(num_classes=2)
        m = build_model(model_name, **kw)
        state = make_torch_state(ref_cpu.model_spec(model_name, **kw))
        if rank == 1:  # rank 1 starts from different weights and buffers: the wrap broadcasts rank 0's
            state = {k: (v + 0.25 if v.is_floating_point() else v) for k, v in state.items()}
        m.load_state_dict(state)
        m = m.to(dev).train()
        m.compute_dtype = dtype
        multitask = model_name == "multitask_unet"
        x, y, c = make_batch(batch, size, seed=1234 + 100000 * rank, with_cls=True)
        x, y, c = x.to(dev), y.to(dev), c.to(dev)
        if multitask:  # a fixed per-rank dropout keep-mask: the local and the DP pass draw the same
            m.dropout_mask = (torch.rand(batch, 512, generator=torch.Generator().manual_seed(77 + rank)) >= 0.5).float()

        def fwd_bwd():
            m._flat_grad.zero_()
            if multitask:  # seg BCE + 1.0 x CE (train.py:213-219 defaults), the bench's C5 step
                seg, cls = m(x)
                loss = multitask_loss(seg, cls, y, c, 1.0, "bce")[0]
            else:
                loss = binary_segmentation_loss(m(x), y, "lovasz_hinge")
            loss.backward()
            torch.cuda.synchronize()
            return loss.item()

        buffers0 = {k: b.clone() for k, b in m.named_buffers()}
        buckets = GradBuckets(m, bucket_mb=4.0, reduce_dtype=torch.bfloat16 if reduce == "bf16" else None)
        # after the wrap every rank holds rank 0's parameters and buffers
        flat0 = m._flat.detach().cpu().clone()
        dist.broadcast(flat0, 0)
        assert torch.equal(m._flat.cpu(), flat0)
        nb = len(buckets.buckets)
        # local gradient of this rank's shard: the same step without the bucket hooks
        hook, after = m._grad_hook, m._after_backward
        m._grad_hook = m._after_backward = None
        bufs = {k: b.clone() for k, b in m.named_buffers()}
        fwd_bwd()
        local = m._flat_grad.detach().clone()
        for k, b in m.named_buffers():  # undo the running-stat update of the local pass
            b.copy_(bufs[k])
        m._grad_hook, m._after_backward = hook, after
        # overlap: Adam + re-pack per bucket on the weight-gradient stream right after its all-reduce
        opt = FusedAdam(m, lr=1e-3, betas=(0.9, 0.999), weight_decay=1e-4, overlap=overlap)
        p_before = m._flat.detach().clone()
        # the DP step: buckets all-reduced (AVG) from inside backward on the weight-gradient stream
        fwd_bwd()
        avg = m._flat_grad.detach().clone()
        opt.step()
        assert opt._step == 1
        torch.cuda.synchronize()
        # single-process Adam with the averaged gradient, for comparison
        pm, gm_ = p_before.clone(), {}
        ref = {"p": pm}
        ref_cpu.adam_step(ref, {"p": avg}, {"p": torch.zeros_like(pm)}, {"p": torch.zeros_like(pm)}, 1, 1e-3)
        # running statistics diverge per rank (different shards); sync_buffers re-broadcasts rank 0's
        drift = any(not torch.equal(b, buffers0[k]) for k, b in m.named_buffers() if k.endswith("running_mean"))
        buckets.sync_buffers()
        rm = torch.cat([b.detach().float().reshape(-1) for k, b in m.named_buffers()]).cpu()
        rm0 = rm.clone()
        dist.broadcast(rm0, 0)
        names = [(n, *m._slices[id(p)]) for n, p in m.named_parameters()]
        q.put((rank, local.cpu().numpy(), avg.cpu().numpy(), m._flat.detach().cpu().numpy(), pm.cpu().numpy(), nb,
               bool(drift), bool(torch.equal(rm, rm0)), names))
        dist.destroy_process_group()
    except BaseException as e:  # report instead of hanging the parent
        import traceback
        q.put((rank, "ERROR " + "".join(traceback.format_exception(e))))
        sys.exit(1)


@pytest.mark.timeout(600)
@pytest.mark.parametrize("model_name,dtype,batch,size,overlap,reduce", [
    ("unet_resnet50", "fp32", 2, 64, False, "fp32"),
    ("unet_resnet50", "bf16", 16, 512, False, "fp32"),   # C3's per-GPU step: the bench dtype, batch and size
    ("multitask_unet", "bf16", 8, 512, False, "fp32"),   # C5's per-GPU step (seg BCE + CE, the cls head's buckets)
    ("unet_resnet50", "bf16", 4, 128, True, "fp32"),     # bench.py's step: Adam inside backward, per bucket
    ("multitask_unet", "bf16", 8, 512, True, "fp32"),
    ("unet_resnet50", "bf16", 16, 512, True, "bf16"),    # opt-in bf16 bucket reduce (bench.py --ddp-bf16)
])
def test_dp2_one_gpu_hip_model(model_name, dtype, batch, size, overlap, reduce):
    """the collectives and the per-bucket Adam run on the comm stream (ddp.comm_stream), the weight-
    gradient stream never waits for them; with reduce="bf16" the average is held to a few bf16
    roundings of the per-rank gradients (8 * 2^-9 * max |g_r|)"""
    if not torch.cuda.is_available():
        pytest.skip("no GPU")
    import numpy as np
    import torch.multiprocessing as mp
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_worker, args=(r, 2, port, model_name, q, dtype, batch, size, overlap, reduce))
             for r in range(2)]
    for p in procs:
        p.start()
    res = {}
    try:
        for _ in range(2):
            item = q.get(timeout=540)
            assert not isinstance(item[1], str), item[1]
            res[item[0]] = item[1:]
    finally:
        for p in procs:
            p.join(60)
            if p.is_alive():
                p.kill()
    for p in procs:
        assert p.exitcode == 0
    (l0, a0, f0, r0, nb, drift, bsync0, names), (l1, a1, f1, r1, _, _, bsync1, _) = res[0], res[1]
    assert nb > 1, "expected several gradient buckets"
    want = 0.5 * (l0.astype(np.float64) + l1.astype(np.float64))
    if reduce == "bf16":
        tol = 8 * 2.0 ** -9 * np.maximum(np.abs(l0), np.abs(l1)).astype(np.float64) + 1e-12
    else:
        tol = 1e-6 * np.abs(want) + 1e-9
    bad = [(n, off, int((np.abs(a0[off:off + k] - want[off:off + k]) > tol[off:off + k]).sum()), k)
           for n, off, k in names]
    bad = [b for b in bad if b[2]]
    assert not bad, f"{len(bad)} parameters differ from the mean of the local gradients: {bad[:12]}"
    if reduce != "bf16":
        np.testing.assert_allclose(a0, want, rtol=1e-6, atol=1e-9)
    assert np.array_equal(a0, a1)
    assert np.array_equal(f0, f1), "parameters out of sync after the DP step"
    np.testing.assert_allclose(f0, r0, rtol=1e-6, atol=1e-8)
    assert drift and bsync0 and bsync1
