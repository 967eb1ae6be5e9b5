"""World-size-2 data-parallel tests on CPU (gloo): the N>1 path of bench.py / train.py without a GPU.

GradBuckets only needs the flat parameter/gradient arenas and the per-parameter "gradient final"
callback the op layer fires; here a stand-in module provides both, and the gradients come from the
CPU oracle on each rank's shard of the batch (the all-reduced gradient must equal the
mean of the per-shard gradients of the reference's algorithm).
"""
import os
import socket

import pytest
import torch
import torch.distributed as dist
import torch.multiprocessing as mp

from conftest import PKG, REPO  # noqa: F401


def _free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    port = s.getsockname()[1]
    s.close()
    return port


class ArenaModel(torch.nn.Module):
    """Parameters as views of one flat fp32 arena, laid out in reverse registration order (like HipModel)."""

    def __init__(self, shapes, seed):
        super().__init__()
        g = torch.Generator().manual_seed(seed)
        total = sum(int(torch.Size(s).numel()) for s in shapes.values())
        self._flat = torch.empty(total)
        self._flat_grad = torch.zeros(total)
        self._slices, self._param_list = {}, []
        off = total
        for name, s in shapes.items():
            n = int(torch.Size(s).numel())
            off -= n
            p = torch.nn.Parameter(self._flat[off:off + n].view(s))
            with torch.no_grad():
                p.copy_(torch.randn(s, generator=g))
            p.grad = self._flat_grad[off:off + n].view(s)
            self.register_parameter(name.replace(".", "_"), p)
            self._slices[id(p)] = (off, n)
            self._param_list.append(p)
        self.register_buffer("running_mean", torch.randn(7, generator=g))


def _worker(rank, world, port, shapes, out_q, reduce_dtype=None):
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port), RANK=str(rank), WORLD_SIZE=str(world))
    torch.set_num_threads(1)
    dist.init_process_group("gloo", rank=rank, world_size=world)
    try:
        from oracle import ref_cpu
        from oracle.weights import make_torch_state
        from unetseg_hip.ddp import GradBuckets
        from utils.synthetic import make_batch

        model = ArenaModel(shapes, seed=100 + rank)  # ranks start from different weights
        buckets = GradBuckets(model, bucket_mb=0.05, reduce_dtype=reduce_dtype)  # several buckets
        # after the broadcast every rank holds rank 0's parameters and buffers
        ref0 = ArenaModel(shapes, seed=100)
        assert torch.equal(model._flat, ref0._flat)
        assert torch.equal(model.running_mean, ref0.running_mean)

        # per-shard oracle gradients of unet_plain (disjoint images per rank, like bench.py's seeds)
        params, bufs = ref_cpu.split_state(make_torch_state(ref_cpu.model_spec("unet_plain", num_classes=2)))
        x, y = make_batch(1, 32, seed=1234 + 100000 * rank)
        _, _, grads = ref_cpu.train_step("unet_plain", params, bufs, x, y, "lovasz_hinge")
        local = {}
        for name, s in shapes.items():
            local[name] = grads[name].reshape(s).clone()
        # backward completes parameters in reverse registration order; the arena is laid out so
        # that buckets finish front to back and are reduced while "backward" continues
        for p, (name, s) in reversed(list(zip(model._param_list, shapes.items()))):
            p.grad.copy_(local[name])
            model._grad_hook(p)
        model._after_backward()
        out = {name: p.grad.numpy().copy() for p, name in zip(model._param_list, shapes)}
        local = {k: v.numpy() for k, v in local.items()}  # plain arrays: no fd sharing across processes
        out_q.put((rank, out, local, len(buckets.buckets)))
    finally:
        dist.destroy_process_group()


@pytest.mark.timeout(600)
@pytest.mark.parametrize("reduce_dtype", [None, torch.bfloat16], ids=["fp32", "bf16"])
def test_grad_buckets_average_matches_oracle_shards(reduce_dtype):
    """fp32 buckets: the average equals the mean of the per-shard oracle gradients to fp32 rounding;
    bf16 buckets (GradBuckets(reduce_dtype=torch.bfloat16), opt-in): to a few bf16 roundings of the
    per-rank magnitudes (<= 8 * 2^-9 * max_r |g_r| per element; gloo's bf16 AVG measured 3.6 * 2^-9),
    identical on both ranks"""
    from oracle import ref_cpu
    from oracle.weights import make_torch_state

    params, _ = ref_cpu.split_state(make_torch_state(ref_cpu.model_spec("unet_plain", num_classes=2)))
    names = list(params)[-12:]  # decoder tail + head: enough tensors for several buckets, small to move
    shapes = {n: tuple(params[n].shape) for n in names}
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_worker, args=(r, 2, port, shapes, q, reduce_dtype)) for r in range(2)]
    for p in procs:
        p.start()
    res = {}
    for _ in range(2):
        r, out, local, nb = q.get(timeout=540)
        res[r] = (out, local, nb)
    for p in procs:
        p.join(60)
        assert p.exitcode == 0
    assert res[0][2] > 1
    for n in names:
        want = 0.5 * (torch.from_numpy(res[0][1][n]) + torch.from_numpy(res[1][1][n]))
        got0, got1 = torch.from_numpy(res[0][0][n]), torch.from_numpy(res[1][0][n])
        if reduce_dtype is None:
            torch.testing.assert_close(got0, want, rtol=1e-6, atol=1e-7)
        else:
            scale = torch.maximum(torch.from_numpy(res[0][1][n]).abs(), torch.from_numpy(res[1][1][n]).abs())
            assert ((got0 - want).abs() <= 8 * 2.0 ** -9 * scale + 1e-30).all(), n
        torch.testing.assert_close(got1, got0, rtol=0, atol=0)


def _soft_worker(rank, world, port, out_q):
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port), RANK=str(rank), WORLD_SIZE=str(world))
    torch.set_num_threads(1)
    dist.init_process_group("gloo", rank=rank, world_size=world)
    try:
        from unetseg_hip import losses
        if rank == 1:  # only rank 1's loss saw a soft seg target
            losses._poison(torch.tensor(True), torch.zeros(3))
        raised = []
        for _ in range(2):  # the second epoch is clean on both ranks
            try:
                losses.raise_if_soft_targets("cpu")
                raised.append(False)
            except ValueError:
                raised.append(True)
        out_q.put((rank, raised))
    finally:
        dist.destroy_process_group()


@pytest.mark.timeout(300)
def test_soft_target_flag_raises_on_every_rank():
    """a soft label seen by one rank makes EVERY rank raise at the epoch check (the flag is
    all-reduced with MAX), instead of the clean ranks blocking in the next collective; the flag is
    cleared afterwards"""
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_soft_worker, args=(r, 2, port, q)) for r in range(2)]
    for p in procs:
        p.start()
    res = dict(q.get(timeout=240) for _ in range(2))
    for p in procs:
        p.join(60)
        assert p.exitcode == 0
    assert res == {0: [True, False], 1: [True, False]}, res
