"""Data-parallel training over RCCL (torch.distributed "nccl" backend == RCCL on ROCm).

The reference is single-process (train.py:98); this is the build's DP path:
  * parameters (one flat fp32 arena) and BN buffers are broadcast from rank 0 at wrap time;
  * gradient buckets are contiguous slices of the flat gradient arena.  The arena is laid out in
    reverse forward order, so the tape's backward completes buckets front to back; the op layer
    reports each finished parameter (``param_done``) and a bucket's all-reduce (AVG) is issued the
    moment its last parameter is final, overlapping the rest of backward (RCCL runs on its own
    stream, fenced against the compute stream by torch.distributed);
  * BatchNorm uses per-GPU batch statistics and rank-local running stats (DDP without SyncBN);
  * with the op layer's weight-gradient stream (ops.OVERLAP) a bucket's collective is enqueued on
    that stream after it has waited for the compute stream, so it follows every writer.

The same bucket tracking serves the optimizer overlap (``FusedAdam(overlap=True)``): per-bucket
actions (``actions``: Adam over the bucket's arena slice and the re-pack of its conv weights) run on
the weight-gradient stream right after the bucket's all-reduce (or, with ``allreduce=False`` on one
GPU, right after its last gradient), so the update of the decoder's parameters overlaps the encoder's
backward instead of running on the compute stream after it.  ``param_done`` is reported by the op
layer only after the last compute-stream kernel that reads a parameter (or its packed image) has been
enqueued, and the side stream waits for the compute stream before a bucket's work, so an update never
overtakes a read of the old value.
"""
from __future__ import annotations

import contextlib

import torch
import torch.distributed as dist

from . import ops


def _nullctx():
    return contextlib.nullcontext()


class GradBuckets:
    def __init__(self, model, bucket_mb: float = 25.0, group=None, allreduce: bool = True):
        self.model = model
        self.group = group
        self.allreduce = allreduce
        prev = getattr(model, "_buckets", None)  # e.g. FusedAdam(overlap=True) made before DDP
        self.actions = prev.actions if prev is not None else []  # fn(bucket, start, end, stream)
        self.finish_actions = prev.finish_actions if prev is not None else []  # fn() after the last bucket
        flat = model._flat
        esz = flat.element_size()
        cap = max(1, int(bucket_mb * 1024 * 1024 / esz))
        # params in arena order
        order = sorted(model._param_list, key=lambda p: model._slices[id(p)][0])
        self.buckets = []  # [start, end, remaining]
        self.owner = {}
        start, count = None, 0
        for p in order:
            off, n = model._slices[id(p)]
            if start is None:
                start = off
            self.owner[id(p)] = len(self.buckets)
            count += 1
            if off + n - start >= cap:
                self.buckets.append([start, off + n, count])
                start, count = None, 0
        if start is not None:
            self.buckets.append([start, flat.numel(), count])
        self._pending = []
        self._left = None
        self._issued = None
        model._grad_hook = self._on_grad
        model._after_backward = self._finish
        model._buckets = self
        if allreduce:
            self.broadcast_state()

    @torch.no_grad()
    def broadcast_state(self):
        dist.broadcast(self.model._flat, 0, group=self.group)
        self.sync_buffers()

    @torch.no_grad()
    def sync_buffers(self):
        """Re-broadcast rank 0's BN running statistics (one coalesced collective).  Between syncs
        they are rank-local (each rank's batch statistics; DDP without SyncBN).  torch DDP's default
        broadcast_buffers=True does this before every forward; here the train loop calls it before
        evaluation and checkpointing, where the running statistics are read."""
        bufs = [b for b in self.model.buffers()]
        if not bufs:
            return
        flat = torch.cat([b.detach().double().reshape(-1) for b in bufs])  # int64 counters survive fp64
        dist.broadcast(flat, 0, group=self.group)
        off = 0
        for b in bufs:
            n = b.numel()
            b.copy_(flat[off:off + n].view(b.shape).to(b.dtype))
            off += n

    def _reset(self):
        self._left = [b[2] for b in self.buckets]
        self._issued = [False] * len(self.buckets)
        self._pending = []

    def _issue(self, i):
        s, e, _ = self.buckets[i]
        view = self.model._flat_grad[s:e]
        side = ops.side_stream(view.device) if (ops.OVERLAP and view.is_cuda) else None
        if side is not None:
            # weight gradients are written on the side stream, BN/bias gradients on the compute
            # stream: the collective is ordered after both (side waits for compute, RCCL for side)
            side.wait_stream(torch.cuda.current_stream(view.device))
        with torch.cuda.stream(side) if side is not None else _nullctx():
            if self.allreduce:
                w = dist.all_reduce(view, op=dist.ReduceOp.AVG, group=self.group, async_op=True)
                if self.actions:
                    w.wait()  # RCCL: the current (side) stream waits; gloo: the host waits
                else:
                    self._pending.append(w)
            for act in self.actions:
                act(i, s, e, side)
        self._issued[i] = True

    def _on_grad(self, p):
        if self._left is None:
            self._reset()
        i = self.owner.get(id(p))
        if i is None:  # a stand-in tensor (e.g. a re-laid-out weight), not a model parameter
            return
        self._left[i] -= 1
        if self._left[i] == 0 and not self._issued[i]:
            self._issue(i)

    def _finish(self):
        if self._left is None:
            self._reset()
        for i in range(len(self.buckets)):
            if not self._issued[i]:
                self._issue(i)
        for w in self._pending:
            w.wait()
        for act in self.finish_actions:
            act()
        self._left = None
        self._pending = []


def init_from_env(backend: str = "nccl"):
    """One process per GPU (torchrun env); returns (rank, world, local_rank).

    UNETSEG_DIST_BACKEND overrides the backend (e.g. ``gloo`` to rehearse the N>1 control flow --
    buckets, the weight-gradient stream, the joins -- with several ranks sharing one GPU; the local
    rank then maps onto the visible devices modulo their count, see ``local_device``)."""
    import os

    backend = os.environ.get("UNETSEG_DIST_BACKEND", backend)
    world = int(os.environ.get("WORLD_SIZE", "1"))
    rank = int(os.environ.get("RANK", "0"))
    local = int(os.environ.get("LOCAL_RANK", "0"))
    if world > 1 and not dist.is_initialized():
        if backend == "nccl" or torch.cuda.device_count() > 0:
            torch.cuda.set_device(local_device(local))
        dist.init_process_group(backend=backend)
    return rank, world, local


def local_device(local: int) -> int:
    """device index of a local rank (identity with one rank per GPU)"""
    n = torch.cuda.device_count()
    return local % n if n > 0 else 0
