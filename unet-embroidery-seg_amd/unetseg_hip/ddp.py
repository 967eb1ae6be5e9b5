"""Data-parallel training over RCCL (torch.distributed "nccl" backend == RCCL on ROCm).

The reference is single-process (train.py:98); this is the build's DP path:
  * parameters (one flat fp32 arena) and BN buffers are broadcast from rank 0 at wrap time;
  * gradient buckets are contiguous slices of the flat gradient arena.  The arena is laid out in
    reverse forward order, so the tape's backward completes buckets front to back; the op layer
    reports each finished parameter (``param_done``) and a bucket's all-reduce (AVG) is issued the
    moment its last parameter is final, overlapping the rest of backward (RCCL runs on its own
    stream, fenced against the compute stream by torch.distributed);
  * BatchNorm uses per-GPU batch statistics and rank-local running stats (DDP without SyncBN);
  * on a GPU each bucket's collective runs on a dedicated COMM stream (``comm_stream``) that first
    waits for the compute stream (BN / bias gradients) and for the bucket's OWN last weight-gradient
    launch (an event recorded on the weight-gradient stream right after the last of the bucket's conv
    weight gradients, ``param_done(..., stream=side)``; not that stream's tail when the bucket
    completes, which may hold later buckets' gradients) -- so it follows every writer -- and the
    bucket's optimizer actions run on that comm
    stream right behind the collective.  The weight-gradient stream never waits on RCCL: the next
    buckets' weight gradients keep running while a bucket is on the wire (three streams: compute,
    weight gradients, comm; the compute stream joins the comm stream once, at the end of backward);
  * ``reduce_dtype=torch.bfloat16`` (opt-in; bench.py --ddp-bf16, UNETSEG_DDP_BF16=1) sends a bf16
    copy of each bucket (87.9 MB instead of 175.7 MB per step for unet_resnet50): the average is then
    rounded to bf16 (relative error <= 2^-9 per element plus the bf16 sums of the ring), and the fp32
    master gradient takes the rounded average.

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
from .plan import py


def _nullctx():
    return contextlib.nullcontext()


_COMM = {}


def comm_stream(device):
    """the per-device stream the bucket collectives (and the optimizer work behind them) run on"""
    key = (device.type, device.index)
    if key not in _COMM:
        _COMM[key] = torch.cuda.Stream(device)
    return _COMM[key]


class GradBuckets:
    def __init__(self, model, bucket_mb: float = 25.0, group=None, allreduce: bool = True, reduce_dtype=None):
        import os

        self.model = model
        self.group = group
        self.allreduce = allreduce
        if reduce_dtype is None and os.environ.get("UNETSEG_DDP_BF16", "0") == "1":
            reduce_dtype = torch.bfloat16
        if reduce_dtype not in (None, torch.float32, torch.bfloat16):
            raise ValueError(f"GradBuckets: reduce_dtype must be float32 or bfloat16, got {reduce_dtype}")
        self.reduce_dtype = None if reduce_dtype == torch.float32 else reduce_dtype
        self._bufs = {}  # bucket -> persistent bf16 send buffer
        self._comm_used = None  # device whose comm stream ran collectives in this backward
        prev = getattr(model, "_buckets", None)  # e.g. FusedAdam(overlap=True) made before DDP
        self.actions = prev.actions if prev is not None else []  # fn(bucket, start, end, stream)
        self.finish_actions = prev.finish_actions if prev is not None else []  # fn() after the last bucket
        flat = model._flat
        esz = flat.element_size()
        cap = max(1, int(bucket_mb * 1024 * 1024 / esz))
        # params in arena order
        order = sorted(model._param_list, key=lambda p: model._slices[id(p)][0])
        self.buckets = []  # [start, end, remaining]
        self._side_ev = []  # per bucket: event after its last weight-gradient launch (reused every step)
        self._side_rec = []  # per bucket: that event was recorded in this backward
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
        self._side_ev = [None] * len(self.buckets)
        self._side_rec = [False] * len(self.buckets)  # the bucket has a writer on the side stream (static)
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

    def _reduce(self, i, view):
        """AVG all-reduce of one bucket on the current stream (fp32, or through a bf16 copy)"""
        if self.reduce_dtype is None:
            return dist.all_reduce(view, op=dist.ReduceOp.AVG, group=self.group, async_op=True), None
        buf = self._bufs.get(i)
        if buf is None or buf.device != view.device:
            buf = self._bufs[i] = torch.empty(view.numel(), dtype=self.reduce_dtype, device=view.device)
        buf.copy_(view)
        return dist.all_reduce(buf, op=dist.ReduceOp.AVG, group=self.group, async_op=True), buf

    def _issue(self, i):
        s, e, _ = self.buckets[i]
        view = self.model._flat_grad[s:e]
        side = ops.side_stream(view.device) if (ops.OVERLAP and view.is_cuda) else None
        if self.allreduce and view.is_cuda:
            # the collective and this bucket's optimizer update on the comm stream, ordered after every
            # writer of the bucket: BN / bias gradients (compute stream), weight gradients (side stream)
            comm = comm_stream(view.device)
            comm.wait_stream(torch.cuda.current_stream(view.device))
            if self._side_rec[i]:
                # the bucket's last weight-gradient launch (every side-stream writer reports its stream:
                # a bucket without one has no writer there)
                comm.wait_event(self._side_ev[i])
            with torch.cuda.stream(comm):
                w, buf = self._reduce(i, view)
                w.wait()  # RCCL: the comm stream waits for the collective; gloo: the host waits
                if buf is not None:
                    view.copy_(buf)
                for act in self.actions:
                    act(i, s, e, comm)
            self._comm_used = view.device
        else:
            if side is not None:
                # weight gradients are written on the side stream, BN/bias gradients on the compute
                # stream: the update is ordered after both
                side.wait_stream(torch.cuda.current_stream(view.device))
            with torch.cuda.stream(side) if side is not None else _nullctx():
                if self.allreduce:
                    w, buf = self._reduce(i, view)
                    if self.actions or buf is not None:
                        w.wait()
                        if buf is not None:
                            view.copy_(buf)
                    else:
                        self._pending.append(w)
                for act in self.actions:
                    act(i, s, e, side)
        self._issued[i] = True

    def _on_grad(self, p, stream=None):
        """p's gradient is final; stream: the weight-gradient stream when its last launch wrote it"""
        if self._left is None:
            self._reset()
        i = self.owner.get(id(p))
        if i is None:  # a stand-in tensor (e.g. a re-laid-out weight), not a model parameter
            return
        if stream is not None and self.allreduce:
            ev = self._side_ev[i]
            if ev is None:
                ev = self._side_ev[i] = torch.cuda.Event()
            py(ev.record, stream)  # re-recorded by later side-written params of the bucket (stream order)
            self._side_rec[i] = True
        self._left[i] -= 1
        if self._left[i] == 0 and not self._issued[i]:
            py(self._issue, i)  # a step plan replays the issue (the update reads Adam's step count then)

    def _finish(self):
        if self._issued is None:  # (not `_left`: a replayed step issues buckets without _on_grad)
            self._reset()
        for i in range(len(self.buckets)):
            if not self._issued[i]:
                self._issue(i)
        for w in self._pending:
            w.wait()
        if self._comm_used is not None:
            # the compute stream (hence the optimizer step and the next forward) follows the last
            # bucket's collective and update
            torch.cuda.current_stream(self._comm_used).wait_stream(comm_stream(self._comm_used))
            self._comm_used = None
        for act in self.finish_actions:
            act()
        self._left = None
        self._pending = []
        self._issued = [False] * len(self.buckets)  # (a replayed step issues without _on_grad's reset)


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
