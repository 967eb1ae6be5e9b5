"""Step plans: one training step's launch sequence recorded once, then replayed from the host.

The op layer enqueues a step from Python: ~500 C-ABI launches, ~600 tensor allocations, the tape's
closures and the autograd engine -- 4-7 ms of host time per step against 10-19 ms of GPU time.  A
B=8 step (multitask_unet, 10 ms on the GPU) then sits close to host-bound, and on a slower or busier
host it becomes host-bound (BASELINE config C5 lost 14 % between two boxes with the same GPU rate).
A HIP graph removes the host cost but runs the weight-gradient stream's branches less concurrently
(round 3: 10.8 vs 10.2 ms per C5 step).  A StepPlan keeps the streams and removes the host work:

* ``record(fn)`` runs ``fn`` (one complete eager step: zero_grad, forward, loss, backward with the
  per-bucket Adam + weight re-pack on the side stream, optimizer step) once with
    - every C-ABI call logged with its arguments (``lib`` hands out logging wrappers),
    - a private memory pool for every allocation of the step (see Memory below) and a
      TorchDispatchMode that logs the few torch kernels of the step (the autograd seed, small fills)
      as replayable calls,
    - the host-side actions that carry per-step state logged as Python calls (``py``): the gradient
      buckets' optimizer updates (Adam's step count is read when they run), the optimizer's step
      commit, the DDP collectives;
  autograd runs single-threaded during the recording so the backward's torch ops are seen too.
* ``replay(inputs)`` re-issues the log in order on the same streams: pointer arguments that fall
  inside a registered input tensor are rebased onto the new batch, ``Dyn`` arguments (e.g. the
  dropout seed) are re-evaluated.  Every kernel of the step runs every replay; only the Python that
  decided which kernels to launch is skipped.

Memory: the recording allocates from a private pool (torch.cuda.MemPool) that the plan owns for its
life, so every recorded pointer stays valid and nothing outside the plan is ever placed there.
Inside the pool the caching allocator reuses freed buffers in stream order, as in the eager step
(deterministic, hence replayable; and a buffer rewritten while still in the 256 MB Infinity Cache
saves the write-back of its old contents); only buffers handed to another stream (record_stream) are
held for the plan's life, because their reuse would depend on GPU progress.  Correctness gate:
tests/test_gpu_plan.py (replayed steps bit-identical to eager steps, every parameter, moment and
BN statistic).
"""
from __future__ import annotations

import threading

import torch
from torch.utils._python_dispatch import TorchDispatchMode

from . import lib as _libmod

#: the plan being recorded (module-global: the backward runs on the recording thread, see record())
RECORDING = None

# C-ABI entry points that only answer host-side shape questions (no device work): not logged
_PURE = frozenset(n for n in _libmod.VALUE_FUNCS if n not in ("conv2d_fwd_mask", "conv2d_dgrad_post",
                                                                 "conv2d_dgrad_post_res")) | {
    "last_error", "device_arch", "abi_version"}


class Dyn(int):
    """an integer argument whose value changes every step: ``getter()`` gives the value of the next
    replay (the recording uses the int value itself)"""

    def __new__(cls, value, getter):
        o = int.__new__(cls, value)
        o.getter = getter
        return o


def py(fn, *args, **kwargs):
    """run fn now; when a plan is being recorded, log it to run again at this point of every replay
    (nothing fn does is logged by itself: its own launches happen when it runs)"""
    rec = RECORDING
    if rec is None or rec.suspended:
        return fn(*args, **kwargs)
    rec.calls.append(("py", fn, args, kwargs))
    rec.suspended += 1
    try:
        return fn(*args, **kwargs)
    finally:
        rec.suspended -= 1


def _wrap(name, fn):
    def logged(*args):
        rec = RECORDING
        if rec is not None and not rec.suspended and name not in _PURE:
            rec.log_c(name, fn, args)
        return fn(*args)
    return logged


# aten ops that launch nothing: allocation (kept alive) and metadata / views
_NO_KERNEL = {"aten::empty", "aten::empty_strided", "aten::empty_like", "aten::new_empty", "aten::new_empty_strided",
              "aten::detach", "aten::alias", "aten::lift_fresh", "aten::_to_copy_noop"}


# out-of-place factories whose result is one constant: name -> (args, kwargs) -> fill value
_FILL = {"aten::zeros": lambda a, k: 0, "aten::zeros_like": lambda a, k: 0, "aten::new_zeros": lambda a, k: 0,
         "aten::ones": lambda a, k: 1, "aten::ones_like": lambda a, k: 1, "aten::new_ones": lambda a, k: 1,
         "aten::full": lambda a, k: a[1] if len(a) > 1 else k["fill_value"],
         "aten::full_like": lambda a, k: a[1] if len(a) > 1 else k["fill_value"]}


def _fill_into(out, value):
    out.fill_(value)


class _Mode(TorchDispatchMode):
    def __init__(self, plan):
        super().__init__()
        self.plan = plan

    def __torch_dispatch__(self, func, types, args=(), kwargs=None):
        kwargs = kwargs or {}
        out = func(*args, **kwargs)
        plan = self.plan
        if threading.get_ident() != plan.thread:
            raise RuntimeError(f"StepPlan: {func} ran on another thread during the recording")
        name = func._schema.name
        if name == "aten::record_stream":
            # a buffer another stream reads: the allocator would reuse it only once that stream's event
            # has completed -- a decision that depends on GPU progress at recording time.  Held for the
            # plan's life instead, so it is never reused.
            plan.keep.append(args[0])
            return out
        if plan.suspended:
            return out
        if name in _NO_KERNEL or name.startswith("profiler::"):
            return out
        sch = func._schema
        is_view = (not sch.is_mutable) and any(r.alias_info is not None for r in sch.returns)
        if is_view:
            return out
        if name == "aten::_local_scalar_dense":
            raise RuntimeError("StepPlan: the step reads a device value on the host (.item()): not replayable")
        stream = torch.cuda.current_stream()
        for a in list(args) + list(kwargs.values()):
            if isinstance(a, torch.Tensor) and a.is_cuda and plan._is_input(a):
                raise RuntimeError(f"StepPlan: torch op {name} reads an input tensor (not rebased on replay)")
        if sch.is_mutable:
            plan.calls.append(("torch", func, args, kwargs, stream, None))
        elif name in _FILL and isinstance(out, torch.Tensor):
            # a constant-filled factory (e.g. a zeroed padded gradient buffer): replay fills the recorded
            # tensor in place -- recomputing it would allocate a fresh tensor and copy it over every replay
            plan.calls.append(("torch", _fill_into, (out, _FILL[name](args, kwargs)), {}, stream, None))
        elif isinstance(out, torch.Tensor):
            # out-of-place: replay computes a fresh result and copies it into the recorded one, which is
            # what later recorded launches read
            plan.calls.append(("torch", func, args, kwargs, stream, out))
        else:
            raise RuntimeError(f"StepPlan: cannot replay {name} (returns {type(out).__name__})")
        plan.n_torch += 1
        plan.torch_names.append(name)
        return out


class StepPlan:
    """A recorded training step (see the module docstring).  ``inputs``: name -> device tensor used by
    the recording; replay() takes tensors of the same shapes, dtypes and strides."""

    def __init__(self, inputs):
        self.inputs = dict(inputs)
        self.calls = []
        self.keep = []
        self.suspended = 0
        self.n_torch = 0
        self.torch_names = []
        self.result = None
        self.thread = None
        self.stream = None
        self._ranges = [(n, t.data_ptr(), t.data_ptr() + t.numel() * t.element_size()) for n, t in self.inputs.items()]
        self._patched = None

    # ---- recording --------------------------------------------------------------------------------
    def _is_input(self, t):
        p = t.data_ptr()
        return any(lo <= p < hi for _, lo, hi in self._ranges)

    def log_c(self, name, fn, args):
        self.calls.append(["c", fn, list(args), name])

    def record(self, fn):
        """run fn (one eager step) once, logging it; returns fn's result (kept: replays write into it)"""
        global RECORDING
        if RECORDING is not None:
            raise RuntimeError("StepPlan: nested recording")
        lib = _libmod.lib
        saved = dict(lib.__dict__)
        lib.__dict__.clear()
        _libmod._WRAP = _wrap
        RECORDING = self
        self.thread = threading.get_ident()
        # the C-ABI calls keep the recording's stream handles, while the py() actions (DDP, Adam) order
        # their side streams against torch's current stream at replay time: the two must agree
        self.stream = torch.cuda.current_stream()
        self.pool = torch.cuda.MemPool()
        try:
            with torch.autograd.set_multithreading_enabled(False), torch.cuda.use_mem_pool(self.pool), _Mode(self):
                self.result = fn()
        finally:
            RECORDING = None
            _libmod._WRAP = None
            lib.__dict__.clear()
            lib.__dict__.update(saved)
        self._finish()
        return self.result

    def _finish(self):
        # argument slots that point into an input tensor (rebased per replay) or carry a Dyn value
        patched = []
        for k, c in enumerate(self.calls):
            if c[0] != "c":
                continue
            slots = []
            for j, a in enumerate(c[2]):
                if isinstance(a, Dyn):
                    slots.append((j, "dyn", a.getter))
                elif isinstance(a, int) and a > 4096:
                    for n, lo, hi in self._ranges:
                        if lo <= a < hi:
                            slots.append((j, n, a - lo))
                            break
            if slots:
                patched.append((k, slots))
            c[2] = [int(a) if isinstance(a, Dyn) else a for a in c[2]]
        self._patched = patched
        self.n_c = sum(1 for c in self.calls if c[0] == "c")
        self.n_py = sum(1 for c in self.calls if c[0] == "py")

    # ---- replay -----------------------------------------------------------------------------------
    def replay(self, **inputs):
        """issue the recorded step again; inputs: name -> tensor replacing the recording's input"""
        if torch.cuda.current_stream() != self.stream:
            raise RuntimeError("StepPlan.replay: the current stream is not the recording's (the recorded launches "
                               "would not be ordered against the replayed stream waits)")
        base = {}
        for n, t in inputs.items():
            ref = self.inputs[n]
            if t.shape != ref.shape or t.dtype != ref.dtype or t.stride() != ref.stride() or t.device != ref.device:
                raise ValueError(f"StepPlan.replay: input {n} {tuple(t.shape)} {t.dtype} does not match the "
                                 f"recording's {tuple(ref.shape)} {ref.dtype}")
            base[n] = t.data_ptr()
        calls = self.calls
        for k, slots in self._patched:
            args = calls[k][2]
            for j, n, off in slots:
                if n == "dyn":
                    args[j] = int(off())
                else:
                    args[j] = base.get(n, self.inputs[n].data_ptr()) + off
        for c in calls:
            kind = c[0]
            if kind == "c":
                c[1](*c[2])
            elif kind == "py":
                c[1](*c[2], **c[3])
            else:
                _, func, args, kwargs, stream, out = c
                with torch.cuda.stream(stream):
                    r = func(*args, **kwargs)
                    if out is not None:
                        out.copy_(r)
        return self.result

    def stats(self):
        try:
            pool = sum(seg["total_size"] for seg in self.pool.snapshot())
        except Exception:  # noqa: BLE001 - diagnostics only
            pool = 0
        return {"c_calls": self.n_c, "py_calls": self.n_py, "torch_ops": self.n_torch,
                "torch_op_names": sorted(set(self.torch_names)), "pool_gib": round(pool / 2 ** 30, 2)}
