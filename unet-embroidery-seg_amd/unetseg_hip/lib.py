"""ctypes binding of libunetseg_hip.so (the C ABI declared in include/unetseg_hip.h).

The library is built in-tree by ``__graft_entry__.build()`` (hipcc --offload-arch=gfx950).  There is
no fallback: if the library or a HIP device is missing, every op raises.
"""
from __future__ import annotations

import ctypes
import os

_HERE = os.path.dirname(os.path.abspath(__file__))
LIB_PATH = os.environ.get("UNETSEG_LIB_PATH") or os.path.join(_HERE, "libunetseg_hip.so")  # override: A/B builds

DT_F32, DT_BF16 = 0, 1

P = ctypes.c_void_p
I = ctypes.c_int
L = ctypes.c_long
F = ctypes.c_float
SZ = ctypes.c_size_t
ULL = ctypes.c_ulonglong
LL = ctypes.c_longlong

# name -> (restype, argtypes)
SIGNATURES = {
    "unetseg_last_error": (ctypes.c_char_p, []),
    "unetseg_abi_version": (I, []),
    "unetseg_device_arch": (I, [ctypes.c_char_p, I]),
    "unetseg_conv_tile_m": (I, []),
    "unetseg_conv2d_fwd": (I, [I, P, I, I, P, I, I, I, I, I, P, I, I, I, I, I, P, I, P, I, P, P]),
    "unetseg_conv2d_fwd_tile_m": (I, [I, I, I, I, I, I, I, I, I, I, I, I, I]),
    "unetseg_conv2d_dgrad": (I, [I, P, I, I, I, I, P, I, I, I, I, I, I, P, I, I, I, I, P]),
    "unetseg_conv2d_wgrad_workspace": (SZ, [I, I, I, I, I, I, I, I]),
    "unetseg_conv2d_wgrad": (I, [I, P, I, I, P, I, I, I, I, I, P, I, I, I, I, I, I, P, SZ, P, I, I, P]),
    "unetseg_conv2d_wgrad_rows": (I, [I, P, I, I, I, I, I, P, I, I, I, I, I, I, P, SZ, P, I, I, I, P]),
    "unetseg_pack_conv_weight": (I, [I, P, I, I, I, I, I, P, P, P]),
    "unetseg_pack_conv_weights": (I, [I, P, I, L, P]),
    "unetseg_pack_tiles": (I, [I, I, I]),
    "unetseg_bn_fold": (I, [I, P, P, P, P, F, P, P, P, P]),
    "unetseg_conv2d_fwd_bnrelu_in": (I, [I, P, I, I, I, I, I, P, I, P, P, P, I, P, I, P, P]),
    "unetseg_conv2d_fwd_bnrelu_in_config": (I, [I, I, I, I, I, I, I]),
    "unetseg_conv2d_fwd_head_ok": (I, [I, I, I, I, I, I, I]),
    "unetseg_upsample2x_bwd_tiles": (I, [I, I, I, I, I]),
    "unetseg_upsample2x_bwd_relu": (I, [I, P, I, I, I, I, I, I, P, I, P, I, P, I, P]),
    "unetseg_conv2d_fwd_head": (I, [I, P, I, I, I, I, P, P, P, I, I, P, P, P, P]),
    "unetseg_conv2d_fwd_mask": (I, [I, P, I, I, I, I, P, P, P, I, P, P]),
    "unetseg_conv2d_wgrad_bnrelu_in": (I, [I, P, I, I, I, I, I, P, I, I, P, P, P, SZ, P, I, I, P]),
    "unetseg_conv2d_fwd_affine": (I, [I, P, I, I, P, I, I, I, I, I, P, I, I, I, I, I, P, P, I, P, I, P]),
    "unetseg_bn_finalize": (I, [P, I, I, L, I, P, P, P, P, P, F, F, P, P, P, P, P]),
    "unetseg_bn_eval_coeffs": (I, [I, P, P, P, P, F, P, P, P]),
    "unetseg_bn_apply": (I, [I, P, I, P, P, P, I, P, P, I, I, P, I, L, I, P]),
    "unetseg_bn_apply_mask": (I, [I, P, I, P, P, P, I, P, P, I, P, I, L, I, P, P]),
    "unetseg_reduce_tiles": (I, [I, L, I, P, P]),
    "unetseg_bn_bwd_reduce": (I, [I, P, I, P, I, P, P, P, I, P, P, P, I, P, P, L, I, P, I, P]),
    "unetseg_bn_bwd_finalize": (I, [P, I, I, L, I, P, P, P, P, P, P, P, P, P, P]),
    "unetseg_bn_bwd_apply": (I, [I, P, I, P, I, P, P, P, I, P, P, P, I, P, I, P, P, P, I, P, P, I, I, L, I, P]),
    "unetseg_relu_bwd_bias": (I, [I, P, I, P, I, P, I, L, I, P, I, P]),
    "unetseg_colsum_finalize": (I, [P, I, I, P, I, P]),
    "unetseg_maxpool_fwd": (I, [I, P, I, I, I, I, I, I, I, I, P, I, P, P, P, P]),
    "unetseg_maxpool_bwd": (I, [I, P, I, P, I, I, I, I, I, I, I, I, P, I, I, P]),
    "unetseg_upsample2x_fwd": (I, [I, P, I, I, I, I, I, I, P, I, P]),
    "unetseg_upsample2x_bwd": (I, [I, P, I, I, I, I, I, I, P, I, I, P]),
    "unetseg_pack_input": (I, [I, P, I, I, I, I, I, P, P]),
    "unetseg_pw_small_tiles": (I, [L]),
    "unetseg_pw_small_tile": (I, [L]),
    "unetseg_pw_small_fwd": (I, [I, P, I, L, I, I, I, P, P, P, P, P]),
    "unetseg_pw_small_bwd": (I, [I, P, P, I, L, I, I, I, P, P, I, I, P, P, P]),
    "unetseg_pw_small_bwd_relu": (I, [I, P, P, I, L, I, I, I, P, P, I, P, P, P, P]),
    "unetseg_attn_apply": (I, [I, P, I, P, P, P, P, P, I, L, I, P]),
    "unetseg_attn_bwd1_tiles": (I, [L]),
    "unetseg_attn_bwd1": (I, [I, P, I, P, I, P, P, P, P, P, I, I, P, L, I, P, P]),
    "unetseg_attn_bwd2": (I, [I, P, P, P, P, P, P, I, P, P, I, L, I, P, P, P]),
    "unetseg_add": (I, [I, P, I, P, I, L, I, P]),
    "unetseg_lovasz_workspace": (SZ, [I, L]),
    "unetseg_lovasz_fwd": (I, [P, I, P, I, L, P, SZ, P, P, P]),
    "unetseg_bce_workspace": (SZ, [I, L]),
    "unetseg_bce_fwd": (I, [P, I, P, I, L, P, P, SZ, P, P, P]),
    "unetseg_dz_to_dout": (I, [P, I, L, I, P, F, P, F, P, P, P]),
    "unetseg_confusion": (I, [P, I, P, I, L, P, P]),
    "unetseg_adam": (I, [P, P, P, P, L, F, F, F, F, F, I, P, P]),
    "unetseg_gap_fwd": (I, [I, P, I, I, I, I, P, P]),
    "unetseg_gap_bwd": (I, [I, P, I, I, I, P, I, I, P]),
    "unetseg_linear_fwd": (I, [P, P, P, I, I, I, I, F, ULL, P, P, P, P, P]),
    "unetseg_linear_bwd": (I, [P, P, P, F, I, P, P, I, I, I, P, P, P, P, P]),
    "unetseg_ce_fwd": (I, [P, P, I, I, P, P, P]),
    "unetseg_scale_grad": (I, [P, L, P, F, P, F, P, P]),
    "unetseg_stream_wait": (I, [P, P]),
    "unetseg_stream_create_cumask": (I, [P, I, P]),
    "unetseg_conv2d_dgrad_post": (I, [I, P, I, I, I, I, P, I, I, I, I, I, I, P, I, I, I, I, P, I, P, P, P, P, P, I,
                                      P]),
    "unetseg_bn_bwd_finalize_rows": (I, [P, I, I, L, P, P, P, P, P, P]),
    "unetseg_fin_merge_rows": (I, [P, I, I, L, I, I, P, P]),
    "unetseg_conv2d_dgrad_post_res": (I, [I, P, I, I, I, I, P, I, I, P, I, P, I, P, P, P, P, I, P, P, P, I, P]),
    "unetseg_bn_bwd_finalize_rows_res": (I, [P, I, I, L, I, P, P, P, P, P, P, P, P, P, P]),
    "unetseg_colsum_rows": (I, [P, I, I, I, P, I, P]),
    "unetseg_pack_input_stem": (I, [P, I, I, I, I, P, P]),
    "unetseg_stem_pack_weight": (I, [P, I, I, P, P]),
    "unetseg_stem_fwd_tile_m": (I, [I, I, I, I]),
    "unetseg_stem_fwd": (I, [P, I, I, I, P, I, P, I, P, P]),
    "unetseg_stem_wgrad_workspace": (SZ, [I, I, I, I]),
    "unetseg_stem_wgrad": (I, [P, I, I, I, P, I, I, P, SZ, P, I, I, P]),
    "unetseg_adam_dev": (I, [P, P, P, P, L, P, P, F, F, F, F, P, P]),
    "unetseg_conv2d_fwd_config": (I, [I, I, I, I, I, I, I, I, I, I, I, I, I, P]),
    "unetseg_conv2d_dgrad_config": (I, [I, I, I, I, I, I, I, I, I, I, I, I, I, I, P, P]),
    "unetseg_conv2d_wgrad_config": (I, [I, I, I, I, I, I, I, I, I, I, I, I, I, I, P]),
    "unetseg_stem_config": (I, [I, I, I, I, P]),
    "unetseg_pw_head_fwd": (I, [I, P, I, L, I, I, I, P, P, P, P]),
    "unetseg_pw_head_tiles": (I, [L]),
    "unetseg_pw_head_bwd": (I, [I, P, P, I, L, I, I, I, P, P, I, I, P, P, P]),
    "unetseg_mc_loss_workspace": (SZ, [I, I, L]),
    "unetseg_mc_loss_fwd": (I, [P, P, I, I, L, P, L, I, F, F, P, I, F, F, P, SZ, P, P]),
    "unetseg_mc_loss_bwd": (I, [P, P, I, I, L, P, L, I, F, F, P, I, F, F, P, P, P, P]),
    "unetseg_mc_confusion": (I, [P, P, I, I, L, P, P]),
    "unetseg_softmax_resize_argmax": (I, [P, I, I, I, I, I, I, I, I, I, P, P]),
    "unetseg_resize_bilinear_fwd": (I, [I, P, I, I, I, I, I, I, I, I, P, I, P]),
    "unetseg_resize_bilinear_bwd": (I, [I, P, I, I, I, I, I, I, I, I, P, I, I, P]),
    "unetseg_pad2d_fwd": (I, [I, P, I, I, I, I, I, I, I, I, I, P, I, P]),
    "unetseg_pad2d_bwd": (I, [I, P, I, I, I, I, I, I, I, I, I, P, I, I, P]),
    "unetseg_confusion_masked": (I, [P, I, P, I, L, L, P, P]),
    "unetseg_masked_loss_workspace": (SZ, [I, L]),
    "unetseg_masked_loss_fwd": (I, [P, I, P, I, L, L, I, P, P, SZ, P, P, P]),
    "unetseg_lovasz_fwd_masked": (I, [P, I, P, I, L, L, P, SZ, P, P, P]),
    "unetseg_channel_stats_tiles": (I, [L, I]),
    "unetseg_channel_stats": (I, [I, P, I, L, I, I, P, P]),
    "unetseg_augment_tables_len": (I, [LL, LL, LL, LL, LL]),
    "unetseg_augment_batch": (I, [P, P, I, P, P, LL, P, LL, P, LL, P, LL, P, LL, I, I, I, I, P, P, P, P]),
    "unetseg_augment_batch_dev": (I, [P, P, I, P, P, LL, P, LL, P, LL, P, LL, P, LL, I, I, I, I, P, P, P, P]),
    "unetseg_augment_tables_dev": (I, [P, I, P, P, I, P]),
}

#: functions returning a value rather than a status (no RuntimeError on non-zero)
VALUE_FUNCS = {"conv2d_fwd_mask", "reduce_tiles", "pw_small_tiles", "conv_tile_m", "abi_version", "conv2d_fwd_tile_m",
               "conv2d_dgrad_post", "conv2d_dgrad_post_res", "stem_fwd_tile_m", "attn_bwd1_tiles", "pw_small_tile", "conv2d_fwd_config",
               "conv2d_dgrad_config", "conv2d_wgrad_config", "stem_config", "pw_head_tiles", "channel_stats_tiles",
               "augment_tables_len", "pack_tiles",
               "conv2d_fwd_bnrelu_in_config", "conv2d_fwd_head_ok", "upsample2x_bwd_tiles"}

_lib = None


class HipUnavailable(RuntimeError):
    pass


def load(path: str = LIB_PATH):
    """Load the shared library and bind every C-ABI symbol (raises if absent)."""
    global _lib
    if _lib is not None:
        return _lib
    if not os.path.exists(path):
        raise HipUnavailable(
            f"libunetseg_hip.so not found at {path}: build it with `python -c 'import __graft_entry__ as g; g.build()'` "
            "(hipcc --offload-arch=gfx950).  There is no CPU fallback.")
    lib = ctypes.CDLL(path)
    for name, (res, args) in SIGNATURES.items():
        fn = getattr(lib, name)
        fn.restype = res
        fn.argtypes = args
    _lib = lib
    return lib


def exported_symbols():
    return list(SIGNATURES)


def last_error() -> str:
    return load().unetseg_last_error().decode("utf-8", "replace")


_FAST = None


def _fast():
    """the CPython fast-call binding (gen_fastcall.py, built next to the library by the csrc Makefile):
    the same entry points without ctypes' per-call conversion cost; None when absent or with
    UNETSEG_NO_FASTCALL=1.  With UNETSEG_LIB_PATH (A/B builds) the binding is taken from that library's
    directory (``make OUT=<dir>/libunetseg_hip.so`` builds both there; its rpath links the library beside
    it), so an A/B arm runs at the production host cost -- or not at all when that directory has none."""
    global _FAST
    if _FAST is None:
        _FAST = False
        if os.environ.get("UNETSEG_NO_FASTCALL", "0") != "1":
            try:
                if os.environ.get("UNETSEG_LIB_PATH") is None:
                    from . import _unetseg_fast
                    _FAST = _unetseg_fast
                else:
                    import glob
                    import importlib.util
                    cand = sorted(glob.glob(os.path.join(os.path.dirname(os.path.abspath(LIB_PATH)),
                                                         "_unetseg_fast*.so")))
                    if cand and os.path.basename(LIB_PATH) == "libunetseg_hip.so":
                        spec = importlib.util.spec_from_file_location("_unetseg_fast", cand[0])
                        mod = importlib.util.module_from_spec(spec)
                        spec.loader.exec_module(mod)
                        _FAST = mod
            except ImportError:
                pass
    return _FAST or None


#: set by plan.StepPlan.record: wraps every callable handed out (logging), none cached meanwhile
_WRAP = None


class _Caller:
    """lib.<name>(...) raises RuntimeError on a non-zero status.  The bound callable is cached on the
    instance after the first lookup (the op layer makes ~500 calls per training step); entry points the
    fast-call binding covers use it (same arguments, same status errors)."""

    def __getattr__(self, item):
        lib_ = load()
        fast = _fast()
        if fast is not None and hasattr(fast, item):
            fn = getattr(fast, item)
        else:
            raw = getattr(lib_, "unetseg_" + item)
            if SIGNATURES["unetseg_" + item][0] is I and item not in VALUE_FUNCS:
                def fn(*args, _raw=raw):
                    rc = _raw(*args)
                    if rc != 0:
                        raise RuntimeError(f"unetseg_{item} failed ({rc}): {last_error()}")
                    return rc
            else:
                fn = raw
        if _WRAP is not None:
            return _WRAP(item, fn)
        self.__dict__[item] = fn
        return fn


lib = _Caller()


# ------------------------------------------------------------------------------------------------
# kernel-configuration queries (host only; used by the parity tests and the bench's config table)
# ------------------------------------------------------------------------------------------------
CFG_NAMES = {0: "halo3", 1: "tn256x64", 2: "tn256x128", 3: "tn128x128", 4: "tn128x128_1step", 5: "tn64x128",
             6: "tn128x64", 7: "ring256x128", 8: "ring128x128", 9: "ring64x128", 10: "ring128x128_5st",
             11: "ring256x64", 12: "ring128x64_4st", 13: "ring128x64", 14: "ring256x64_8w", 17: "multi128x128",
             18: "multi64x128", 19: "tn128x128_1st", 20: "tn128x64_1st", 21: "ring256x128_halo", 22: "ring256x64_halo",
             23: "ring128x128_halo", 24: "ring256x128_hp", 25: "ring256x64_hp", 30: "stem_halo", 31: "first3x3", 100: "generic"}
WG_NAMES = {0: "halo3_wgrad", 1: "wgrad64x256_row", 2: "wgrad128_row", 3: "wgrad64x256", 4: "wgrad128",
            5: "wgrad_generic", 6: "wgrad_ring64x256", 7: "wgrad_ring128"}


def _cfg_name(cfg, taps):
    n = CFG_NAMES.get(cfg, str(cfg))
    return f"{n}_t{taps}" if taps else n


def fwd_config(dtype, c1, ldc1, c2, ldc2, n, h, w, cout, r, s, stride, pad):
    taps = ctypes.c_int(0)
    cfg = load().unetseg_conv2d_fwd_config(dtype, c1, ldc1, c2, ldc2, n, h, w, cout, r, s, stride, pad,
                                           ctypes.byref(taps))
    return _cfg_name(cfg, taps.value)


def dgrad_config(dtype, ldy, n, p, q, cout, cin, r, s, stride, pad, ldx, h, w):
    """list of configuration names, one per launched output-parity class"""
    cfg = (ctypes.c_int * 4)()
    taps = (ctypes.c_int * 4)()
    load().unetseg_conv2d_dgrad_config(dtype, ldy, n, p, q, cout, cin, r, s, stride, pad, ldx, h, w, cfg, taps)
    return [_cfg_name(cfg[i], taps[i]) for i in range(stride * stride) if cfg[i] >= 0]


def wgrad_config(dtype, c1, ldc1, c2, ldc2, n, h, w, ldy, cout, r, s, stride, pad):
    """(kernel name, split-K slabs, reduce kernel name)"""
    sp = ctypes.c_int(0)
    kind = load().unetseg_conv2d_wgrad_config(dtype, c1, ldc1, c2, ldc2, n, h, w, ldy, cout, r, s, stride, pad,
                                              ctypes.byref(sp))
    return WG_NAMES.get(kind, str(kind)), sp.value, "reduce"


def stem_config(n, h, w, K):
    sp = ctypes.c_int(0)
    cfg = load().unetseg_stem_config(n, h, w, K, ctypes.byref(sp))
    return CFG_NAMES.get(cfg, str(cfg)), sp.value
