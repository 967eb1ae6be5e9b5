"""CPU checks of the drop-in boundary: the C-ABI header, the built library and the ctypes binding agree.

No compute is launched (this container has no GPU): the library must load, export every symbol
include/unetseg_hip.h declares, and the ctypes signature table must match the header's parameter
types one for one.  Error reporting (unetseg_last_error) is exercised through an argument check that
fails before any launch.
"""
import ctypes
import os
import re

import pytest

from conftest import REPO

HEADER = os.path.join(REPO, "include", "unetseg_hip.h")

# 8-byte integers (long, size_t, [unsigned] long long) share one ctypes class on LP64 Linux
_CTYPE = {"int": "I", "long": "Q", "float": "F", "size_t": "Q", "unsigned long long": "Q", "long long": "Q"}


def _prototypes():
    src = open(HEADER).read()
    src = re.sub(r"/\*.*?\*/", "", src, flags=re.S)
    protos = {}
    for m in re.finditer(r"^\s*([A-Za-z_][\w\s\*]*?)\b(unetseg_\w+)\s*\(([^;]*?)\)\s*;", src, re.S | re.M):
        ret, name, args = m.group(1).strip(), m.group(2), " ".join(m.group(3).split())
        params = [] if args in ("", "void") else [a.strip() for a in args.split(",")]
        protos[name] = (ret, params)
    return protos


def _kind(decl):
    """Map a C parameter/return declaration to the letter the ctypes table uses."""
    d = re.sub(r"\b(const|unsigned\s+char)\b", lambda m: "" if m.group(0) == "const" else m.group(0), decl)
    if "*" in d:
        return "S" if re.match(r"\s*char\s*\*", d) and "unsigned" not in d else "P"
    d = re.sub(r"\s+\w+$", "", d.strip()) if len(d.split()) > 1 else d.strip()
    return _CTYPE.get(" ".join(d.split()), d)


def test_header_parses():
    protos = _prototypes()
    assert len(protos) >= 40
    for must in ("unetseg_conv2d_fwd", "unetseg_conv2d_dgrad", "unetseg_conv2d_wgrad", "unetseg_bn_finalize",
                 "unetseg_lovasz_fwd", "unetseg_bce_fwd", "unetseg_confusion", "unetseg_adam", "unetseg_last_error"):
        assert must in protos


def test_signature_table_matches_header():
    from unetseg_hip import lib

    protos = _prototypes()
    assert set(protos) == set(lib.SIGNATURES), (set(protos) ^ set(lib.SIGNATURES))
    def letter(t):
        if t is ctypes.c_char_p:
            return "S"
        if t is ctypes.c_void_p:
            return "P"
        if t is ctypes.c_float:
            return "F"
        return {4: "I", 8: "Q"}[ctypes.sizeof(t)]

    for name, (ret, params) in protos.items():
        rt, at = lib.SIGNATURES[name]
        assert [letter(t) for t in at] == [_kind(p) for p in params], name
        assert letter(rt) == _kind(ret + " r"), (name, ret, rt)


def test_library_exports_every_symbol():
    from unetseg_hip import lib

    if not os.path.exists(lib.LIB_PATH):
        pytest.skip("libunetseg_hip.so not built (run __graft_entry__.build())")
    so = ctypes.CDLL(lib.LIB_PATH)
    missing = [n for n in _prototypes() if not hasattr(so, n)]
    assert not missing, missing
    assert so.unetseg_abi_version() == 1


def test_argument_errors_reported_without_device():
    """An argument check fails before any HIP call, sets the thread-local message and returns non-zero."""
    from unetseg_hip import lib

    if not os.path.exists(lib.LIB_PATH):
        pytest.skip("libunetseg_hip.so not built")
    raw = lib.load()
    rc = raw.unetseg_pack_input(0, None, 1, 3, 4, 4, 2, None, None)  # cpad < c
    assert rc != 0
    assert b"cpad" in raw.unetseg_last_error()
    with pytest.raises(RuntimeError, match="cpad"):
        lib.lib.pack_input(0, None, 1, 3, 4, 4, 2, None, None)
    # the round-6 row merge: null partials, and a statistics merge without nq == 2
    assert raw.unetseg_fin_merge_rows(None, 64, 1024, 0, 0, 2, None, None) != 0
    assert b"fin_merge_rows" in raw.unetseg_last_error()
    with pytest.raises(RuntimeError, match="statistics merge"):
        lib.lib.fin_merge_rows(16, 64, 1024, 4096, 256, 3, 16, None)


def test_fastcall_binding_matches_ctypes():
    """The CPython fast-call binding (unetseg_hip/gen_fastcall.py) covers every int / float / pointer
    entry point, returns what the ctypes call returns and raises the same status errors."""
    from unetseg_hip import lib

    if not os.path.exists(lib.LIB_PATH):
        pytest.skip("libunetseg_hip.so not built")
    raw = lib.load()
    fast = lib._fast()
    if fast is None:
        pytest.skip("fast-call binding not built (make -C unet-embroidery-seg_amd/csrc)")
    from unetseg_hip.gen_fastcall import supported
    names = [n[len("unetseg_"):] for n, _, _ in supported()]
    assert len(names) >= 90 and all(hasattr(fast, n) for n in names)
    # value-returning queries agree with ctypes
    for args in ((1, 1 << 20, 64, None, None), (0, 4096, 2048, None, None)):
        assert fast.reduce_tiles(*args) == raw.unetseg_reduce_tiles(*args)
    assert fast.conv2d_wgrad_workspace(1, 16, 128, 128, 64, 64, 3, 3) == \
        raw.unetseg_conv2d_wgrad_workspace(1, 16, 128, 128, 64, 64, 3, 3)
    assert fast.abi_version() == 1
    # status errors: same exception type and message as the ctypes wrapper
    with pytest.raises(RuntimeError, match="unetseg_pack_input failed .*cpad"):
        fast.pack_input(0, None, 1, 3, 4, 4, 2, None, None)
    with pytest.raises(TypeError):
        fast.pack_input(0, None)
    assert lib.lib.pack_input is fast.pack_input  # the op layer's lib.<name> resolves to the binding
