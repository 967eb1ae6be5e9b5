"""CPU: host AddressSanitizer run over the C ABI's host code.

``make -C unet-embroidery-seg_amd/csrc asan`` compiles the library's own sources with the host side
instrumented (``-Xarch_host -fsanitize=address``; device code unchanged and never launched) and links
tests/asan/cabi_asan.cpp, which drives every host-side path that runs before a launch -- the
kernel-configuration / tile / workspace queries over a grid of shapes covering the BASELINE models'
layers plus ragged and degenerate ones, the argument checks of the launching entry points (each must
refuse with status 1 and a message), and the augmentation's walk over caller-provided descriptor /
table arrays.  ASan aborts the run on any out-of-bounds access, use after free or undefined shift
it instruments; the driver exits non-zero on a failed expectation.
"""
import os
import shutil
import subprocess

import pytest

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
CSRC = os.path.join(REPO, "unet-embroidery-seg_amd", "csrc")


@pytest.mark.timeout(900)
def test_cabi_host_asan():
    if not os.path.exists("/opt/rocm/bin/hipcc") or shutil.which("make") is None:
        pytest.skip("hipcc / make not available")
    jobs = str(min(8, os.cpu_count() or 2))
    b = subprocess.run(["make", "-C", CSRC, "asan", f"-j{jobs}"], capture_output=True, text=True)
    assert b.returncode == 0, b.stdout[-3000:] + b.stderr[-3000:]
    env = dict(os.environ, ASAN_OPTIONS="detect_leaks=0:verify_asan_link_order=0:abort_on_error=0:halt_on_error=1")
    r = subprocess.run([os.path.join(CSRC, "build", "asan", "cabi_asan")], capture_output=True, text=True, env=env,
                       timeout=600)
    out = r.stdout + r.stderr
    assert "AddressSanitizer" not in out, out[-4000:]
    assert r.returncode == 0, out[-4000:]
    assert " 0 failed" in r.stdout, r.stdout
