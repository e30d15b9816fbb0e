"""Host-side AddressSanitizer run of the C ABI's validation paths.

`make -C articulated-object-nerf_amd/csrc asan` (run by __graft_entry__.build()) builds
lib/asan/libaonerf_asan.so -- the library with its host code under -fsanitize=address -- and
tools/asan_capi.cpp against it.  The driver calls entry points with invalid arguments (null
pointers, bad shapes, misaligned buffers, bad precisions / scales / counts) that must fail
validation before any GPU work, with a message in aon_last_error(); ASan (leak checking on)
aborts on any out-of-bounds access, use-after-free or leak on those paths.  No GPU needed.
"""
import os
import subprocess

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
BIN = os.path.join(ROOT, "articulated-object-nerf_amd", "lib", "asan", "asan_capi")


@pytest.mark.skipif(not os.path.exists(BIN), reason="ASan build absent (make -C csrc asan)")
def test_capi_validation_under_asan():
    env = dict(os.environ, ASAN_OPTIONS="detect_leaks=1:abort_on_error=0")
    env.pop("LD_PRELOAD", None)  # the driver links its own sanitizer runtime
    r = subprocess.run([BIN], capture_output=True, text=True, env=env, timeout=120)
    print(r.stdout[-2000:], r.stderr[-2000:])
    assert r.returncode == 0 and "ASAN_CAPI_OK" in r.stdout
