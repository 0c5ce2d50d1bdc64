"""Host-code AddressSanitizer run of libptk's C ABI (SURVEY §5 "race detection / sanitizers": a debug build with
-fsanitize=address for host code).  CPU only: `make asan` compiles every product source with its host side
instrumented (-Xarch_host -fsanitize=address; device code untouched) and links tests/asan/host_abi_check.cpp,
which drives the host-side work of the ABI (workspace layouts, resize coefficients, validation, census, stage
timers).  A negative control proves the instrumentation is live: an undersized buffer must trip ASan."""
import os
import shutil
import subprocess

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
CSRC = os.path.join(ROOT, "projectiontrainer_amd", "csrc")
BIN = os.path.join(ROOT, "build", "asan", "host_abi_check")
ENV = {**os.environ, "ASAN_OPTIONS": "detect_leaks=0:abort_on_error=0", "PTK_STAGE_TIMERS": "0"}


@pytest.fixture(scope="module")
def asan_bin():
    if not os.path.exists("/opt/rocm/bin/hipcc") or shutil.which("make") is None:
        pytest.skip("hipcc / make not available")
    subprocess.run(["make", "-s", "-j8", "-C", CSRC, "asan"], check=True, timeout=900,
                   stdout=subprocess.DEVNULL, stderr=subprocess.PIPE)
    return BIN


def test_host_abi_under_asan(asan_bin):
    r = subprocess.run([asan_bin], env=ENV, capture_output=True, text=True, timeout=300)
    assert "AddressSanitizer" not in r.stderr, r.stderr[-4000:]
    assert r.returncode == 0, r.stderr[-4000:]
    assert "host_abi_check: ok" in r.stdout


def test_asan_instrumentation_is_live(asan_bin):
    r = subprocess.run([asan_bin, "--overflow-probe"], env=ENV, capture_output=True, text=True, timeout=300)
    assert r.returncode != 0
    assert "heap-buffer-overflow" in r.stderr and "ptk_resize_coeffs" in r.stderr
