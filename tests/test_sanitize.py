"""The CPU checker's C code under AddressSanitizer + UBSan: builds
oracle/_san/libhfvoracle_san.so and runs tests/san_driver.py against it in a child process
with libasan preloaded.  CPU only."""
import os
import subprocess
import sys

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
SAN_SO = os.path.join(ROOT, "oracle", "_san", "libhfvoracle_san.so")


def _libasan():
    try:
        p = subprocess.run(["gcc", "-print-file-name=libasan.so"], capture_output=True, text=True, check=True)
    except (OSError, subprocess.CalledProcessError):
        return None
    path = p.stdout.strip()
    return path if os.path.isabs(path) and os.path.exists(path) else None


def test_oracle_under_asan_ubsan():
    asan = _libasan()
    if asan is None:
        pytest.skip("no libasan for the host compiler")
    b = subprocess.run(["make", "-C", os.path.join(ROOT, "oracle"), "san"], capture_output=True, text=True)
    if b.returncode != 0:
        pytest.skip("sanitizer build unavailable: " + b.stderr[-300:])
    env = dict(os.environ, LD_PRELOAD=asan, HFV_ORACLE_SO=SAN_SO,
               ASAN_OPTIONS="detect_leaks=0:abort_on_error=1",
               UBSAN_OPTIONS="halt_on_error=1:print_stacktrace=1")
    r = subprocess.run([sys.executable, os.path.join(ROOT, "tests", "san_driver.py")], env=env,
                       capture_output=True, text=True, timeout=600)
    assert r.returncode == 0, (r.stdout[-2000:], r.stderr[-4000:])
    assert "san ok" in r.stdout
