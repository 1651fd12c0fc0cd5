"""Host ASan + UBSan build of the native planning code (SURVEY §5 sanitizers):
tests/native/host_selftest.cpp via scripts/host_sanitize.sh -- fastdiv exactness,
conv split-K / workspace plans over ~7k shapes, head / BN workspace sizing.
Runs on the CPU (the device code is compiled, never launched)."""
import os
import shutil
import subprocess

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


@pytest.mark.skipif(not (shutil.which("hipcc") or os.path.exists("/opt/rocm/bin/hipcc")), reason="no hipcc")
def test_host_selftest_under_asan_ubsan():
    r = subprocess.run(["bash", os.path.join(ROOT, "scripts", "host_sanitize.sh")], capture_output=True, text=True,
                       timeout=900)
    assert r.returncode == 0, (r.stdout[-2000:], r.stderr[-4000:])
    assert "HOST_SELFTEST_OK" in r.stdout
