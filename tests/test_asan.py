"""Host-side AddressSanitizer + UBSan runs: the BVH builder
(csrc/bvh.cpp) over random and degenerate primitive sets with its structural
invariants checked, and the CPU oracle over small scenes with every primitive
kind and NaN / zero / axis-parallel query rays (tools/asan/)."""
import os
import shutil
import subprocess

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
ASAN = os.path.join(ROOT, "tools", "asan")


@pytest.fixture(scope="module")
def built():
    if not (shutil.which("gcc") and os.path.exists("/opt/rocm/bin/hipcc")):
        pytest.skip("needs gcc and hipcc")
    subprocess.run(["make", "-s", "-C", ASAN, "cpu"], check=True, capture_output=True, timeout=600)
    return os.path.join(ASAN, "build")


@pytest.mark.parametrize("exe", ["bvh_asan", "oracle_asan"])
def test_sanitized_driver(built, exe):
    env = dict(os.environ, ASAN_OPTIONS="detect_leaks=1:halt_on_error=1", UBSAN_OPTIONS="halt_on_error=1")
    r = subprocess.run([os.path.join(built, exe)], capture_output=True, text=True, timeout=300, env=env)
    assert r.returncode == 0, r.stdout[-2000:] + r.stderr[-4000:]
    assert "ALL OK" in r.stdout
    assert "runtime error" not in r.stderr and "AddressSanitizer" not in r.stderr
