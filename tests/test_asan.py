"""Sanitizer runs: the host C++ of liboaxaca_boot (CSV reader, builder frame logic,
inference, sharding glue) and the oracle's C restatement, built with AddressSanitizer +
UndefinedBehaviorSanitizer (tests/asan/Makefile, host side only) and driven through their C
entry points (tests/asan/host_asan.cpp, tests/asan/oracle_asan.c). CPU only."""
import os
import shutil
import subprocess

import pytest

HERE = os.path.join(os.path.dirname(os.path.abspath(__file__)), "asan")


@pytest.fixture(scope="module")
def built():
    if not shutil.which("make") or not os.path.exists("/opt/rocm/bin/hipcc"):
        pytest.skip("needs make and hipcc")
    jobs = str(min(8, os.cpu_count() or 2))
    subprocess.run(["make", "-s", "-j", jobs, "-C", HERE], check=True, capture_output=True, timeout=900)
    return os.path.join(HERE, "build")


def _run(exe, *args):
    env = dict(os.environ, ASAN_OPTIONS="detect_leaks=1:abort_on_error=0", UBSAN_OPTIONS="print_stacktrace=1")
    p = subprocess.run([exe, *args], capture_output=True, text=True, timeout=300, env=env)
    out = p.stdout + p.stderr
    assert "AddressSanitizer" not in out and "runtime error" not in out and "LeakSanitizer" not in out, out
    assert p.returncode == 0, out
    return out


def test_host_code_under_asan_ubsan(built, tmp_path):
    assert "host_asan: ok" in _run(os.path.join(built, "host_asan"), str(tmp_path))


def test_oracle_under_asan_ubsan(built):
    assert "oracle_asan: ok" in _run(os.path.join(built, "oracle_asan"))
