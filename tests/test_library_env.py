"""The shipped engine library reads no environment (CPU only).

Every switch that used to come from an OB_* environment variable (Gram path, digit slices, the
Heckman erfc, the Machado-Mata reduction and tuning, timing ablations) is now an explicit option
(ob_set_option, include/oaxaca_boot.h); only `make tuning` builds read the environment. The A/B
variant that lost (A fragments through LDS, oz_gram_la_kernel) is gone from the source.
"""
import ctypes as C
import math
import os
import re
import subprocess

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
SO = os.path.join(ROOT, "oaxaca-blinder-rs_amd", "liboaxaca_boot.so")
LLVM = "/opt/rocm/lib/llvm/bin"


@pytest.fixture(scope="module")
def so_bytes():
    if not os.path.exists(SO):
        pytest.skip("engine library missing (run __graft_entry__.build())")
    with open(SO, "rb") as f:
        return f.read()


def _undefined_symbols():
    nm = os.path.join(LLVM, "llvm-nm") if os.path.exists(os.path.join(LLVM, "llvm-nm")) else "nm"
    out = subprocess.run([nm, "-D", "--undefined-only", SO], capture_output=True, text=True, check=True).stdout
    return {line.split()[-1].split("@")[0] for line in out.splitlines() if line.strip()}


def test_library_imports_no_getenv(so_bytes):
    und = _undefined_symbols()
    assert und, "nm listed no imports: the check would be vacuous"
    assert not {"getenv", "secure_getenv", "__secure_getenv"} & und


def test_library_names_no_tuning_variables(so_bytes):
    names = set(re.findall(rb"OB_(?:GRAM|MM|HK|L1|OZ)_[A-Z0-9_]+", so_bytes))
    assert not names, sorted(names)
    assert b"oz_gram_la_kernel" not in so_bytes


def test_options_are_explicit(N):
    lib = N.lib()
    assert lib.ob_tuning_build() == 0
    assert lib.ob_set_option(b"no_such_option", 1.0) == N.OB_E_INVALID
    assert lib.ob_set_option(b"gram_diag", 2.0) == N.OB_E_UNSUPPORTED  # ablations: tuning builds only
    assert lib.ob_set_option(b"gram_diag", math.nan) == N.OB_OK
    with N.option("gram_path", 1):
        pass
    N.set_option("mm_reduce", None)


def test_option_block_restores_the_outer_value(N):
    """option() restores what was set before the block, not the default."""
    assert N.get_option("mm_kappa") is None
    with N.option("mm_kappa", 3.5):
        assert N.get_option("mm_kappa") == 3.5
        with N.option("mm_kappa", 5.0):
            assert N.get_option("mm_kappa") == 5.0
        assert N.get_option("mm_kappa") == 3.5
    assert N.get_option("mm_kappa") is None
    v = __import__("ctypes").c_double()
    assert N.lib().ob_get_option(b"no_such_option", __import__("ctypes").byref(v)) == N.OB_E_INVALID

