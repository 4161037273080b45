"""The hand-counted vector-memory waits of the i8 Gram, checked on the built gfx950 ISA (CPU only).

oz_gram_kernel (ob_gram_i8.hip) stages B sub-tiles by inline-asm LDS-DMA the compiler does not
track and publishes them with hand-counted `s_waitcnt vmcnt(N)` before each barrier. Round 3
shipped, then reverted (632ee2d), a variant whose untracked A loads had their registers reused by
the compiler while in flight -- a GPU fault that no source review showed. tools/isa_vmem_check.py
walks the kernel's control flow with the outstanding vector-memory operations and reports a DMA
still in flight at a barrier two or more barriers after it was issued, and any instruction that
touches a register an un-waited load will still write ("Waits").
"""
import os
import re
import sys

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "tools"))
import isa_vmem_check as C  # noqa: E402

SO = os.path.join(ROOT, "oaxaca-blinder-rs_amd", "liboaxaca_boot.so")
GRAM = "_ZN12_GLOBAL__N_114oz_gram_kernelILi0EEEvNS_6OzArgsE"  # oz_gram_kernel<0>: the default


@pytest.fixture(scope="module")
def gram_isa():
    if not os.path.exists(SO) or not os.path.exists(os.path.join(C.LLVM, "llvm-objdump")):
        pytest.skip("engine library or llvm-objdump missing (run __graft_entry__.build())")
    return C.disassemble_symbol(SO, GRAM)


def test_shipped_gram_kernel_waits_are_clean(gram_isa):
    insns = C.parse(gram_isa, GRAM)
    dma = sum(1 for i in insns if i.mnem.startswith("global_load_lds"))
    bars = sum(1 for i in insns if i.mnem == "s_barrier")
    assert dma >= 64 and bars >= 40, (len(insns), dma, bars)  # the loop bodies were parsed
    assert C.check(insns) == []


def test_checker_flags_the_reverted_manual_a_variant():
    """The compiled code of commit 32e45ae (tests/isa/reverted_manual_a.s, tools/isa_reverted_excerpt.sh):
    the epilogue writes v42 while the dead inline-asm A load into v[42:45] is still in flight."""
    with open(os.path.join(ROOT, "tests", "isa", "reverted_manual_a.s")) as f:
        insns = C.parse(f.read())
    found = C.check(insns)
    assert ("vgpr-busy", 0x26F10) in {(r, a) for r, a, _ in found}, found[:3]


def test_checker_flags_a_wait_that_leaves_a_published_stage_in_flight(gram_isa):
    """The shipped ISA with every partial wait (vmcnt(N), N > 0: the publishing waits leave the
    wave's loads of the last steps in flight) widened to vmcnt(62): the stages published at a
    barrier are no longer guaranteed to have landed."""
    mutated = re.sub(r"s_waitcnt vmcnt\([1-9][0-9]?\)", "s_waitcnt vmcnt(62)", gram_isa)
    assert mutated != gram_isa
    rules = {r for r, _, _ in C.check(C.parse(mutated, GRAM))}
    assert "dma-age" in rules


def test_checker_flags_a_register_reused_under_a_load():
    text = """0000000000001000 <k>:
	global_load_dwordx4 v[8:11], v2, s[4:5]                    // 000000001000: DC5C8000 08040002
	v_mov_b32_e32 v9, 0                                        // 000000001008: 7E120280
	s_waitcnt vmcnt(0)                                         // 00000000100C: BF8C0F70
	v_mov_b32_e32 v10, 0                                       // 000000001010: 7E140280
	s_endpgm                                                   // 000000001014: BF810000
"""
    found = C.check(C.parse(text))
    assert [(r, a) for r, a, _ in found] == [("vgpr-busy", 0x1008)]


WIDE = "_ZN12_GLOBAL__N_116oz_gram_w_kernelILi0EEEvNS_6OzArgsE"  # oz_gram_w_kernel: the wide tile (round 6)


def test_shipped_wide_gram_kernel_waits_are_clean():
    """The wide-tile kernel uses the same untracked LDS-DMA ring with hand-counted waits (a 4-stage
    ring, one barrier per sub-tile, PER = 2 NB + 12) and pins its accumulators to AGPRs through
    inline-asm MFMAs: the walk must find no DMA older than two barriers at a barrier and no
    register (VGPR or AGPR) touched under an un-waited load."""
    if not os.path.exists(SO) or not os.path.exists(os.path.join(C.LLVM, "llvm-objdump")):
        pytest.skip("engine library or llvm-objdump missing (run __graft_entry__.build())")
    isa = C.disassemble_symbol(SO, WIDE)
    insns = C.parse(isa, WIDE)
    dma = sum(1 for i in insns if i.mnem.startswith("global_load_lds"))
    bars = sum(1 for i in insns if i.mnem == "s_barrier")
    mfma = sum(1 for i in insns if i.mnem.startswith("v_mfma_i32_16x16x64_i8"))
    assert dma >= 64 and bars >= 40 and mfma >= 1000, (len(insns), dma, bars, mfma)
    assert C.check(insns) == []
