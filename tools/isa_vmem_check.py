#!/usr/bin/env python3
"""Static check of the vector-memory waits in a gfx950 kernel's final ISA (llvm-objdump output).

Why: oz_gram_kernel (ob_gram_i8.hip) issues its B sub-tiles as untracked inline-asm LDS-DMA and
waits for them with hand-counted `s_waitcnt vmcnt(N)` before each publishing barrier. Whether
those counts are right depends on the issue order the compiler emits, and round 3 once shipped
a variant (commit 32e45ae, reverted by 632ee2d) whose untracked A-fragment loads had their
destination registers reused by the compiler while the loads were still in flight -- a GPU
fault. Neither shows in a source diff; both show in the ISA. This walks the kernel's control-
flow graph with the set of outstanding vector-memory operations (in issue order, as `vmcnt`
counts them: loads, stores and LDS-DMA together) and reports:

  dma-age     an LDS-DMA still outstanding at an `s_barrier` although it was issued before the
              barrier two barriers back: the ring publishes stage s + 1 at barrier s, and that
              stage was issued right after barrier s - 3 (ob_gram_i8.hip, oz_gram_body's step):
              only the pieces issued after barriers s - 2 and s - 1 may still be in flight;
  vgpr-busy   an instruction that reads or writes a VGPR / AGPR that an outstanding load will
              still write (RAW or WAW on the destination of an un-waited load).

Usage: isa_vmem_check.py <disassembly.s> [symbol]   (exit 1 and one line per finding on failure)
       isa_vmem_check.py --so liboaxaca_boot.so <symbol>   (extracts the gfx950 code object)
"""
from __future__ import annotations

import os
import re
import struct
import subprocess
import sys
import tempfile

LLVM = "/opt/rocm/lib/llvm/bin"
MAX_DMA_AGE = 2  # barriers a DMA may have passed and still be outstanding at the next one

_LINE = re.compile(r"^\s+([a-z][a-z0-9_]*)(.*?)//\s*([0-9A-Fa-f]+):")
_TARGET = re.compile(r"<[^>+]*\+0x([0-9a-fA-F]+)>")
_REG = re.compile(r"\b([va])(?:\[(\d+):(\d+)\]|(\d+)\b)")
_VMCNT = re.compile(r"vmcnt\((\d+)\)")


class Insn:
    __slots__ = ("addr", "mnem", "ops", "target")

    def __init__(self, addr, mnem, ops, target):
        self.addr, self.mnem, self.ops, self.target = addr, mnem, ops, target


def parse(text: str, symbol: str | None = None):
    """Instructions of one function of an llvm-objdump -d listing (the first one if no symbol)."""
    out, base, on = [], None, symbol is None
    for line in text.splitlines():
        m = re.match(r"^([0-9a-fA-F]+) <([^>]+)>:", line)
        if m:
            if on and out:
                break
            on = symbol is None or m.group(2) == symbol
            base = int(m.group(1), 16)
            continue
        if not on:
            continue
        m = _LINE.match(line)
        if not m:
            continue
        mnem, ops, addr = m.group(1), m.group(2).strip(), int(m.group(3), 16)
        t = _TARGET.search(line)
        target = base + int(t.group(1), 16) if (t and base is not None and mnem.startswith("s_")) else None
        out.append(Insn(addr, mnem, ops, target))
    return out


def regs(ops: str):
    """Registers named in an operand string: {('v', n), ('a', n), ...}."""
    r = set()
    for kind, lo, hi, one in _REG.findall(ops):
        if one:
            r.add((kind, int(one)))
        else:
            r.update((kind, i) for i in range(int(lo), int(hi) + 1))
    return r


def first_operand_regs(ops: str):
    head = ops.split(",")[0] if ops else ""
    return regs(head)


def is_vmem(m):
    return m.startswith(("global_", "buffer_", "scratch_", "flat_"))


def vmem_entry(insn: Insn):
    """(kind, dst registers) of a vector-memory instruction."""
    m = insn.mnem
    if "_lds" in m and "load" in m:
        return ("dma", frozenset())
    if "load" in m or ("atomic" in m and (" sc0" in insn.ops or " glc" in insn.ops)):
        return ("load", frozenset(first_operand_regs(insn.ops)))
    return ("store", frozenset())


def blocks(insns):
    """Basic blocks: start index -> (end index exclusive, successor start indices)."""
    idx = {ins.addr: i for i, ins in enumerate(insns)}
    leaders = {0}
    for i, ins in enumerate(insns):
        if ins.target is not None and ins.mnem.startswith(("s_branch", "s_cbranch")):
            if ins.target in idx:  # a target outside the listing (an excerpt) is an exit
                leaders.add(idx[ins.target])
            leaders.add(i + 1)
        elif ins.mnem in ("s_endpgm", "s_setpc_b64"):
            leaders.add(i + 1)
    starts = sorted(x for x in leaders if x < len(insns))
    bb = {}
    for k, s in enumerate(starts):
        e = starts[k + 1] if k + 1 < len(starts) else len(insns)
        last = insns[e - 1]
        succ = []
        tgt = [idx[last.target]] if last.target in idx else []
        if last.mnem.startswith("s_branch") and last.target is not None:
            succ = tgt
        elif last.mnem.startswith("s_cbranch") and last.target is not None:
            succ = tgt + ([e] if e < len(insns) else [])
        elif last.mnem in ("s_endpgm", "s_setpc_b64"):
            succ = []
        elif e < len(insns):
            succ = [e]
        bb[s] = (e, succ)
    return bb


KEEP = 24  # newest outstanding operations tracked one by one; older ones are folded into a summary


def step(insn: Insn, state, findings, where):
    """One instruction on one abstract state (tail, queue): queue = the newest outstanding
    operations (kind, age, dsts), oldest first, at most KEEP of them; tail = None, or a summary
    (dsts, oldest DMA age or -1) of older ones that may still be outstanding (a wait that leaves
    KEEP or more in flight cannot retire them). Returns the new state."""
    tail, q = state
    m = insn.mnem
    if m == "s_waitcnt":
        v = _VMCNT.search(insn.ops)
        if v:
            n = int(v.group(1))
            if n < len(q):
                q, tail = q[len(q) - n:], None
            elif n < len(q) + (tail is not None):
                tail = None if n == len(q) else tail
        return (tail, q)
    touched = regs(insn.ops)
    if is_vmem(m) and vmem_entry(insn)[0] == "load":
        # a load into a register a pending load also writes is ordered behind it (loads return in
        # issue order); only its address and data operands must not be pending
        touched = regs(",".join(insn.ops.split(",")[1:]))
    if touched:
        busy = [d for k, _, d in q if k == "load"] + ([tail[0]] if tail else [])
        for dst in busy:
            hit = dst & touched
            if hit:
                findings.add(("vgpr-busy", where, f"{m} {insn.ops} touches {sorted(hit)[:4]} of an un-waited load"))
                break
    if m == "s_barrier":
        ages = [a for k, a, _ in q if k == "dma"] + ([tail[1]] if tail and tail[1] >= 0 else [])
        if ages and max(ages) >= MAX_DMA_AGE:
            findings.add(("dma-age", where, f"LDS-DMA issued {max(ages)} barriers back still outstanding"))
        q = tuple((k, min(a + 1, MAX_DMA_AGE + 1) if k == "dma" else a, d) for k, a, d in q)
        if tail and tail[1] >= 0:
            tail = (tail[0], min(tail[1] + 1, MAX_DMA_AGE + 1))
        return (tail, q)
    if is_vmem(m):
        kind, dst = vmem_entry(insn)
        q = q + ((kind, 0, dst),)
        if len(q) > KEEP:
            (k0, a0, d0), q = q[0], q[1:]
            a0 = a0 if k0 == "dma" else -1
            tail = (d0 if k0 == "load" else frozenset(), a0) if tail is None else \
                (tail[0] | (d0 if k0 == "load" else frozenset()), max(tail[1], a0))
    return (tail, q)


def check(insns, max_states=500_000):
    """Fixed point over the CFG with a set of abstract states per block entry. Returns findings
    [(rule, address, message)] sorted by address."""
    if not insns:
        raise ValueError("no instructions (symbol not found?)")
    bb = blocks(insns)
    entry = {0: {(None, ())}}
    work = [0]
    findings = set()
    seen = 0
    while work:
        s = work.pop()
        e, succ = bb[s]
        outs = set()
        for st in entry[s]:
            for i in range(s, e):
                st = step(insns[i], st, findings, insns[i].addr)
            outs.add(st)
        for t in succ:
            cur = entry.setdefault(t, set())
            new = outs - cur
            if new:
                cur |= new
                seen += len(new)
                if seen > max_states:
                    raise RuntimeError("abstract state set did not converge")
                work.append(t)
    return sorted(findings, key=lambda f: (f[1], f[0]))


def extract_gfx950(so_path, out_dir):
    """The gfx950 code objects of an uncompressed clang offload bundle set inside a host binary."""
    data = open(so_path, "rb").read()
    magic = b"__CLANG_OFFLOAD_BUNDLE__"
    paths, i, k = [], 0, 0
    while True:
        i = data.find(magic, i)
        if i < 0:
            break
        (n,) = struct.unpack_from("<Q", data, i + 24)
        p = i + 32
        for _ in range(n):
            off, size, tl = struct.unpack_from("<QQQ", data, p)
            p += 24
            triple = data[p:p + tl].decode()
            p += tl
            if "gfx950" in triple and size:
                path = os.path.join(out_dir, f"co{k}.elf")
                with open(path, "wb") as f:
                    f.write(data[i + off:i + off + size])
                paths.append(path)
        k += 1
        i += len(magic)
    return paths


def disassemble_symbol(so_path, symbol):
    """llvm-objdump listing of `symbol` from whichever gfx950 code object of so_path defines it."""
    with tempfile.TemporaryDirectory() as d:
        for co in extract_gfx950(so_path, d):
            syms = subprocess.run([f"{LLVM}/llvm-readelf", "-s", co], capture_output=True, text=True).stdout
            if symbol in syms:
                return subprocess.run([f"{LLVM}/llvm-objdump", "-d", "--mcpu=gfx950", f"--disassemble-symbols={symbol}",
                                       co], capture_output=True, text=True, check=True).stdout
    raise FileNotFoundError(f"{symbol} not in any gfx950 code object of {so_path}")


def main(argv):
    if len(argv) >= 3 and argv[0] == "--so":
        text, sym = disassemble_symbol(argv[1], argv[2]), argv[2]
    else:
        text, sym = open(argv[0]).read(), (argv[1] if len(argv) > 1 else None)
    insns = parse(text, sym)
    f = check(insns)
    for rule, addr, msg in f:
        print(f"{rule} @0x{addr:x}: {msg}")
    print(f"{len(insns)} instructions, {sum(1 for i in insns if 'global_load_lds' in i.mnem)} LDS-DMA, "
          f"{sum(1 for i in insns if i.mnem == 's_barrier')} barriers: {len(f)} findings", file=sys.stderr)
    return 1 if f else 0


if __name__ == "__main__":
    sys.exit(main(sys.argv[1:]))
