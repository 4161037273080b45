"""Summarise a kernel's ISA from `hipcc -S --cuda-device-only` output: scratch accesses,
barriers, vmcnt waits (counted vs full drains), VMEM instruction counts.
usage: python tools/isa_waits.py file.s kernel_substring [kernel_substring ...]"""
import re
import sys
from collections import Counter


def kernels(text):
    for m in re.finditer(r"^(_Z\S+):\s*; @", text, re.M):
        yield m.group(1), m.start()


def main():
    text = open(sys.argv[1]).read()
    for want in sys.argv[2:]:
        for name, start in kernels(text):
            if want not in name:
                continue
            end = text.index(".Lfunc_end", start)
            body = text[start:end].splitlines()
            sc = sum("scratch_" in l for l in body)
            bars = [k for k, l in enumerate(body) if "s_barrier" in l]
            waits = Counter(l.strip() for l in body if "s_waitcnt" in l and "vmcnt" in l)
            vm = Counter(l.split()[0] for l in body if re.match(r"\s+(global|buffer)_(load|store)", l))
            print(f"{name}\n  lines {len(body)} scratch {sc} barriers at {bars}")
            print("  vmcnt waits:", dict(waits.most_common(10)))
            print("  vmem:", dict(vm))
            for b in bars:  # the waits just before each barrier
                pre = [l.strip() for l in body[max(0, b - 4):b] if "s_waitcnt" in l]
                print(f"  barrier {b}: {pre}")


if __name__ == "__main__":
    main()
