"""Instruction histogram of one kernel in a `hipcc -S --cuda-device-only` file.
usage: python tools/isa_hist.py file.s kernel_substring [top]"""
import re
import sys
from collections import Counter

text = open(sys.argv[1]).read()
want, top = sys.argv[2], int(sys.argv[3]) if len(sys.argv) > 3 else 40
for m in re.finditer(r"^(_Z\S+):\s*; @", text, re.M):
    if want not in m.group(1):
        continue
    body = text[m.start():text.index(".Lfunc_end", m.start())].splitlines()
    ins = [l.split()[0] for l in body if re.match(r"\s+[a-z_]+[0-9a-z_]*\s", l) and not l.strip().startswith(";")]
    c = Counter(ins)
    print(m.group(1), "instructions", len(ins))
    cls = Counter()
    for k, v in c.items():
        cls["mfma" if "mfma" in k else k.split("_")[0] + ("_f64" if "f64" in k else "")] += v
    print(" classes:", dict(cls.most_common()))
    print(" top:", c.most_common(top))
