"""Per-IPM-iteration MM kernel durations of the last batch in a rocprofv3 kernel trace:
python tools/mm_iters.py DIR  (DIR = rocprofv3 -d output of tools/profile_mm.sh)."""
import csv
import glob
import re
import sys

rows = list(csv.DictReader(open(glob.glob(sys.argv[1] + "/**/*kernel_trace.csv", recursive=True)[0])))


def short(n):
    m = re.search(r"(mm_\w+|ob_\w+|__amd\w+)", n)
    return m.group(1) if m else n


seq = sorted(((short(r["Kernel_Name"]), (int(r["End_Timestamp"]) - int(r["Start_Timestamp"])) / 1e6,
               int(r["Start_Timestamp"]), int(r["End_Timestamp"])) for r in rows), key=lambda s: s[2])
st = [i for i, s in enumerate(seq) if s[0] == "mm_rows_kernel"][-1]
sub = seq[st:]
its, cur = [], {}
for nm, d, _, _ in sub:
    key = {"mm_assemble_mfma_kernel": "asm", "mm_affine_kernel": "aff", "mm_final_kernel": "fin",
           "mm_reduce_kernel": "red"}.get(nm, "other")
    if key == "asm":
        its.append(cur)
        cur = {}
    cur[key] = cur.get(key, 0.0) + d
its.append(cur)
tot = {}
for i, c in enumerate(its):
    for k, v in c.items():
        tot[k] = tot.get(k, 0.0) + v
    print(i, {k: round(v, 2) for k, v in c.items()}, round(sum(c.values()), 2))
print("iterations", len(its) - 1, {k: round(v, 1) for k, v in tot.items()}, "sum", round(sum(tot.values()), 1))
print("wall of the batch (ms)", round((sub[-1][3] - sub[0][2]) / 1e6, 1))
