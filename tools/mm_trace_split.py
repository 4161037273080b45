"""Split a rocprofv3 kernel trace of bench.py --mm by phase: kernel time per (kernel, grid x) and
the idle gaps between kernels. usage: python tools/mm_trace_split.py run_kernel_trace.csv"""
import collections
import csv
import sys

rows = sorted(csv.DictReader(open(sys.argv[1])), key=lambda r: int(r["Start_Timestamp"]))
tot = collections.defaultdict(lambda: [0, 0.0])
gap = 0.0
prev_end = None
first = int(rows[0]["Start_Timestamp"])
for r in rows:
    s, e = int(r["Start_Timestamp"]), int(r["End_Timestamp"])
    name = r["Kernel_Name"].replace("(anonymous namespace)::", "").replace("void ", "")
    name = name.split("(")[0]
    key = (name, int(r["Grid_Size_X"]) // max(1, int(r["Workgroup_Size_X"])))
    tot[key][0] += 1
    tot[key][1] += (e - s) / 1e6
    if prev_end is not None and s > prev_end:
        gap += (s - prev_end) / 1e6
    prev_end = max(prev_end or 0, e)
span = (prev_end - first) / 1e6
print(f"span {span:.1f} ms, kernel-free gaps {gap:.1f} ms")
for k, (n, ms) in sorted(tot.items(), key=lambda kv: -kv[1][1])[:30]:
    print(f"{ms:9.2f} ms {n:6d}x  {k[0]} grid.x={k[1]}")
