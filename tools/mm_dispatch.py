"""Per-dispatch durations of the MM kernels from a rocprofv3 kernel trace: python tools/mm_dispatch.py DIR [N]."""
import csv
import glob
import sys

rows = list(csv.DictReader(open(glob.glob(sys.argv[1] + "/**/*kernel_trace.csv", recursive=True)[0])))
n = int(sys.argv[2]) if len(sys.argv) > 2 else 40
out = []
for r in rows:
    name = r["Kernel_Name"]
    if "mm_" not in name:
        continue
    short = name.split("mm_")[1].split("(")[0].split("<")[0]
    out.append((short, (int(r["End_Timestamp"]) - int(r["Start_Timestamp"])) / 1e6))
for i, (nm, d) in enumerate(out[:n]):
    print(i, nm, round(d, 3))
