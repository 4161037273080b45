"""Average rocprofv3 --pmc counters per dispatch for kernels matching a substring.
usage: python tools/pmc_kernel.py DIR SUBSTRING [SUBSTRING...]"""
import csv
import glob
import os
import sys
from collections import defaultdict

d, subs = sys.argv[1], sys.argv[2:]
per = defaultdict(lambda: defaultdict(float))  # (kernel, dispatch) -> counter -> value
for path in glob.glob(os.path.join(d, "**", "*counter_collection.csv"), recursive=True):
    for row in csv.DictReader(open(path)):
        name = row.get("Kernel_Name", "")
        hit = next((s for s in subs if s in name), None)
        if hit is None:
            continue
        key = (hit, row.get("Dispatch_Id") or row.get("Correlation_Id"))
        per[key][row["Counter_Name"]] += float(row["Counter_Value"])
agg = defaultdict(lambda: defaultdict(list))
for (k, _), cs in per.items():
    for c, v in cs.items():
        agg[k][c].append(v)
for k in subs:
    if k not in agg:
        continue
    print(k, "dispatches", len(next(iter(agg[k].values()))))
    for c, vs in sorted(agg[k].items()):
        print(f"  {c:28s} mean {sum(vs) / len(vs):.4e}")
