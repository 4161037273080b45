"""f64 VALU FLOPs per dispatch of one kernel from a rocprofv3 --pmc run of SQ_INSTS_VALU_{ADD,MUL,
FMA,TRANS}_F64 (wave-level instruction counts; FLOPs = 64 lanes x (ADD + MUL + TRANS + 2 FMA), i.e.
every lane counted, masked-off lanes included). Only the dispatches with the largest grid count
(the bootstrap segment, not the one-replicate point estimate). Writes the JSON summary bench.py
--heckman reads.
usage: python tools/pmc_f64.py DIR KERNEL_SUBSTRING OUT.json [key=value ...]"""
import csv
import glob
import json
import os
import sys
from collections import defaultdict

d, sub, out = sys.argv[1], sys.argv[2], sys.argv[3]
extra = dict(a.split("=", 1) for a in sys.argv[4:])
per = defaultdict(lambda: defaultdict(float))
grid = {}
for path in glob.glob(os.path.join(d, "**", "*counter_collection.csv"), recursive=True):
    for row in csv.DictReader(open(path)):
        if sub not in row.get("Kernel_Name", ""):
            continue
        key = row.get("Dispatch_Id") or row.get("Correlation_Id")
        per[key][row["Counter_Name"]] += float(row["Counter_Value"])
        grid[key] = int(row.get("Grid_Size") or 0)
if not per:
    sys.exit(f"no dispatch of {sub} in {d}")
gmax = max(grid.values())
per = {k: v for k, v in per.items() if grid[k] == gmax}
tot = defaultdict(float)
for cs in per.values():
    for c, v in cs.items():
        tot[c] += v
n = len(per)
flops = 64.0 * (tot["SQ_INSTS_VALU_ADD_F64"] + tot["SQ_INSTS_VALU_MUL_F64"] + tot["SQ_INSTS_VALU_TRANS_F64"]
                + 2.0 * tot["SQ_INSTS_VALU_FMA_F64"])
res = {"kernel": sub, "dispatches": n, "grid_size": gmax, "counters_total": dict(tot), "f64_flops_per_dispatch": flops / n,
       "note": "FLOPs = 64 x (ADD + MUL + TRANS + 2 FMA) f64 VALU wave instructions, summed over dispatches / n"}
res.update({k: (int(v) if v.isdigit() else v) for k, v in extra.items()})
json.dump(res, open(out, "w"), indent=1)
print(json.dumps(res, indent=1))
