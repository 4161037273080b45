"""Sum rocprofv3 PMC counters and kernel-trace durations over every dispatch of one kernel.

usage: python tools/pmc_sum.py PMC_DIR KERNEL_SUBSTRING   (one line: counters, dispatches, wall_ms)
"""
import csv
import glob
import os
import sys


def main():
    d, sub = sys.argv[1], sys.argv[2]
    tot, disp = {}, set()
    for path in glob.glob(os.path.join(d, "**", "*counter_collection.csv"), recursive=True):
        for row in csv.DictReader(open(path)):
            if sub in row.get("Kernel_Name", ""):
                tot[row["Counter_Name"]] = tot.get(row["Counter_Name"], 0.0) + float(row["Counter_Value"])
                disp.add(row.get("Dispatch_Id") or row.get("Correlation_Id"))
    wall = 0.0
    for path in glob.glob(os.path.join(d, "**", "*kernel_trace.csv"), recursive=True):
        for row in csv.DictReader(open(path)):
            if sub in row.get("Kernel_Name", ""):
                wall += (float(row["End_Timestamp"]) - float(row["Start_Timestamp"])) * 1e-6
    print(f"{sub}: dispatches={len(disp)} wall_ms={wall:.2f} " + " ".join(f"{k}={v:.4g}" for k, v in sorted(tot.items())))


if __name__ == "__main__":
    main()
