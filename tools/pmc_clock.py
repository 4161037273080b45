"""Effective clock and MFMA-busy fraction of the Gram kernel from rocprofv3 PMC passes.

usage: python tools/pmc_clock.py PMC_DIR [kernel-substring]
Reads *counter_collection.csv (GRBM_GUI_ACTIVE, SQ_VALU_MFMA_BUSY_CYCLES, SQ_BUSY_CYCLES ...) and
*kernel_trace.csv of the same pass. Effective clock = GRBM_GUI_ACTIVE / 8 XCDs / wall
(MI355X_MICROARCH.md 'DVFS give-back'); the counters are summed per dispatch and averaged.
"""
import csv
import glob
import os
import sys


def main():
    d = sys.argv[1]
    sub = sys.argv[2] if len(sys.argv) > 2 else "ob_gram"
    per = {}
    for path in glob.glob(os.path.join(d, "**", "*counter_collection.csv"), recursive=True):
        for row in csv.DictReader(open(path)):
            if sub not in row.get("Kernel_Name", ""):
                continue
            key = row.get("Dispatch_Id") or row.get("Correlation_Id")
            c = per.setdefault(key, {})
            c[row["Counter_Name"]] = c.get(row["Counter_Name"], 0.0) + float(row["Counter_Value"])
    dur = {}
    for path in glob.glob(os.path.join(d, "**", "*kernel_trace.csv"), recursive=True):
        for row in csv.DictReader(open(path)):
            if sub in row.get("Kernel_Name", ""):
                dur[row.get("Dispatch_Id") or row.get("Correlation_Id")] = (
                    float(row["End_Timestamp"]) - float(row["Start_Timestamp"])) * 1e-9
    for key in sorted(per, key=lambda k: int(k)):
        c = per[key]
        t = dur.get(key)
        line = f"dispatch {key}: " + " ".join(f"{k}={v:.4g}" for k, v in sorted(c.items()))
        if t:
            line += f" wall_ms={t * 1e3:.2f}"
            if "GRBM_GUI_ACTIVE" in c:
                clk = c["GRBM_GUI_ACTIVE"] / 8 / t
                line += f" clock_GHz={clk / 1e9:.3f}"
                if "SQ_VALU_MFMA_BUSY_CYCLES" in c:
                    line += f" mfma_busy/(clk*wall*1024 SIMD)={c['SQ_VALU_MFMA_BUSY_CYCLES'] / (clk * t * 1024):.3f}"
        print(line)


if __name__ == "__main__":
    main()
