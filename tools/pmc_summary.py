"""Summarize rocprofv3 --pmc CSVs for ob_gram_kernel into profiles/pmc_gram.json.

FETCH_SIZE and WRITE_SIZE are collected in separate passes (they do not fit one pass on gfx950)
and are in KiB; on gfx950 FETCH_SIZE reports half the bytes of a wide coalesced streaming read
(MI355X_MICROARCH.md §HBM), so the read side is doubled before use.
usage: python tools/pmc_summary.py FETCH_DIR WRITE_DIR ROWS PREDS REPS OUT_JSON [KERNEL]
"""
import csv
import glob
import json
import os
import sys


def per_dispatch(d, counter, kernel):
    vals = {}
    for path in glob.glob(os.path.join(d, "**", "*counter_collection.csv"), recursive=True):
        for row in csv.DictReader(open(path)):
            if kernel not in row.get("Kernel_Name", ""):
                continue
            if row.get("Counter_Name") != counter:
                continue
            key = row.get("Dispatch_Id") or row.get("Correlation_Id")
            vals[key] = vals.get(key, 0.0) + float(row["Counter_Value"])
    return list(vals.values())


def main():
    fdir, wdir, rows, preds, reps, out = sys.argv[1:7]
    kernel = sys.argv[7] if len(sys.argv) > 7 else "ob_gram_kernel"
    f = per_dispatch(fdir, "FETCH_SIZE", kernel)
    w = per_dispatch(wdir, "WRITE_SIZE", kernel)
    fk = sum(f) / max(len(f), 1)
    wk = sum(w) / max(len(w), 1)
    res = {"kernel": kernel, "rows": int(rows), "preds": int(preds), "reps": int(reps),
           "dispatches": [len(f), len(w)], "FETCH_SIZE_KiB": fk, "WRITE_SIZE_KiB": wk,
           "hbm_bytes_per_launch": (2.0 * fk + wk) * 1024.0,
           "note": "read side = 2 x FETCH_SIZE (gfx950 correction), write side = WRITE_SIZE; KiB -> bytes"}
    json.dump(res, open(out, "w"), indent=1)
    print(json.dumps(res))


if __name__ == "__main__":
    main()
