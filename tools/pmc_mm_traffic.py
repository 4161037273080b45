"""HBM bytes of the Machado-Mata IPM kernels over one `bench.py --mm` step, from two rocprofv3 PMC
passes (FETCH_SIZE, WRITE_SIZE: separate runs). The bench line of the FETCH pass gives the step's
live (fit, row) count, so the measured bytes per live fit-row sit beside the 48 B the assemble
pass's model counts.

Calibration (MI355X_MICROARCH.md: FETCH_SIZE halves 16-B-per-lane streaming reads; other widths
are uncalibrated). These kernels stream their state with 8-B-per-lane loads, 512 B a wave. The
affine pass reads exactly x, z, w of every live (fit, row) -- 24 B -- plus ~2 B of design rows and
lists; its FETCH_SIZE per live fit-row came out at 23.7 B (round 5), so for this access width
FETCH_SIZE counts the bytes themselves: read = FETCH_SIZE (x 2 would put 47 B through a pass that
can read at most ~26). Both readings are in the output.

usage: python tools/pmc_mm_traffic.py FETCH_DIR WRITE_DIR FETCH_PASS_BENCH_LOG > profiles/pmc_mm.json
"""
import csv
import glob
import json
import os
import sys

KERNELS = ("mm_assemble_mfma_kernel<16, true>", "mm_affine_kernel<16>", "mm_final_kernel<16>")


def per_kernel(d, counter):
    tot = {}
    for path in glob.glob(os.path.join(d, "**", "*counter_collection.csv"), recursive=True):
        for row in csv.DictReader(open(path)):
            if row["Counter_Name"] != counter:
                continue
            for k in KERNELS:
                if k in row.get("Kernel_Name", ""):
                    t = tot.setdefault(k, [0.0, set()])
                    t[0] += float(row["Counter_Value"])
                    t[1].add(row.get("Dispatch_Id") or row.get("Correlation_Id"))
    return {k: (v[0], len(v[1])) for k, v in tot.items()}


def main():
    fetch = per_kernel(sys.argv[1], "FETCH_SIZE")
    write = per_kernel(sys.argv[2], "WRITE_SIZE")
    line = None
    for ln in open(sys.argv[3]):
        if ln.startswith("{") and '"metric"' in ln:
            line = json.loads(ln)
    fit_rows = line["roofline"]["live_fit_rows"] if line else None
    out = {"workload": "configs[4] bench.py --mm, one step", "rows": line["config"]["rows"] if line else None,
           "predictors": line["config"]["predictors"] if line else None,
           "simulations": line["config"]["simulations"] if line else None,
           "replicates": line["config"]["replicates_per_gpu_per_step"] if line else None,
           "live_fit_rows": fit_rows, "kernels": {},
           "note": "hbm_bytes = FETCH_SIZE + WRITE_SIZE (8-B-per-lane reads, calibrated on the affine pass; "
                   "hbm_bytes_x2 applies the 16-B-per-lane correction instead), KiB -> bytes, summed over the "
                   "step's dispatches"}
    for k in KERNELS:
        f, nf = fetch.get(k, (0.0, 0))
        w, nw = write.get(k, (0.0, 0))
        b = (f + w) * 1024.0
        b2 = (2.0 * f + w) * 1024.0
        out["kernels"][k] = {"dispatches": [nf, nw], "FETCH_SIZE_KiB": f, "WRITE_SIZE_KiB": w, "hbm_bytes": b,
                             "bytes_per_live_fit_row": b / fit_rows if fit_rows else None, "hbm_bytes_x2": b2,
                             "bytes_per_live_fit_row_x2": b2 / fit_rows if fit_rows else None}
    print(json.dumps(out, indent=1))


if __name__ == "__main__":
    main()
