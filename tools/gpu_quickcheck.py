"""Quick GPU parity + timing probe (development aid): engine rows vs the oracle on small panels,
then a timed 1M x 20 WLS boot. Run on the GPU box: python tools/gpu_quickcheck.py"""
import importlib
import os
import sys
import time

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
sys.path.insert(0, os.path.join(ROOT, "oracle"))
import oracle as O  # noqa: E402

ob = importlib.import_module("oaxaca-blinder-rs_amd")


def compare(n, p, weighted, ref, reps, seed=77):
    d = O.synthetic_panel(n, p, weighted, seed=seed)
    panel = ob.Panel(d["xa"], d["ya"], d["xb"], d["yb"], d["wa"], d["wb"])
    cfg = O.PassConfig(p + 1, p, ref, weighted)
    xa, xb = O.with_intercept(d["xa"]), O.with_intercept(d["xb"])
    rc, prow = O.single_pass(cfg, xa, d["ya"], d["wa"], xb, d["yb"], d["wb"])
    grow = panel.point_estimate(ref)
    pe = np.max(np.abs(grow - prow) / np.maximum(np.abs(prow), 1e-3))
    t0 = time.time()
    rows, ok = panel.boot(0xB5EED, 0, reps, ref)
    tg = time.time() - t0
    t0 = time.time()
    orow, ook = O.boot_ref(cfg, xa, d["ya"], d["wa"], xb, d["yb"], d["wb"], 0xB5EED, 0, reps, full=False)
    to = time.time() - t0
    okm = ok.astype(bool) & ook.astype(bool)
    be = np.max(np.abs(rows[okm] - orow[okm]) / np.maximum(np.abs(orow[okm]), 1e-3)) if okm.any() else -1
    print(f"n={n} p={p} w={weighted} ref={ref} reps={reps}: point rc={rc} maxrel={pe:.3e}; boot ok {ok.sum()}/{ook.sum()}"
          f" same={np.array_equal(ok, ook)} maxrel={be:.3e}; gpu {tg:.3f}s oracle {to:.3f}s", flush=True)
    return pe, be


if __name__ == "__main__":
    compare(2000, 3, False, 0, 64)
    compare(4000, 5, True, 1, 130)
    compare(3000, 20, True, 2, 100)
    compare(5000, 20, False, 3, 70)
    # timing at the bench shape
    d = O.synthetic_panel(1_000_000, 20, True)
    panel = ob.Panel(d["xa"], d["ya"], d["xb"], d["yb"], d["wa"], d["wb"])
    for reps in (256, 2048, 10000):
        t0 = time.time()
        rows, ok = panel.boot(0xB5EED, 0, reps, 0)
        dt = time.time() - t0
        t = panel.timing()
        print(f"1Mx20 WLS reps={reps}: {dt*1e3:.1f} ms wall, {reps/dt:.0f} reps/s, timing={t}", flush=True)
