"""Machado-Mata reduced vs unreduced solve at configs[4]'s size, fit by fit (diagnostic).

For the point pass and replicates 0, 1 of a 500k x 15 panel with 1,000 simulations: the fits'
convergence flags on both paths, the largest coefficient difference, and for the fits that differ
most the objective sum_i c_i rho_tau(y_i - x_i beta) of both betas on the pass's counts.
    python tools/mm_diag_r5.py [n] [sims]
"""
import importlib
import os
import sys

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
sys.path.insert(0, os.path.join(ROOT, "tests"))
sys.path.insert(0, os.path.join(ROOT, "oracle"))
ob = importlib.import_module("oaxaca-blinder-rs_amd")
import oracle as O  # noqa: E402  (test infrastructure: the MM-1 taus)
from test_gpu_mm import mm_data  # noqa: E402

SEED = 0x0B5EED
n = int(sys.argv[1]) if len(sys.argv) > 1 else 500_000
sims = int(sys.argv[2]) if len(sys.argv) > 2 else 1000
d = mm_data(n, 15, seed=45)
panel = ob.Panel(d["xa"], d["ya"], d["xb"], d["yb"])
X = [np.hstack([np.ones((len(d["ya"]), 1)), d["xa"]]), np.hstack([np.ones((len(d["yb"]), 1)), d["xb"]])]
Y = [d["ya"], d["yb"]]
for rep in (0xFFFFFFFF, 0, 1):
    br, dr = panel.debug_mm_betas(SEED, sims, rep)
    with ob._native.option("mm_reduce", 0):
        bf, df = panel.debug_mm_betas(SEED, sims, rep)
    print(f"rep {rep:#x}: reduced not converged {int(dr.size - dr.sum())}, full not converged {int(df.size - df.sum())}")
    for g in (0, 1):
        bad = np.flatnonzero(dr[g] != df[g])
        if bad.size:
            print(f"  group {g}: convergence differs at sims {bad[:20].tolist()} taus "
                  f"{[round(O.mm_tau(SEED, rep, int(s)), 5) for s in bad[:20]]} reduced {dr[g][bad[:20]].tolist()}")
        both = (dr[g] == 1) & (df[g] == 1)
        diff = np.abs(br[g] - bf[g]).max(axis=1)
        diff[~both] = 0
        order = np.argsort(-diff)[:5]
        if rep == 0xFFFFFFFF:
            c = np.ones(len(Y[g]))
        else:
            _, rc = panel.debug_counts(SEED, rep, 1, g)
            c = rc[0].astype(float)
        for s in order:
            tau = O.mm_tau(SEED, rep, int(s))
            obj = []
            for b in (br[g][s], bf[g][s]):
                r = Y[g] - X[g] @ b
                obj.append(float(np.sum(c * np.where(r >= 0, tau * r, (tau - 1.0) * r))))
            print(f"  group {g} sim {s} tau {tau:.5f}: max |dbeta| {diff[s]:.3e}, objective reduced {obj[0]:.12e} "
                  f"full {obj[1]:.12e} (rel {(obj[0] - obj[1]) / abs(obj[1]):.2e})")
panel.close()
