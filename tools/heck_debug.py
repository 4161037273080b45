"""Heckman debugging on the GPU: python tools/heck_debug.py {boot|point|swap}."""
import os
import sys

os.environ["OB_GRAM_DIAG"] = "8"
ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
sys.path.insert(0, os.path.join(ROOT, "tests"))
sys.path.insert(0, os.path.join(ROOT, "oracle"))
import importlib

import numpy as np

from test_gpu_heckman import heckman_frame

ob = importlib.import_module("oaxaca-blinder-rs_amd")
import oracle as O

np.set_printoptions(precision=6, linewidth=220)
f = heckman_frame(2000, seed=2000)
mode = sys.argv[1]
if mode == "swap":
    f = dict(f)
    f["group"] = ["B" if v == "A" else "A" for v in f["group"]]
if mode in ("boot", "swap"):
    b = ob.OaxacaBuilder(f, "outcome", "group", "B").predictors(["x"]).heckman_selection("selection", ["z"]).bootstrap_reps(8).seed(0x0B5EED)
    pr = b.prepare()
    rows, ok = pr.boot(0, 8)
    print(mode, "status", ok, "iters", pr.timing()["probit_iterations"])
    o = O.OracleBuilder(f, "outcome", "group", "B").set(["x"], reps=8, seed=0x0B5EED).heckman("selection", ["z"]).run()
    print("gpu rows[0]", rows[0])
    print("orc rows[0]", o["rows"][0])
    pr.close()
else:
    for ref in (0, 1):
        b2 = (ob.OaxacaBuilder(f, "outcome", "group", "B").predictors(["x"]).heckman_selection("selection", ["z"])
              .bootstrap_reps(0).reference_coefficients(ref))
        r = b2.run()
        o2 = O.OracleBuilder(f, "outcome", "group", "B").set(["x"], reps=0, ref_mode=ref).heckman("selection", ["z"]).run()
        print("ref", ref, "gpu beta_star", r.beta_star, "xb", r.xb_mean, "sel", [c.estimate for c in r.two_fold.detailed_selection])
        print("ref", ref, "orc beta_star", o2["beta_star"], "xb", o2["xb_mean"], "sel", [c["estimate"] for c in o2["two_fold"]["detailed_selection"]])
