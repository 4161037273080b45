"""Times Machado-Mata passes at configs[4]'s shape: python tools/mm_time.py ROWS PREDS SIMS REPS."""
import importlib
import os
import sys
import time

import numpy as np

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path.insert(0, os.path.join(os.path.dirname(os.path.dirname(os.path.abspath(__file__))), "tests"))
from test_gpu_mm import mm_data  # noqa: E402

ob = importlib.import_module("oaxaca-blinder-rs_amd")
rows, preds, sims, reps = (int(v) for v in sys.argv[1:5])
d = mm_data(rows, preds, seed=5)
panel = ob.Panel(d["xa"], d["ya"], d["xb"], d["yb"])
t0 = time.perf_counter()
r, ok = panel.mm(0x0B5EED, sims, [0.1, 0.25, 0.5, 0.75, 0.9], 0, 0, with_point=True)
t1 = time.perf_counter()
print(f"point pass: {t1 - t0:.3f} s ok={ok.tolist()}", flush=True)
r, ok = panel.mm(0x0B5EED, sims, [0.1, 0.25, 0.5, 0.75, 0.9], 0, reps, with_point=False)
t2 = time.perf_counter()
print(f"{reps} bootstrap passes: {t2 - t1:.3f} s ({(t2 - t1) / max(reps, 1):.3f} s/replicate) ok={ok.tolist()}")
print("q50 gap", r[:, 6])
