"""One Machado-Mata pass of replicate REP with the per-iteration trace (option mm_trace), unreduced or
reduced: python tools/mm_trace_rep.py REP REDUCE [n] [sims]  (diagnostic)"""
import importlib
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
sys.path.insert(0, os.path.join(ROOT, "tests"))
ob = importlib.import_module("oaxaca-blinder-rs_amd")
from test_gpu_mm import QS, mm_data  # noqa: E402

rep, red = int(sys.argv[1]), int(sys.argv[2])
n = int(sys.argv[3]) if len(sys.argv) > 3 else 500_000
sims = int(sys.argv[4]) if len(sys.argv) > 4 else 1000
d = mm_data(n, 15, seed=45)
panel = ob.Panel(d["xa"], d["ya"], d["xb"], d["yb"])
ob._native.set_option("mm_trace", 1)
ob._native.set_option("mm_reduce", red)
rows, ok = panel.mm(0x0B5EED, sims, QS, rep, 1, with_point=False)
print("ok", ok, "rows", rows)
panel.close()
