"""Ablation timing of the Gram kernel at the bench shape (1M x 20 WLS panel).

OB_GRAM_DIAG bits (read once per process): 2 no MFMAs, 4 no sub-tile DMA.
Prints min/median of 5 runs.
"""
import importlib, os, statistics, sys
sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import bench
ob = importlib.import_module("oaxaca-blinder-rs_amd")
d = bench.synthetic(1_000_000, 20, True)
panel = ob.Panel(d["xa"], d["ya"], d["xb"], d["yb"], d["wa"], d["wb"])
reps = int(sys.argv[1]) if len(sys.argv) > 1 else 10000
g, l1, cn = [], [], []
for it in range(6):
    panel.boot(0xB5EED, 0, reps, 0)
    t = panel.timing()
    if it:
        g.append(t["gram_ms"])
        l1.append(t["level1_ms"])
        cn.append(t["counts_ms"])
gm = min(g)
print(f"diag={os.environ.get('OB_GRAM_DIAG', '0')} reps={reps} gram_ms min={gm:.2f} med={statistics.median(g):.2f} "
      f"level1_ms={min(l1):.2f} counts_ms={min(cn):.2f} TF={504e6 * reps / (gm * 1e-3) / 1e12:.1f}", flush=True)
