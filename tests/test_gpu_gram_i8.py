"""The exact integer-sliced Gram (ob_gram_i8.hip) against the f64 MFMA Gram (ob_gram_kernel).

Both compute G_r = sum_i c_ri v_i v_i^T (v = sqrt(w) [1, x, y], ols.rs:68-78) for the same
OBRS-1 counts. The i8 path's only approximation is the 56-bit fixed-point split of each pair
product relative to its chunk's power of two (2^-57 of the chunk's largest |P| per row), so the
two Grams must agree to 1e-12 of the natural scale sqrt(G_aa G_bb) of every entry; and the rows
the engine returns (default path: i8) must equal the f64 path's rows to 1e-9 relative.
"""
import os

import numpy as np
import pytest

pytestmark = pytest.mark.gpu
SEED = 0x0B5EED


def _pairs(k1):
    return [(a, b) for a in range(k1) for b in range(a, k1)]


def _check_gram(g8, g64, k1):
    pairs = _pairs(k1)
    diag = [pairs.index((a, a)) for a in range(k1)]
    worst = 0.0
    for gi in range(2):
        d = np.abs(g64[:, gi, diag])  # [rep, k1]
        for e, (a, b) in enumerate(pairs):
            scale = np.sqrt(d[:, a] * d[:, b])
            err = np.abs(g8[:, gi, e] - g64[:, gi, e])
            ok = (err <= 1e-12 * scale) | (scale == 0)
            assert ok.all(), (gi, a, b, float((err / np.maximum(scale, 1e-300)).max()))
            worst = max(worst, float((err / np.maximum(scale, 1e-300))[scale > 0].max(initial=0.0)))
    return worst


@pytest.mark.parametrize("n,p,weighted,ny", [
    (777, 0, False, 1), (3000, 1, True, 1), (20001, 5, False, 1), (65537, 20, True, 1),
    (9000, 20, True, 3), (2600, 40, False, 1), (1, 2, True, 1), (300_000, 20, True, 1),
])
def test_i8_gram_equals_f64_gram(ob, O, n, p, weighted, ny):
    d = O.synthetic_panel(max(n, 4), p, weighted, seed=n + p)
    ya, yb = d["ya"], d["yb"]
    if ny > 1:
        ya = np.column_stack([ya] + [ya * (t + 2) - 3.0 for t in range(ny - 1)])
        yb = np.column_stack([yb] + [yb * (t + 2) - 3.0 for t in range(ny - 1)])
    panel = ob.Panel(d["xa"], ya, d["xb"], yb, d["wa"], d["wb"])
    try:
        reps = 300 if n < 100_000 else 70
        g64 = panel.debug_gram(SEED, 11, reps, path=1)
        g8 = panel.debug_gram(SEED, 11, reps, path=2)
        k1 = p + 1 + ny
        worst = _check_gram(g8, g64, k1)
        assert worst < 1e-12
        assert panel.timing()["gram_path"] == 2
    finally:
        panel.close()


def test_i8_rows_equal_f64_rows(ob, O):
    """Default (i8) rows vs OB_GRAM_PATH=f64 rows, all reference modes, with dummies."""
    d = O.synthetic_panel(12000, 6, True, seed=4)
    rng = np.random.default_rng(4)
    cat_a = rng.integers(0, 4, d["xa"].shape[0])
    cat_b = rng.integers(0, 4, d["xb"].shape[0])
    xa = np.column_stack([d["xa"]] + [(cat_a == j).astype(float) for j in (1, 2, 3)])
    xb = np.column_stack([d["xb"]] + [(cat_b == j).astype(float) for j in (1, 2, 3)])
    panel = ob.Panel(xa, d["ya"], xb, d["yb"], d["wa"], d["wb"], n_num=6)
    try:
        for ref in (0, 1, 2, 3):
            r8, ok8 = panel.boot(SEED, 0, 200, ref)
            assert panel.timing()["gram_path"] == 2
            os.environ["OB_GRAM_PATH"] = "f64"
            try:
                r64, ok64 = panel.boot(SEED, 0, 200, ref)
                assert panel.timing()["gram_path"] == 1
            finally:
                del os.environ["OB_GRAM_PATH"]
            assert np.array_equal(ok8, ok64)
            gap = np.abs(r64[:, 5:6])
            assert np.all(np.abs(r8 - r64) <= 1e-9 * np.maximum(np.abs(r64), gap)), ref
    finally:
        panel.close()
