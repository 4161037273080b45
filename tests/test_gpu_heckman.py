"""Heckman two-step on the MI355X engine (builder .heckman_selection) vs the oracle's restatement of
math/probit.rs, heckman.rs, estimation.rs:114-260 and builder.rs:477-534: replicate rows, results
tables, errors, shard invariance and per-replicate identities at a larger size."""
import numpy as np
import pytest

from test_gpu_parity import RTOL, SEED, close, compare_results

pytestmark = pytest.mark.gpu


def heckman_frame(n, seed=42, weighted=False, null_unselected=False):
    """Selection on z, z2 and x2 with corr(u, e) = 0.8 (tests/heckman_test.rs's design, widened)."""
    rng = np.random.default_rng(seed)
    z, z2 = rng.normal(size=n), rng.normal(size=n)
    x = z + 0.5 * rng.normal(size=n)
    x2 = rng.uniform(0.0, 3.0, n)
    u, e0 = rng.normal(size=n), rng.normal(size=n)
    e = 0.8 * u + 0.6 * e0
    grp = np.where(rng.random(n) < 0.5, "A", "B")
    s = (0.3 + 0.5 * z - 0.4 * z2 + 0.2 * x2 + 0.3 * (grp == "A") + u > 0).astype(float)
    y = 1.0 + 2.0 * x + 0.5 * x2 + 0.4 * (grp == "A") + e
    out = [None if (null_unselected and si != 1.0) else float(v) for v, si in zip(y, s)]
    f = {"outcome": out, "x": x.tolist(), "x2": x2.tolist(), "z": z.tolist(), "z2": z2.tolist(),
         "selection": s.tolist(), "group": grp.tolist()}
    if weighted:
        f["w"] = rng.uniform(0.5, 2.0, n).tolist()
    return f


def builders(ob, O, f, preds, zs, reps, ref, weighted):
    b = (ob.OaxacaBuilder(f, "outcome", "group", "B").predictors(preds).heckman_selection("selection", zs)
         .bootstrap_reps(reps).reference_coefficients(ref).seed(SEED))
    o = O.OracleBuilder(f, "outcome", "group", "B").set(preds, reps=reps, ref_mode=ref, seed=SEED,
                                                         weights="w" if weighted else None)
    if weighted:
        b = b.weights("w")
    return b, o.heckman("selection", zs)


CASES = [  # (rows, predictors, selection predictors, ref, weighted)
    (2000, ["x"], ["z"], 0, False),
    (3000, ["x", "x2"], ["z", "z2"], 1, True),
    (2500, ["x", "x2"], ["z", "z2", "x2"], 3, False),
    (4000, ["x"], ["z", "z2", "x2"], 4, True),
    (1200, [], ["z"], 1, False),
]


@pytest.mark.parametrize("n,preds,zs,ref,weighted", CASES)
def test_heckman_rows_match_oracle(ob, O, n, preds, zs, ref, weighted):
    f = heckman_frame(n, seed=n, weighted=weighted)
    b, o = builders(ob, O, f, preds, zs, 64, ref, weighted)
    want = o.run()
    pr = b.prepare()
    try:
        rows, ok = pr.boot(0, 64)
    finally:
        pr.close()
    assert rows.shape == want["rows"].shape == (64, O.heckman_row_len(len(preds) + 1, len(zs) + 1))
    assert (ok.astype(bool) == want["ok"].astype(bool)).all()
    good, (worst) = close(rows[ok.astype(bool)], want["rows"][want["ok"].astype(bool)], want["total_gap"])
    assert good, worst


@pytest.mark.parametrize("n,preds,zs,ref,weighted", CASES[:3])
def test_heckman_results_match_oracle(ob, O, n, preds, zs, ref, weighted):
    f = heckman_frame(n, seed=n + 1, weighted=weighted)
    b, o = builders(ob, O, f, preds, zs, 100, ref, weighted)
    r, want = b.run(), o.run()
    compare_results(r, want)
    names = [c.name for c in r.two_fold.detailed_explained]
    assert names[-1] == "IMR" and names == [c["name"] for c in want["two_fold"]["detailed_explained"]]
    got, exp = r.two_fold.detailed_selection, want["two_fold"]["detailed_selection"]
    assert [c.name for c in got] == ["__ob_intercept__"] + zs == [c["name"] for c in exp]
    scale = abs(want["total_gap"])
    for c, w in zip(got, exp):
        for fld in ("estimate", "std_err", "ci_lower", "ci_upper"):
            assert abs(getattr(c, fld) - w[fld]) <= RTOL * max(abs(w[fld]), scale), (c.name, fld)
    assert len(r.residuals) == len(want["residuals"]) and not np.any(r.residuals)


def test_heckman_reference_test_frame(ob, O):  # tests/heckman_test.rs:55-66
    """Outcome null on unselected rows: clean_dataframe drops them, so every s is 1 and the probit
    runs its 100 iterations without converging; the run still reports an IMR term."""
    f = heckman_frame(2000, null_unselected=True)
    r = (ob.OaxacaBuilder(f, "outcome", "group", "B").predictors(["x"]).heckman_selection("selection", ["z"])
         .bootstrap_reps(0).run())
    assert any(c.name == "IMR" for c in r.two_fold.detailed_explained)
    o = O.OracleBuilder(f, "outcome", "group", "B").set(["x"], reps=0).heckman("selection", ["z"]).run()
    assert r.n_a == o["n_a"] and r.n_b == o["n_b"] and len(r.residuals) == r.n_b
    assert abs(r.total_gap - o["total_gap"]) <= 1e-9 * max(1.0, abs(o["total_gap"]))


def test_heckman_errors(ob, N):
    f = heckman_frame(1500)
    with pytest.raises(N.OaxacaError) as e:  # builder.rs:547-589 panics for Pooled: refused up front
        ob.OaxacaBuilder(f, "outcome", "group", "B").predictors(["x"]).heckman_selection(
            "selection", ["z"]).reference_coefficients(2).bootstrap_reps(0).run()
    assert e.value.code == N.OB_E_UNSUPPORTED
    g = dict(f)
    g["selection"] = [0.0 if grp == "B" else s for grp, s in zip(f["group"], f["selection"])]
    with pytest.raises(N.OaxacaError) as e:  # estimation.rs:219-223
        ob.OaxacaBuilder(g, "outcome", "group", "B").predictors(["x"]).heckman_selection(
            "selection", ["z"]).bootstrap_reps(0).run()
    assert e.value.code == N.OB_E_GROUP and "No observed outcomes" in str(e.value)
    with pytest.raises(N.OaxacaError) as e:
        ob.OaxacaBuilder(f, "outcome", "group", "B").predictors(["x"]).heckman_selection(
            "selection", ["nope"]).bootstrap_reps(0).run()
    assert e.value.code == N.OB_E_COLUMN


def test_heckman_shard_invariant_and_deterministic(ob):
    f = heckman_frame(5000, seed=3)
    b = (ob.OaxacaBuilder(f, "outcome", "group", "B").predictors(["x", "x2"]).heckman_selection("selection", ["z", "z2"])
         .bootstrap_reps(300).seed(SEED))
    pr = b.prepare()
    try:
        r0, k0 = pr.boot(0, 300)
        r1, k1 = pr.boot(120, 180)
        r2, _ = pr.boot(0, 300)
    finally:
        pr.close()
    assert np.array_equal(r0, r2, equal_nan=True)
    assert np.array_equal(r0[120:], r1, equal_nan=True) and np.array_equal(k0[120:], k1)


def test_heckman_identities_at_size(ob):
    """200k rows, 512 replicates: per replicate explained + unexplained = xa.ba - xb.bb over the
    K + 1 terms (IMR included), the detailed terms sum to the aggregates, and the intercept's
    selection term is 0 (its selection mean is 1 in both groups)."""
    f = heckman_frame(200_000, seed=8, weighted=True)
    b = (ob.OaxacaBuilder(f, "outcome", "group", "B").predictors(["x", "x2"]).weights("w")
         .heckman_selection("selection", ["z", "z2", "x2"]).bootstrap_reps(512).reference_coefficients(0).seed(SEED))
    pr = b.prepare()
    try:
        rows, ok = pr.boot(0, 512)
        tm = pr.timing()
    finally:
        pr.close()
    assert ok.all() and tm["probit_iterations"] >= 3
    k1 = 4  # intercept, x, x2, IMR
    dex, dun = rows[:, 6:6 + k1], rows[:, 6 + k1:6 + 2 * k1]
    ba, bb, xa, xb = (rows[:, 6 + 2 * k1 + i * k1: 6 + 2 * k1 + (i + 1) * k1] for i in range(4))
    assert np.allclose(rows[:, 0] + rows[:, 1], (xa * ba).sum(1) - (xb * bb).sum(1), rtol=1e-9, atol=1e-12)
    assert np.allclose(dex.sum(1), rows[:, 0], rtol=1e-9, atol=1e-12)
    assert np.allclose(dun.sum(1), rows[:, 1], rtol=1e-9, atol=1e-12)
    sel = rows[:, 6 + 7 * k1:]
    assert sel.shape[1] == 4 and np.all(sel[:, 0] == 0.0)
    assert np.all(np.abs(ba[:, 1] - 2.0) < 0.1)  # the outcome slope on x survives selection


def test_normal_pdf_cdf_device(N):
    """npdf_ncdf (Cody's rational erfc sharing phi's exponential, the default in the
    probit and IMR kernels) on the device over z in [-40, 40], the three CALERF regions, the
    region edges (|x| = 0.46875, 4 with x = -z / sqrt 2) and the probit's clamp thresholds
    (Phi = 1e-10 near z = -6.36), against the standard library's erfc and exp: the cdf to 1e-13
    relative on |z| <= 12 (and within the exponent-rounding bound beyond), 1e-13 absolute
    everywhere, the pdf to 1e-14 relative plus the same tail bound."""
    import ctypes as C
    import math

    edges = [s * e * math.sqrt(2.0) for e in (0.46875, 4.0) for s in (-1, 1)]
    z = np.concatenate([np.linspace(-40.0, 40.0, 80001), edges, np.nextafter(edges, np.inf),
                        np.nextafter(edges, -np.inf), [-6.361340902404056, -6.3613409024040557, -5.66, 5.66]])
    pdf, cdf = np.empty_like(z), np.empty_like(z)
    dp = C.POINTER(C.c_double)
    N.check(N.lib().ob_debug_normal(0, z.ctypes.data_as(dp), z.size, pdf.ctypes.data_as(dp), cdf.ctypes.data_as(dp)))
    want_cdf = np.array([0.5 * math.erfc(-v / math.sqrt(2.0)) for v in z])
    want_pdf = np.array([math.exp(-0.5 * v * v) / math.sqrt(2.0 * math.pi) for v in z])
    # exp(-z^2 / 2) carries the rounding of z^2 / 2 into its exponent: |z|^2 eps relative error in
    # both implementations, so far in the tail the bound grows with z^2 (and stays below 1e-13 on
    # |z| <= 12, where the clamped probabilities of the probit live)
    tol = 1e-13 + 8.0 * z * z * 2.2e-16
    big = want_cdf > 1e-300
    rel = np.abs(cdf[big] - want_cdf[big]) / want_cdf[big]
    assert np.all(rel <= tol[big]), (rel.max(), z[big][np.argmax(rel - tol[big])])
    assert np.all(rel[np.abs(z[big]) <= 12.0] <= 1e-13)
    assert np.all(np.abs(cdf - want_cdf) <= 1e-13)
    assert np.all(cdf[~big] <= 1e-300)
    relp = np.abs(pdf - want_pdf) / np.maximum(want_pdf, 1e-300)
    live = want_pdf > 1e-300
    assert np.all(relp[live] <= 1e-14 + tol[live] - 1e-13), relp.max()
    assert np.all((cdf >= 0.0) & (cdf <= 1.0)) and np.all(np.diff(cdf[:80001]) >= 0.0)


@pytest.mark.parametrize("n,preds,zs,ref,weighted", CASES[1:2])
def test_heckman_rows_match_oracle_library_erfc(ob, O, N, n, preds, zs, ref, weighted):
    """The same parity under option hk_erfc = 0 (the library erfc beside a second exp)."""
    f = heckman_frame(n, seed=n, weighted=weighted)
    b, o = builders(ob, O, f, preds, zs, 64, ref, weighted)
    want = o.run()
    with N.option("hk_erfc", 0):
        pr = b.prepare()
        try:
            rows, ok = pr.boot(0, 64)
        finally:
            pr.close()
    assert (ok.astype(bool) == want["ok"].astype(bool)).all()
    good, worst = close(rows[ok.astype(bool)], want["rows"][want["ok"].astype(bool)], want["total_gap"])
    assert good, worst
