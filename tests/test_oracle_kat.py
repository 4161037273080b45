"""Pins the oracle (CPU restatement) to every known-answer test the reference holds for the
bootstrap path, plus an exact rational cross-check of its OLS. CPU only."""
import json
import os
from fractions import Fraction

import numpy as np
import pytest

KAT = json.load(open(os.path.join(os.path.dirname(__file__), "golden", "reference_kat.json")))


def test_philox_random123_vectors(O):
    for ctr, key, want in KAT["philox4x32_10"]["cases"]:
        assert O.philox(ctr, key) == want


def test_ols_simple(O):  # ols.rs:151-162
    k = KAT["ols_simple"]
    rc, beta, _ = O.ols(np.array(k["y"], float), np.array(k["x"], float))
    assert rc == O.ORC_OK
    assert np.allclose(beta, k["beta"], atol=k["tol"], rtol=0)


def test_ols_singular(O):  # ols.rs:164-181
    k = KAT["ols_singular"]
    rc, _, _ = O.ols(np.array(k["y"], float), np.array(k["x"], float))
    assert rc == O.ORC_E_CHOLESKY


def test_ols_insufficient(O):  # ols.rs:183-209
    k = KAT["ols_insufficient"]
    rc, _, _ = O.ols(np.array(k["y"], float), np.array(k["x"], float))
    assert rc == O.ORC_E_INSUFFICIENT


def test_ols_negative_weight(O):  # ols.rs:60-66
    x = np.array([[1, 0], [1, 1], [1, 2.0]])
    rc, _, _ = O.ols(np.array([1, 2, 3.0]), x, np.array([1.0, -1.0, 1.0]))
    assert rc == O.ORC_E_NEGWEIGHT


def _exact_ols(x, y, w=None):
    """Normal equations in exact rationals (independent of the oracle's float Cholesky)."""
    n, k = len(x), len(x[0])
    w = w or [1] * n
    A = [[sum(Fraction(w[i]) * Fraction(x[i][a]) * Fraction(x[i][b]) for i in range(n)) for b in range(k)]
         for a in range(k)]
    rhs = [sum(Fraction(w[i]) * Fraction(x[i][a]) * Fraction(y[i]) for i in range(n)) for a in range(k)]
    for c in range(k):  # Gauss-Jordan
        piv = next(r for r in range(c, k) if A[r][c] != 0)
        A[c], A[piv], rhs[c], rhs[piv] = A[piv], A[c], rhs[piv], rhs[c]
        for r in range(k):
            if r != c and A[r][c] != 0:
                f = A[r][c] / A[c][c]
                A[r] = [A[r][j] - f * A[c][j] for j in range(k)]
                rhs[r] -= f * rhs[c]
    return [float(rhs[i] / A[i][i]) for i in range(k)]


def test_ols_matches_exact_rationals(O):
    rng = np.random.default_rng(3)
    x = np.column_stack([np.ones(40), rng.integers(0, 20, 40), rng.integers(-5, 5, 40)]).astype(float)
    y = rng.integers(0, 100, 40).astype(float)
    w = rng.integers(1, 4, 40).astype(float)
    for weights in (None, w):
        rc, beta, _ = O.ols(y, x, weights)
        exact = _exact_ols(x.tolist(), y.tolist(), None if weights is None else weights.tolist())
        assert rc == 0
        assert np.allclose(beta, exact, rtol=1e-12, atol=1e-12)


def _pass(O, xa, ya, xb, yb, ref, norm=None, n_num=None, weights=(None, None)):
    k = xa.shape[1]
    cfg = O.PassConfig(k, k - 1 if n_num is None else n_num, ref, weights[0] is not None, norm)
    rc, row = O.single_pass(cfg, xa, ya, weights[0], xb, yb, weights[1])
    assert rc == 0
    return cfg, row


def _exact_groups():
    # group A: x mean 5, y = 2 + 4x exactly; group B: x mean 3, y = 1 + 3x exactly (decomposition.rs:131-134)
    xa = np.array([[1, 4], [1, 5], [1, 6.0]])
    xb = np.array([[1, 2], [1, 3], [1, 4.0]])
    return xa, 2 + 4 * xa[:, 1], xb, 1 + 3 * xb[:, 1]


def test_three_fold_kat(O):  # decomposition.rs:129-139
    k = KAT["three_fold"]
    xa, ya, xb, yb = _exact_groups()
    _, row = _pass(O, xa, ya, xb, yb, O.REF["group_b"])
    assert abs(row[2] - k["endowments"]) < k["tol"]
    assert abs(row[3] - k["coefficients"]) < k["tol"]
    assert abs(row[4] - k["interaction"]) < k["tol"]


@pytest.mark.parametrize("ref", ["group_b", "group_a"])
def test_detailed_sums_kat(O, ref):  # decomposition.rs:141-184
    xa, ya, xb, yb = _exact_groups()
    cfg, row = _pass(O, xa, ya, xb, yb, O.REF[ref])
    kd = cfg.k + cfg.n_base
    assert abs(row[6:6 + kd].sum() - row[0]) < 1e-9
    assert abs(row[6 + kd:6 + 2 * kd].sum() - row[1]) < 1e-9


def test_p_values_kat(O):  # inference.rs:40-57
    for vals, p in KAT["p_values"]["cases"]:
        assert abs(O.bootstrap_stats(vals)[1] - p) < 1e-9


def test_bootstrap_stats_conventions(O):  # inference.rs:4-34
    se, p, (lo, hi) = O.bootstrap_stats([])
    assert np.isnan(se) and np.isnan(p) and np.isnan(lo) and np.isnan(hi)
    v = np.arange(100.0)
    se, p, (lo, hi) = O.bootstrap_stats(v[::-1])
    assert abs(se - np.std(v, ddof=1)) < 1e-12
    assert lo == 2.0 and hi == 97.0  # floor(0.025 n), floor(0.975 n)
    _, _, (lo, hi) = O.bootstrap_stats([3.0])
    assert lo == 3.0 and hi == 3.0


def test_normalization_kat(O):  # normalization.rs:58-111
    # both groups: y = 10 + 2 [B] + 4 [C] exactly -> beta = [10, 2, 4] -> normalized [12, 0, 2]
    lv = np.array([0, 1, 2, 0, 1, 2, 0, 1, 2])
    x = np.column_stack([np.ones(9), lv == 1, lv == 2]).astype(float)
    y = 10 + 2 * x[:, 1] + 4 * x[:, 2]
    norm = {"start": [0, 2], "idx": [1, 2], "m": [3], "pstart": [0, 2], "pidx": [2, 3], "has_base": [1]}
    cfg, row = _pass(O, x, y, x, y, O.REF["group_a"], norm=norm, n_num=0)
    k, kd = cfg.k, cfg.k + cfg.n_base
    beta_a = row[6 + 2 * kd: 6 + 2 * kd + k]
    assert np.allclose(beta_a, KAT["normalization"]["expected"], atol=1e-9)


def _frame(d, keys):
    return {k: d[k] for k in keys}


@pytest.mark.parametrize("mode", [1, 0, 2, 3])
def test_integration_runs(O, mode):  # tests/integration_test.rs:105-144
    k = KAT["integration_frame"]
    ob = O.OracleBuilder(_frame(k, ["wage", "education", "gender"]), "wage", "gender", "F")
    ob.set(predictors=["education"], reps=5, ref_mode=mode)
    r = ob.run(threads=2)
    assert abs(r["total_gap"] - 10.0) < 1e-9
    agg = {c["name"]: c["estimate"] for c in r["two_fold"]["aggregate"]}
    assert abs(agg["explained"] + agg["unexplained"] - r["total_gap"]) < 1e-9
    assert r["n_a"] == 10 and r["n_b"] == 10


def test_integration_categorical_normalize(O):  # tests/integration_test.rs:146-163
    k = KAT["integration_categorical"]
    ob = O.OracleBuilder(_frame(k, ["wage", "education", "gender", "union"]), "wage", "gender", "F")
    ob.set(predictors=["education"], categorical=["union"], normalize=["union"], reps=5)
    r = ob.run(threads=2)
    agg = {c["name"]: c["estimate"] for c in r["two_fold"]["aggregate"]}
    assert abs(r["total_gap"] - 10.0) < 1e-9
    assert abs(agg["explained"] + agg["unexplained"] - r["total_gap"]) < 1e-9
    names = [c["name"] for c in r["two_fold"]["detailed_explained"]]
    assert names == ["__ob_intercept__", "education", "union_union", "union_union_plus", "union_none"]


def test_weights_kat(O):  # tests/weights_test.rs
    k = KAT["weights"]
    fr = _frame(k, ["outcome", "group", "weight", "x"])
    ob = O.OracleBuilder(fr, "outcome", "group", "B").set(predictors=["x"], reps=0)
    assert abs(ob.run()["total_gap"] - k["gap_unweighted"]) < k["tol"]
    ob = O.OracleBuilder(fr, "outcome", "group", "B").set(predictors=["x"], reps=0, weights="weight")
    assert abs(ob.run()["total_gap"] - k["gap_weighted"]) < k["tol"]


def test_null_handling_kat(O):  # tests/null_handling_test.rs
    k = KAT["nulls"]
    ob = O.OracleBuilder(_frame(k, ["outcome", "group", "education"]), "outcome", "group", "B")
    ob.set(predictors=["education"], reps=20)
    # each group: 3 rows, K = 2 -> the point estimate is solvable; gap = 11 - 16
    r = ob.run(threads=2)
    assert r["n_a"] == 3 and r["n_b"] == 3


def test_rif_kat(O):  # tests/rif_test.rs
    k = KAT["rif"]
    ob = O.OracleBuilder(_frame(k, ["wage", "group", "education"]), "wage", "group", "F")
    ob.set(predictors=["education"], reps=10)
    assert ob.decompose_quantile(0.9, threads=2)["total_gap"] > 0.0


def test_budget_gap_kat(O):  # tests/optimize_budget_test.rs:34
    k = KAT["budget"]
    ob = O.OracleBuilder(_frame(k, ["wage", "education", "group"]), "wage", "group", "B")
    ob.set(predictors=["education"], reps=0)
    r = ob.run()
    assert abs(r["total_gap"] - 16.0) < 1e-9
    assert sorted(np.round(r["residuals"], 9).tolist()) == [-5, -5, 0, 0, 5, 5]


@pytest.mark.parametrize("mode", [3, 2])
def test_reference_groups_kat(O, mode):  # tests/features_test.rs:14-35 (Cotton, Neumark)
    k = KAT["reference_groups"]
    ob = O.OracleBuilder(_frame(k, ["wage", "education", "experience", "gender"]), "wage", "gender", "F")
    ob.set(predictors=["education", "experience"], reps=20, ref_mode=mode)
    assert ob.run(threads=2)["total_gap"] > 0.0


@pytest.mark.parametrize("c", [1, 100, 128, 129, 777, 4095, 4096, 4097, 9000, 70001, 500000])
def test_obrs2_split_is_binomial(O, c):
    """OBRS-2's level-1 split (popcount below 4096 draws; from 4096 up Knuth-Yao B(2^j, 1/2)
    samples over the binary digits of c plus a popcount of c & 127 bits): Binomial(c, 1/2) in law
    -- chi-square over central quantile bins, mean and variance within 5 standard errors."""
    from scipy import stats

    n = 6000 if c < 100_000 else 2000
    xs = np.array([O.binomial_half(c, 0xB17, r, 1, 5) for r in range(n)], dtype=float)
    assert xs.min() >= 0 and xs.max() <= c
    assert abs(xs.mean() - c / 2) < 5 * np.sqrt(c / 4 / n)
    assert abs(xs.var() - c / 4) < 5 * (c / 4) * np.sqrt(2.0 / n) + 1e-9
    if c >= 100:
        edges = np.unique(np.round(stats.binom.ppf(np.linspace(0.002, 0.998, 21), c, 0.5)))
        edges = np.concatenate([[-1.0], edges, [float(c)]])
        obs = np.histogram(xs, bins=edges + 0.5)[0]
        exp = np.diff(stats.binom.cdf(edges, c, 0.5)) * n
        keep = exp > 5
        chi2 = ((obs[keep] - exp[keep]) ** 2 / exp[keep]).sum()
        assert stats.chi2.sf(chi2, keep.sum() - 1) > 1e-4, chi2


def test_resample_is_multinomial(O):
    """OBRS-3 draws: exact count n per replicate and a uniform per-row law (chi-square)."""
    n = 1500
    tot = np.zeros(n)
    for rep in range(200):
        idx = O.resample_indices(0xABC, rep, 1, n)
        assert len(idx) == n and idx.max() < n
        tot += np.bincount(idx, minlength=n)
    exp = 200.0
    chi2 = ((tot - exp) ** 2 / exp).sum()
    assert abs(chi2 - (n - 1)) < 6 * np.sqrt(2 * (n - 1))
    m = O.level1_counts(0xABC, 7, 0, 100_000)
    assert m.sum() == 100_000 and len(m) == (100_000 + 255) // 256
    # the binomial tree's shape edges: one tile, exact powers of two, 257 tiles with a 1-row tail
    for n in (1, 3, 255, 256, 257, 512, 65536, 65537, 131372):
        for rep in range(3):
            m = O.level1_counts(0x5EED, rep, 1, n)
            assert m.sum() == n and len(m) == (n + 255) // 256
    tail = np.array([O.level1_counts(0x5EED, rep, 0, 257)[-1] for rep in range(400)])
    assert abs(tail.mean() - 1.0) < 0.25  # a 1-row tail tile: E m = 257 / 257
    # tile counts of a 2M-row group (splits of ~2M, 1M, ... draws): each ~ Binomial(n, 1/T)
    n, reps = 2_000_003, 40
    ms = np.array([O.level1_counts(0x5EED, rep, 0, n) for rep in range(reps)], dtype=float)
    t = ms.shape[1]
    p = np.full(t, 256.0 / n)
    p[-1] = (n - 256 * (t - 1)) / n
    z = (ms.sum(0) - reps * n * p) / np.sqrt(reps * n * p * (1 - p))
    assert abs(z.mean()) < 6 / np.sqrt(t) and abs(z.var() - 1.0) < 0.1


# --- Heckman two-step (heckman.rs, estimation.rs:114-260, math/probit.rs) ---------------------
def test_probit_basic_convergence_kat(O):  # math/probit.rs:179-213
    y = np.array([0.0, 1.0, 0.0, 1.0, 0.0, 1.0])
    x = np.column_stack([np.ones(6), [-1.5, -0.5, 0.0, 0.5, 1.0, 1.5]])
    r = O.probit(y, x, 100, 1e-6, full=True)
    assert r["converged"] and r["iterations"] > 0 and len(r["coefficients"]) == 2
    assert r["coefficients"][1] > 0.0


def test_probit_non_convergence_kat(O):  # math/probit.rs:215-228
    y = np.array([0.0, 0.0, 1.0, 1.0])
    x = np.column_stack([np.ones(4), [-1.0, -0.5, 0.5, 1.0]])
    r = O.probit(y, x, 1, 1e-15, full=True)
    assert not r["converged"] and r["iterations"] == 1


def test_probit_recovers_latent_index(O):
    """A well-posed probit (n = 20000, index 0.3 + 0.8 z): Fisher scoring recovers it."""
    rng = np.random.default_rng(5)
    z = rng.normal(size=20000)
    s = (0.3 + 0.8 * z + rng.normal(size=z.size) > 0).astype(float)
    r = O.probit(s, np.column_stack([np.ones_like(z), z]), full=True)
    assert r["converged"] and np.allclose(r["coefficients"], [0.3, 0.8], atol=0.05)


def heckman_frame(n=2000, seed=42, null_unselected=True):
    """tests/heckman_test.rs's recipe (z, x = z + 0.5 e, corr(u, e) = 0.8, s = [0.5 z + u > 0],
    y = 1 + 2x + e, group A/B at random) with numpy draws in place of rand's StdRng."""
    rng = np.random.default_rng(seed)
    z = rng.normal(size=n)
    x = z + 0.5 * rng.normal(size=n)
    u, e0 = rng.normal(size=n), rng.normal(size=n)
    e = 0.8 * u + np.sqrt(1 - 0.64) * e0
    s = (0.5 * z + u > 0).astype(float)
    y = 1.0 + 2.0 * x + e
    grp = np.where(rng.random(n) < 0.5, "A", "B")
    out = [float(v) if (si == 1.0 or not null_unselected) else None for v, si in zip(y, s)]
    return {"outcome": out, "x": x.tolist(), "z": z.tolist(), "selection": s.tolist(), "group": grp.tolist()}


def test_heckman_imr_in_detailed_kat(O):  # tests/heckman_test.rs:55-66
    ob = O.OracleBuilder(heckman_frame(), "outcome", "group", "B").set(predictors=["x"], reps=0)
    r = ob.heckman("selection", ["z"]).run()
    assert any(c["name"] == "IMR" for c in r["two_fold"]["detailed_explained"])
    # the reference drops null outcomes before the probit (builder.rs:760-784): every s is 1
    assert len(r["residuals"]) == r["n_b"]


def _two_step_by_hand(O, fr, grp):
    """heckman.rs:38-108 written out with numpy lstsq for one group of a frame."""
    g = np.array(fr["group"]) == grp
    s, x, y, z = (np.array(fr[c]) for c in ("selection", "x", "outcome", "z"))
    gam = O.probit(s[g], np.column_stack([np.ones(g.sum()), z[g]]))
    sel = g & (s == 1)
    zg = gam[0] + gam[1] * z[sel]
    imr = O._npdf(zg) / O._ncdf(zg)
    coef = np.linalg.lstsq(np.column_stack([np.ones(sel.sum()), x[sel], imr]), y[sel], rcond=None)[0]
    return gam, coef, np.array([1.0, x[sel].mean(), imr.mean()])


@pytest.mark.parametrize("ref_mode", [0, 1, 3])
def test_heckman_two_step_consistency(O, ref_mode):
    """Outcomes present on unselected rows: the builder's means equal the two steps written out
    by hand, explained + unexplained = xa.ba - xb.bb, and the intercept's selection term is 0
    (builder.rs:510-530)."""
    fr = heckman_frame(null_unselected=False)
    ob = O.OracleBuilder(fr, "outcome", "group", "B").set(predictors=["x"], reps=8, ref_mode=ref_mode)
    r = ob.heckman("selection", ["z"]).run()
    assert r["n_failed"] == 0 and r["rows"].shape == (8, O.heckman_row_len(2, 2))
    gam_a, ba, xa = _two_step_by_hand(O, fr, "A")
    _, bb, xb = _two_step_by_hand(O, fr, "B")
    assert gam_a[1] > 0.2
    assert np.allclose(r["xa_mean"], xa, rtol=1e-12) and np.allclose(r["xb_mean"], xb, rtol=1e-12)
    est = {c["name"]: c["estimate"] for c in r["two_fold"]["aggregate"]}
    assert abs(est["explained"] + est["unexplained"] - (xa @ ba - xb @ bb)) < 1e-8
    assert {c["name"] for c in r["two_fold"]["detailed_explained"]} == {"__ob_intercept__", "x", "IMR"}
    sel = r["two_fold"]["detailed_selection"]
    assert [c["name"] for c in sel] == ["__ob_intercept__", "z"] and sel[0]["estimate"] == 0.0


def test_heckman_pooled_unsupported(O):  # builder.rs:500-507 panics: beta_star lacks the IMR entry
    ob = O.OracleBuilder(heckman_frame(null_unselected=False), "outcome", "group", "B").set(predictors=["x"], reps=0,
                                                                                             ref_mode=2)
    with pytest.raises(O.OracleError):
        ob.heckman("selection", ["z"]).run()


# --- Machado-Mata (quantile_decomposition.rs, math/quantile_regression.rs) ------------------
@pytest.mark.parametrize("tau", [0.5, 0.25])
def test_qr_linear_data_kat(O, tau):  # quantile_regression.rs:136-170 (tolerance 1e-4 there)
    y = np.array([1.0, 2.0, 3.0, 4.0, 5.0])
    x = np.column_stack([np.ones(5), [1.0, 2.0, 3.0, 4.0, 5.0]])
    b = O.qr_exact(x, y, np.ones(5, dtype=np.int64), tau)
    assert len(b) == 2 and abs(b[0]) < 1e-9 and abs(b[1] - 1.0) < 1e-9


def test_qr_counts_equal_duplicated_rows(O):
    """Counts c_i are the bootstrap's duplicated rows: the weighted LP equals the LP on the
    expanded sample."""
    rng = np.random.default_rng(0)
    x = np.column_stack([np.ones(40), rng.normal(size=40)])
    y = x @ [1.0, 2.0] + rng.standard_t(3, 40)
    c = rng.integers(0, 3, 40)
    idx = np.repeat(np.arange(40), c)
    b1 = O.qr_exact(x, y, c, 0.3)
    b2 = O.qr_exact(x[idx], y[idx], np.ones(len(idx), dtype=np.int64), 0.3)
    assert np.allclose(b1, b2, atol=1e-9)


def test_mm_integration_kat(O):  # tests/integration_test.rs:165-198
    f = {"wage": [10.0, 12.0, 11.0, 13.0, 15.0, 20.0, 22.0, 21.0, 23.0, 25.0, 9.0, 18.0],
         "education": [12.0, 16.0, 14.0, 16.0, 18.0, 12.0, 16.0, 14.0, 16.0, 18.0, 10.0, 20.0],
         "gender": ["F"] * 6 + ["M"] * 6}
    r = O.OracleQuantileDecomposition(f, "wage", "gender", "F").set(["education"], quantiles=[0.25, 0.5, 0.75],
                                                                     simulations=10, reps=2).run()
    assert sorted(r["results_by_quantile"]) == ["q25", "q50", "q75"]
    for det in r["results_by_quantile"].values():
        gap, ch, co = (det[k]["estimate"] for k in ("Total Gap", "Characteristics", "Coefficients"))
        assert abs(ch + co - gap) < 1e-9


def test_mm1_draws(O):
    """MM-1: tau_s in [0.01, 0.99) with the uniform law; row picks exactly uniform (chi-square)."""
    taus = np.array([O.mm_tau(0xABC, 3, s) for s in range(4000)])
    assert taus.min() >= 0.01 and taus.max() < 0.99 and abs(taus.mean() - 0.5) < 0.02
    n = 37
    cnt = np.bincount([O.mm_pick(0xABC, 5, 1, i, n) for i in range(37 * 200)], minlength=n)
    chi2 = ((cnt - 200.0) ** 2 / 200.0).sum()
    assert abs(chi2 - (n - 1)) < 6 * np.sqrt(2 * (n - 1))
