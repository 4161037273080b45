"""Full-size parity, the configs[0] CLI path, and the failure-mask rule for near-singular designs.

* configs[1] (1M rows x 20 predictors, WLS; GroupA and Pooled): SE / p / CI of every reported
  component over 256 replicates (inference.rs:4-34 over builder.rs:816-839's replicates) vs the
  oracle's reference algorithm on the same OBRS-3 stream, within 1e-6 (mixed tolerance).
* configs[0] (the CLI mean path, main.rs:161-232): a 10k-row x 5-predictor CSV written here,
  read back through ob.read_csv (the LazyCsvReader stand-in), OaxacaBuilder.run() with 200
  unweighted replicates vs OracleBuilder on an independent parse of the same file.
* Failure masks near singularity (ols.rs:107-111: the reference drops a replicate iff a
  Cholesky pivot is <= 0). Where the oracle's smallest pivot relative to its diagonal entry
  exceeds 1e-9, the sign of every pivot is decided well above both summation orders' rounding
  (f64 Gram error ~1e-13 relative), so the engine's ok mask and rows must equal the oracle's.
  Below that band the pivot is rounding noise in the reference too and its outcome is not a
  property of the data: there the engine must be deterministic and its ok rows finite.
"""
import csv
import hashlib
import json
import os

import numpy as np
import pytest

pytestmark = pytest.mark.gpu
SEED = 0x0B5EED
RTOL = 1e-6
BAND = 1e-9


def _threads():
    try:
        return max(1, int(os.environ.get("OMP_NUM_THREADS", "0"))) or len(os.sched_getaffinity(0))
    except ValueError:
        return len(os.sched_getaffinity(0))


def _stats_close(rows_e, ok_e, rows_o, ok_o, cols, gap_scale, ob, O):
    assert np.array_equal(ok_e, ok_o)
    st_e = ob.aggregate(rows_e, ok_e, np.asarray(cols, dtype=np.int32))
    m = ok_o.astype(bool)
    for j, c in enumerate(cols):
        se, p, (lo, hi) = O.bootstrap_stats(rows_o[m, c])
        for got, want in ((st_e[j, 0], se), (st_e[j, 2], lo), (st_e[j, 3], hi)):
            assert abs(got - want) <= RTOL * max(abs(want), gap_scale), (c, got, want)
        assert st_e[j, 1] == p, (c, st_e[j, 1], p)  # sign counts: exact


@pytest.mark.parametrize("ref", [0, 2])
def test_configs1_se_ci_p_match_oracle(ob, O, ref):
    d = O.synthetic_panel(1_000_000, 20, True)
    panel = ob.Panel(d["xa"], d["ya"], d["xb"], d["yb"], d["wa"], d["wb"])
    try:
        rows, ok = panel.boot(SEED, 0, 256, ref)
    finally:
        panel.close()
    cfg = O.PassConfig(21, 20, O.REF_FROM_ENUM[ref], True)
    xa, xb = O.with_intercept(d["xa"]), O.with_intercept(d["xb"])
    orows, ook = O.boot_ref(cfg, xa, d["ya"], d["wa"], xb, d["yb"], d["wb"], SEED, 0, 256, threads=_threads(),
                            full=False)
    gap = abs(float(np.nanmedian(orows[:, 5])))
    # every reported component: two-fold (2), three-fold (3), total gap, detailed (2 x 21)
    _stats_close(rows, ok, orows, ook, list(range(6 + 2 * 21)), gap, ob, O)
    scale = np.maximum(np.abs(orows), gap)
    assert np.all(np.abs(rows - orows) <= RTOL * scale)


def test_configs0_csv_cli_path(ob, O, tmp_path):
    """10k rows, P = 5, unweighted, 200 replicates (BASELINE configs[0]) through the CSV reader."""
    d = O.synthetic_panel(10_000, 5, False, seed=20260424)
    path = tmp_path / "wage.csv"
    names = [f"x{j + 1}" for j in range(5)]
    with open(path, "w", newline="") as f:
        w = csv.writer(f)
        w.writerow(["wage", "gender"] + names)
        for g, x, y in (("M", d["xa"], d["ya"]), ("F", d["xb"], d["yb"])):
            for i in range(len(y)):
                w.writerow([repr(float(y[i])), g] + [repr(float(v)) for v in x[i]])
    frame = ob.read_csv(str(path))
    r = (ob.OaxacaBuilder(frame, "wage", "gender", "F").predictors(names).bootstrap_reps(200).seed(SEED).run())
    parsed = {k: [] for k in ["wage", "gender"] + names}
    with open(path) as f:
        for row in csv.DictReader(f):
            for k in parsed:
                parsed[k].append(row[k] if k == "gender" else float(row[k]))
    o = O.OracleBuilder(parsed, "wage", "gender", "F").set(names, reps=200, seed=SEED).run()
    from test_gpu_parity import compare_results

    compare_results(r, o)
    assert r.n_a == 5000 and r.n_b == 5000 and r.n_failed == 0
    assert abs(r.two_fold.aggregate[0].estimate + r.two_fold.aggregate[1].estimate - r.total_gap) <= 1e-9


def _rel_pivot(g):
    """Smallest Cholesky pivot of g relative to its diagonal entry (nalgebra's column order);
    <= 0 where the reference's cholesky() fails."""
    k = g.shape[0]
    L = np.zeros_like(g)
    worst = np.inf
    for j in range(k):
        v = g[j, j] - L[j, :j] @ L[j, :j]
        worst = min(worst, v / g[j, j])
        if v <= 0:
            return v / g[j, j]
        L[j, j] = np.sqrt(v)
        for i in range(j + 1, k):
            L[i, j] = (g[i, j] - L[i, :j] @ L[j, :j]) / L[j, j]
    return worst


@pytest.mark.parametrize("eps", [0.0, 1e-7, 1e-3])
def test_near_singular_failure_rule(ob, O, eps):
    """x3 = x1 + x2 + eps z: exact-in-math collinearity (eps = 0), rounding-size pivots (1e-7,
    relative pivot ~1e-14), and a resolvable design (1e-3, ~1e-7 > BAND)."""
    rng = np.random.default_rng(17)
    n = 3000

    def design(shift):
        x1, x2, z = rng.normal(size=n) + shift, rng.normal(size=n), rng.normal(size=n)
        x = np.column_stack([x1, x2, x1 + x2 + eps * z])
        y = 1.0 + x1 - 0.5 * x2 + rng.normal(size=n)
        return x, y

    xa, ya = design(0.2)
    xb, yb = design(0.0)
    panel = ob.Panel(xa, ya, xb, yb)
    rows, ok = panel.boot(SEED, 0, 256, 0)
    rows2, ok2 = panel.boot(SEED, 0, 256, 0)
    assert np.array_equal(ok, ok2) and np.array_equal(rows, rows2, equal_nan=True)  # deterministic
    assert np.isfinite(rows[ok.astype(bool)]).all()
    cfg = O.PassConfig(4, 3, 0, False)
    XA, XB = O.with_intercept(xa), O.with_intercept(xb)
    orows, ook = O.boot_ref(cfg, XA, ya, None, XB, yb, None, SEED, 0, 256, threads=_threads(), full=False)
    resolved = 0
    for r in range(256):
        piv = min(_rel_pivot((X.T * np.bincount(O.resample_indices(SEED, r, g, n), minlength=n)) @ X)
                  for g, X in ((0, XA), (1, XB)))
        if abs(piv) > BAND:
            resolved += 1
            assert ok[r] == ook[r], (r, piv)
            if ok[r]:
                gap = abs(orows[r, 5])
                assert np.all(np.abs(rows[r] - orows[r]) <= RTOL * np.maximum(np.abs(orows[r]), gap)), r
    if eps == 1e-3:
        assert resolved == 256 and ok.all()
    if eps <= 1e-7:
        assert resolved == 0  # every replicate is inside the band: no mask comparison is meaningful


@pytest.mark.parametrize("ref", [0, 2])
def test_configs1_scale_normalized_categorical(ob, O, ref):
    """configs[1] scale with a normalized categorical (normalization.rs:5-51, builder.rs:547-590):
    1M rows, 15 numeric predictors + a 6-level categorical (5 dummies, normalized), WLS, GroupA
    and Pooled; every row and the SE/CI/p of every reported column vs the oracle (1e-6)."""
    n = 1_000_000
    d = O.synthetic_panel(n, 15, True, seed=31)
    rng = np.random.default_rng(31)
    lev_a = rng.integers(0, 6, d["xa"].shape[0])
    lev_b = np.minimum(rng.integers(0, 7, d["xb"].shape[0]), 5)  # a different level mix in B
    dum = lambda lv: np.column_stack([lv == j for j in range(1, 6)]).astype(float)
    xa = np.hstack([d["xa"], dum(lev_a)])
    xb = np.hstack([d["xb"], dum(lev_b)])
    norm = {"start": [0, 5], "idx": [16, 17, 18, 19, 20], "m": [6], "pstart": [0, 5],
            "pidx": [17, 18, 19, 20, 21], "has_base": [1]}
    panel = ob.Panel(xa, d["ya"], xb, d["yb"], d["wa"], d["wb"], n_num=15, norm=norm)
    try:
        rows, ok = panel.boot(SEED, 0, 128, ref)
    finally:
        panel.close()
    cfg = O.PassConfig(21, 15, O.REF_FROM_ENUM[ref], True, norm)
    orows, ook = O.boot_ref(cfg, O.with_intercept(xa), d["ya"], d["wa"], O.with_intercept(xb), d["yb"], d["wb"],
                            SEED, 0, 128, threads=_threads(), full=False)
    assert ook.all()
    gap = abs(float(np.nanmedian(orows[:, 5])))
    _stats_close(rows, ok, orows, ook, list(range(orows.shape[1])), gap, ob, O)
    scale = np.maximum(np.abs(orows), gap)
    assert np.all(np.abs(rows - orows) <= RTOL * scale)


def test_configs3_rif_multi_tau_full_size(ob, O):
    """configs[3] at its size (builder.rs:711-757, rif.rs:14-88): 1M rows x 20
    predictors, WLS, RIF outcomes at tau = 0.1, 0.5, 0.9 through the public decompose_quantiles
    (one panel, one bootstrap for all three quantiles: K1 = 24 columns, 300 pairs, two-valued RIF
    columns), 128 replicates. Per tau: every component's estimate / SE / CI / p vs the oracle's
    reference algorithm on the RIF outcome (1e-6, mixed), and the result equal to a single-tau
    decompose_quantile run bitwise."""
    taus = (0.1, 0.5, 0.9)
    reps = 128
    d = O.synthetic_panel(1_000_000, 20, True)
    na, nb = len(d["ya"]), len(d["yb"])
    names = [f"x{j + 1}" for j in range(20)]
    x = np.vstack([d["xa"], d["xb"]])
    frame = {"wage": np.concatenate([d["ya"], d["yb"]]), "gender": np.array(["M"] * na + ["F"] * nb, dtype=object),
             "w": np.concatenate([d["wa"], d["wb"]])}
    frame.update({nm: np.ascontiguousarray(x[:, j]) for j, nm in enumerate(names)})

    def builder():
        return (ob.OaxacaBuilder(frame, "wage", "gender", "F").predictors(names).weights("w")
                .bootstrap_reps(reps).seed(SEED))

    multi = builder().decompose_quantiles(taus)
    from test_gpu_parity import compare_results

    xa, xb = O.with_intercept(d["xa"]), O.with_intercept(d["xb"])
    cfg = O.PassConfig(21, 20, 0, True)
    agg = O.OracleBuilder({}, "wage", "gender", "F")
    for t, q in enumerate(taus):
        single = builder().decompose_quantile(q)
        for tab in ("two_fold", "three_fold"):
            for cm, cs in zip(getattr(multi[t], tab).aggregate, getattr(single, tab).aggregate):
                assert (cm.name, cm.estimate, cm.std_err, cm.p_value, cm.ci_lower, cm.ci_upper) == \
                       (cs.name, cs.estimate, cs.std_err, cs.p_value, cs.ci_lower, cs.ci_upper), (q, cm.name)
        for tab in ("detailed_explained", "detailed_unexplained"):
            for cm, cs in zip(getattr(multi[t].two_fold, tab), getattr(single.two_fold, tab)):
                assert (cm.estimate, cm.std_err, cm.ci_lower, cm.ci_upper) == \
                       (cs.estimate, cs.std_err, cs.ci_lower, cs.ci_upper), (q, tab, cm.name)
        ra, rb = O.rif(d["ya"], q), O.rif(d["yb"], q)
        rc, point, resid = O.single_pass(cfg, xa, ra, d["wa"], xb, rb, d["wb"], residuals=True)
        assert rc == 0
        rows, ok = O.boot_ref(cfg, xa, ra, d["wa"], xb, rb, d["wb"], SEED, 0, reps, threads=_threads(), full=False)
        prep = {"cfg": cfg, "detail_names": ["__ob_intercept__"] + names, "ya": ra, "yb": rb}
        o = agg.aggregate(prep, point, rows, ok, resid)
        compare_results(multi[t], o)
        assert multi[t].n_failed == 0


def _qr_objectives(x, y, c, betas, taus, block=100):
    """sum_i c_i rho_tau(y_i - x_i beta) for every fit (quantile_regression.rs:22-129's objective)."""
    out = np.empty(len(taus))
    for s0 in range(0, len(taus), block):
        r = y[:, None] - x @ betas[s0: s0 + block].T
        t = np.asarray(taus[s0: s0 + block])[None, :]
        out[s0: s0 + block] = (c[:, None] * np.where(r >= 0.0, t * r, (t - 1.0) * r)).sum(axis=0)
    return out


def test_configs4_machado_mata_full_size(ob, O):
    """configs[4] at its size (quantile_decomposition.rs:173-279): 500k rows x 15
    predictors, 1,000 simulations per group, 2 replicates plus the point pass.
    * Every quantile regression converges, on the default (row-reduced) path and on the unreduced
      solve (option mm_reduce = 0): the reference drops a fit only when Clarabel does not report
      Solved, so a fit the engine drops would shift the simulation pairing (:238-258).
    * The reduced optimum is the full LP's: on the point pass every fit's objective
      sum c rho_tau(y - x beta) agrees between the two paths to 1e-11 relative (the IPM stops at a
      1e-12 relative gap; the optimal beta itself is only determined to about 1e-6 in flat
      directions at this size).
    * Characteristics + coefficients = gap at every quantile, and the rows of both paths agree to
      1e-6 of the largest value (x beta at drawn rows of those betas)."""
    from test_gpu_mm import QS, mm_data

    d = mm_data(500_000, 15, seed=45)
    sims = 1000
    panel = ob.Panel(d["xa"], d["ya"], d["xb"], d["yb"])
    try:
        rows, ok = panel.mm(SEED, sims, QS, 0, 2)
        t_red = panel.timing()
        conv, betas = {}, {}
        for rep in (0xFFFFFFFF, 0, 1):  # the point pass and both replicates
            b_r, done_r = panel.debug_mm_betas(SEED, sims, rep)
            with ob._native.option("mm_reduce", 0):
                b_f, done_f = panel.debug_mm_betas(SEED, sims, rep)
            conv[rep] = (int(done_r.size - done_r.sum()), int(done_f.size - done_f.sum()))
            betas[rep] = (b_r, b_f)
        point = betas[0xFFFFFFFF]
        rep1_counts = [panel.debug_counts(SEED, 1, 1, g)[1][0].astype(np.int64) for g in (0, 1)]
        with ob._native.option("mm_reduce", 0):
            rows0, ok0 = panel.mm(SEED, sims, QS, 0, 2)
            t_full = panel.timing()
    finally:
        panel.close()
    assert all(v == (0, 0) for v in conv.values()), conv
    assert t_red["mm_reduced"] == 1 and t_full["mm_reduced"] == 0
    assert ok.all() and ok0.all()
    taus = [O.mm_tau(SEED, 0xFFFFFFFF, s) for s in range(sims)]
    for g, (x, y) in enumerate(((d["xa"], d["ya"]), (d["xb"], d["yb"]))):
        xi = np.hstack([np.ones((len(y), 1)), x])
        c = np.ones(len(y))
        o_r = _qr_objectives(xi, y, c, point[0][g], taus)
        o_f = _qr_objectives(xi, y, c, point[1][g], taus)
        assert np.all(np.abs(o_r - o_f) <= 1e-11 * np.abs(o_f)), np.max(np.abs(o_r - o_f) / np.abs(o_f))
    # the HiGHS-exact optima of tests/golden/make_mm_fullsize.py (the oracle's
    # solve_qr restatement, quantile_regression.rs:22-129) at this size -- point-pass fits of both
    # groups at 8 taus over [0.01, 0.99] and replicate 1's first fit -- against the engine's
    # objective at its beta on both paths, 1e-10 relative (the objective is the same at every
    # optimal beta, so it pins degenerate faces too)
    gold = json.load(open(os.path.join(os.path.dirname(__file__), "golden", "mm_fullsize_objectives.json")))
    assert (gold["rows"], gold["predictors"], gold["data_seed"], gold["simulations"], gold["seed"]) == (
        500_000, 15, 45, sims, SEED)
    worst = 0.0
    for f in gold["fits"]:
        g, rep, sim = f["group"], f["rep"], f["sim"]
        x, y = (d["xa"], d["ya"]) if g == 0 else (d["xb"], d["yb"])
        xi = np.hstack([np.ones((len(y), 1)), x])
        if rep == 0xFFFFFFFF:
            c = np.ones(len(y))
        else:
            assert rep == 1
            c = rep1_counts[g]
            assert int(c.sum()) == f["counts_sum"]
            assert hashlib.sha256(c.astype(np.uint8).tobytes()).hexdigest() == f["counts_sha256"]
        assert O.mm_tau(SEED, rep, sim) == f["tau"]
        want = f["primal_objective"]
        assert abs(f["dual_objective"] - want) <= 1e-11 * abs(want)  # HiGHS's own duality gap
        for path in (0, 1):  # reduced, unreduced
            got = _qr_objectives(xi, y, c, betas[rep][path][g][sim: sim + 1], [f["tau"]])[0]
            rel = abs(got - want) / abs(want)
            worst = max(worst, rel)
            assert rel <= 1e-10, (g, hex(rep), sim, f["tau"], path, got, want, rel)
    print(f"configs[4] HiGHS objectives: {len(gold['fits'])} fits x 2 paths, worst relative {worst:.2e}")
    r = rows.reshape(len(rows), len(QS), 3)
    assert np.allclose(r[..., 1] + r[..., 2], r[..., 0], rtol=0, atol=1e-9)
    assert np.allclose(rows, rows0, rtol=0, atol=1e-6 * np.abs(rows0).max()), np.abs(rows - rows0).max()
