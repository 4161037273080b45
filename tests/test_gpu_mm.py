"""Machado-Mata on the MI355X engine (QuantileDecompositionBuilder, ob_mm.hip) vs the oracle:
HiGHS-exact quantile regressions and the same MM-1 draws (oracle.mm_single_pass). Pass rows,
builder results, the reference's MM test frame, determinism and identities at a larger size.
The GPU's interior-point QR matches the exact LP vertex to ~1e-10 (tools/qr_ipm_proto.py); the
tolerance below is the suite's 1e-6, relative to the scale of the compared quantities."""
import numpy as np
import pytest

from test_gpu_parity import RTOL, SEED, close

pytestmark = pytest.mark.gpu

QS = [0.1, 0.25, 0.5, 0.75, 0.9]


def mm_data(n, p, seed):
    """Continuous covariates (unique QR optima); heteroskedastic t(4) errors so quantiles differ."""
    rng = np.random.default_rng(seed)
    out = {}
    for g, ng in (("a", n // 2), ("b", n - n // 2)):
        x = rng.normal(size=(ng, p)) + (0.3 if g == "a" else 0.0)
        x[:, 0] = rng.uniform(8.0, 20.0, ng)
        y = 1.0 + x @ np.linspace(0.1, 0.5, p) + (0.3 if g == "a" else 0.0) + rng.standard_t(4, ng) * (
            0.5 + 0.05 * x[:, 0])
        out["x" + g], out["y" + g] = x, y
    return out


def oracle_rows(O, d, sims, qs, reps, fail_mask=None):
    """Point pass then replicates 0..reps-1; a pass the reference would fail (:231-236) is a NaN row
    with ok = 0, as the engine reports it."""
    xa, xb = O.with_intercept(d["xa"]), O.with_intercept(d["xb"])
    na, nb = len(d["ya"]), len(d["yb"])
    counts = [(np.ones(na, np.int64), np.ones(nb, np.int64), O.MM_POINT_REP)]
    for r in range(reps):
        counts.append((np.bincount(O.resample_indices(SEED, r, 0, na), minlength=na),
                       np.bincount(O.resample_indices(SEED, r, 1, nb), minlength=nb), r))
    rows, ok = [], []
    for ca, cb, rep in counts:
        try:
            rows.append(O.mm_single_pass(xa, d["ya"], ca, xb, d["yb"], cb, SEED, rep, sims, qs, fail_mask))
            ok.append(1)
        except O.OracleError:
            rows.append(np.full(3 * len(qs), np.nan))
            ok.append(0)
    return (np.array(rows), np.array(ok, np.uint8)) if fail_mask is not None else np.array(rows)


def close_mm(rows, want, n_q):
    """Mixed per-quantity tolerance: |d| <= 1e-6 max(|want|, |gap of that pass at that quantile|)
    for the gap, characteristics and coefficients effects of every pass and quantile."""
    r = np.asarray(rows, float).reshape(len(rows), n_q, 3)
    w = np.asarray(want, float).reshape(len(want), n_q, 3)
    scale = np.maximum(np.abs(w), np.abs(w[..., :1]))
    err = np.abs(r - w)
    nan_ok = np.isnan(r) & np.isnan(w)
    bad = ~(err <= RTOL * scale) & ~nan_ok
    return not bad.any(), float(np.nanmax(np.where(nan_ok, 0.0, err / np.maximum(scale, 1e-300))))


@pytest.mark.parametrize("n,p,sims", [(600, 1, 30), (1500, 3, 40), (3000, 5, 24), (5000, 15, 12),
                                      (6000, 16, 8), (6000, 23, 8), (8000, 31, 6)])
def test_mm_rows_match_oracle(ob, O, n, p, sims):
    d = mm_data(n, p, seed=n + p)
    panel = ob.Panel(d["xa"], d["ya"], d["xb"], d["yb"])
    try:
        rows, ok = panel.mm(SEED, sims, QS, 0, 3)
    finally:
        panel.close()
    want = oracle_rows(O, d, sims, QS, 3)
    assert ok.all()
    good, worst = close_mm(rows, want, len(QS))
    assert good, worst


def test_mm_point_pass_only_on_a_fresh_panel(ob, O):
    """The point pass alone (no bootstrap replicate: no count images drawn) on a panel that never
    ran a boot: the overflow flag the call checks is its own, not the allocation's garbage."""
    d = mm_data(900, 2, seed=13)
    panel = ob.Panel(d["xa"], d["ya"], d["xb"], d["yb"])
    try:
        rows, ok = panel.mm(SEED, 16, QS, 0, 0)
    finally:
        panel.close()
    want = oracle_rows(O, d, 16, QS, 0)
    assert list(ok) == [1]
    good, worst = close_mm(rows, want, len(QS))
    assert good, worst


def mm_frame(n, seed=4):
    rng = np.random.default_rng(seed)
    g = np.where(rng.random(n) < 0.5, "M", "F")
    edu = rng.uniform(8, 20, n)
    exp_ = rng.uniform(0, 40, n)
    sector = rng.choice(["a", "b", "c"], n)
    y = 1.0 + 0.08 * edu + 0.02 * exp_ + 0.2 * (g == "M") + 0.1 * (sector == "c") + rng.standard_t(4, n) * 0.4
    return {"wage": y.tolist(), "education": edu.tolist(), "experience": exp_.tolist(), "sector": sector.tolist(),
            "gender": g.tolist()}


def test_mm_builder_matches_oracle(ob, O):
    f = mm_frame(2400)
    r = (ob.QuantileDecompositionBuilder(f, "wage", "gender", "F").predictors(["education", "experience"])
         .categorical_predictors(["sector"]).quantiles([0.1, 0.5, 0.9]).simulations(30).bootstrap_reps(6)
         .seed(SEED).run())
    o = (O.OracleQuantileDecomposition(f, "wage", "gender", "F")
         .set(["education", "experience"], ["sector"], [0.1, 0.5, 0.9], 30, 6, SEED).run())
    assert (r.n_a, r.n_b) == (o["n_a"], o["n_b"]) and r.n_failed == 0
    assert sorted(r.results_by_quantile) == sorted(o["results_by_quantile"]) == ["q10", "q50", "q90"]
    scale = np.abs(o["rows"]).max()
    for key, det in r.results_by_quantile.items():
        want = o["results_by_quantile"][key]
        for c in (det.total_gap, det.characteristics_effect, det.coefficients_effect):
            w = want[c.name]
            for fld in ("estimate", "std_err", "ci_lower", "ci_upper"):
                assert abs(getattr(c, fld) - w[fld]) <= RTOL * max(abs(w[fld]), scale), (key, c.name, fld)
            assert c.p_value == w["p_value"]


def test_mm_reference_test_frame(ob):  # tests/integration_test.rs:165-198
    f = {"wage": [10.0, 12.0, 11.0, 13.0, 15.0, 20.0, 22.0, 21.0, 23.0, 25.0, 9.0, 18.0],
         "education": [12.0, 16.0, 14.0, 16.0, 18.0, 12.0, 16.0, 14.0, 16.0, 18.0, 10.0, 20.0],
         "gender": ["F"] * 6 + ["M"] * 6}
    r = (ob.QuantileDecompositionBuilder(f, "wage", "gender", "F").predictors(["education"])
         .quantiles([0.25, 0.5, 0.75]).simulations(10).bootstrap_reps(2).run())
    for key in ("q25", "q50", "q75"):
        d = r.results_by_quantile[key]
        assert abs(d.characteristics_effect.estimate + d.coefficients_effect.estimate - d.total_gap.estimate) < 1e-9
    assert r.n_a == 6 and r.n_b == 6


def test_mm_errors(ob, N):
    f = mm_frame(200)
    with pytest.raises(N.OaxacaError) as e:
        ob.QuantileDecompositionBuilder(f, "wage", "gender", "F").predictors(["nope"]).run()
    assert e.value.code == N.OB_E_COLUMN
    g = dict(f, wage=[None] + f["wage"][1:])
    with pytest.raises(N.OaxacaError) as e:  # quantile_decomposition.rs:103-110
        ob.QuantileDecompositionBuilder(g, "wage", "gender", "F").predictors(["education"]).run()
    assert e.value.code == N.OB_E_GROUP and "Null outcome" in str(e.value)
    h = dict(f, gender=["F"] * 199 + ["M"])
    with pytest.raises(N.OaxacaError) as e:  # :202-206
        ob.QuantileDecompositionBuilder(h, "wage", "gender", "F").predictors(["education"]).run()
    assert "insufficient data" in str(e.value)


def test_mm_width_limit(ob, N):
    """32 columns (intercept + 31 predictors) run; 33 are refused with OB_E_UNSUPPORTED."""
    d = mm_data(800, 32, seed=3)
    panel = ob.Panel(d["xa"], d["ya"], d["xb"], d["yb"])
    try:
        with pytest.raises(N.OaxacaError) as e:
            panel.mm(SEED, 8, QS, 0, 1)
        assert e.value.code == N.OB_E_UNSUPPORTED
    finally:
        panel.close()


def test_mm_deterministic_and_shard_invariant(ob):
    d = mm_data(4000, 4, seed=7)
    panel = ob.Panel(d["xa"], d["ya"], d["xb"], d["yb"])
    try:
        r0, k0 = panel.mm(SEED, 64, QS, 0, 6)
        r1, k1 = panel.mm(SEED, 64, QS, 2, 4, with_point=False)
        r2, _ = panel.mm(SEED, 64, QS, 0, 6)
    finally:
        panel.close()
    assert np.array_equal(r0, r2) and k0.all()
    assert np.array_equal(r0[3:], r1) and np.array_equal(k0[3:], k1)


def test_mm_identities_at_size(ob):
    """200k rows, 15 predictors (K = 16, configs[4]'s width), 100 simulations, 3 replicates: every
    pass succeeds, characteristics + coefficients = gap at every quantile, and the median gap is the
    raw median difference up to simulation noise."""
    d = mm_data(200_000, 15, seed=11)
    panel = ob.Panel(d["xa"], d["ya"], d["xb"], d["yb"])
    try:
        rows, ok = panel.mm(SEED, 100, QS, 0, 3)
    finally:
        panel.close()
    assert ok.all()
    r = rows.reshape(len(rows), len(QS), 3)
    assert np.allclose(r[..., 1] + r[..., 2], r[..., 0], rtol=0, atol=1e-9)
    # the point gap at the median approximates the difference of the groups' median outcomes
    assert abs(r[0, 2, 0] - (np.median(d["ya"]) - np.median(d["yb"]))) < 0.3


@pytest.fixture
def reduce_env(ob):
    """Option mm_reduce: "1" forces the row reduction (subsample, bands, reduced LPs, verification)
    at any size, "0" turns it off; "" (unset) runs it when both groups have >= 2^16 rows."""
    def set_(v):
        ob._native.set_option("mm_reduce", int(v) if v else None)
    yield set_
    ob._native.set_option("mm_reduce", None)


@pytest.mark.parametrize("n,p,sims", [(3000, 2, 40), (6000, 5, 24), (20000, 15, 8)])
def test_mm_row_reduction_matches_oracle(ob, O, reduce_env, n, p, sims):
    """Forced row reduction against the oracle's HiGHS-exact fits: when every fixed row's sign
    verifies, the reduced LP's optimum is the full LP's (Portnoy & Koenker 1997)."""
    reduce_env("1")
    d = mm_data(n, p, seed=n + p + 1)
    panel = ob.Panel(d["xa"], d["ya"], d["xb"], d["yb"])
    try:
        rows, ok = panel.mm(SEED, sims, QS, 0, 3)
        t = panel.timing()
    finally:
        panel.close()
    assert t["mm_reduced"] == 1
    want = oracle_rows(O, d, sims, QS, 3)
    assert ok.all()
    good, worst = close_mm(rows, want, len(QS))
    assert good, worst


def test_mm_row_reduction_equals_full_solve(ob, reduce_env):
    """At 150k rows (K = 16) the default path reduces; its rows equal the unreduced solve's (both
    reach the same LP optima, to the IPM's 1e-12 gap)."""
    d = mm_data(150_000, 15, seed=21)
    panel = ob.Panel(d["xa"], d["ya"], d["xb"], d["yb"])
    try:
        reduce_env("")
        r1, k1 = panel.mm(SEED, 128, QS, 0, 2)
        t1 = panel.timing()
        reduce_env("0")
        r0, k0 = panel.mm(SEED, 128, QS, 0, 2)
        t0 = panel.timing()
    finally:
        panel.close()
    assert t1["mm_reduced"] == 1 and t0["mm_reduced"] == 0
    assert k1.all() and k0.all()
    assert np.allclose(r1, r0, rtol=0, atol=1e-8 * np.abs(r0).max()), np.abs(r1 - r0).max()
    assert t1["mm_fit_rows"] < t0["mm_fit_rows"], (t1["mm_fit_rows"], t0["mm_fit_rows"])


def test_mm_failed_fits_pair_by_index_and_sims_half_rule(ob, O):
    """The reference drops a failed solve_qr per group independently (filter_map, :221-229), pairs
    the survivors by index (:238-258) and fails a pass with fewer than simulations / 2 survivors
    in a group (:231-236). Forced failures (ob_debug_mm_fail), the oracle applying the same rules:
    * every pass: A loses simulations 2, 5, 11 (A's betas shift against B's);
    * replicate 1: B also loses simulation 7;
    * replicate 2: A loses 8 more (11 of 20 fail, 9 survivors < 10): the pass fails;
    * replicate 3: A loses 7 more (exactly 10 = sims / 2 survivors): the pass holds."""
    d = mm_data(1500, 3, seed=5)
    sims = 20
    mask = np.zeros((2, sims), np.uint8)
    mask[0, [2, 5, 11]] = 0xFF
    mask[1, 7] |= 1 << 1
    mask[0, 12:20] |= 1 << 2
    mask[0, 12:19] |= 1 << 3
    panel = ob.Panel(d["xa"], d["ya"], d["xb"], d["yb"])
    try:
        panel.debug_mm_fail(mask)
        rows, ok = panel.mm(SEED, sims, QS, 0, 4)
        panel.debug_mm_fail(None)
        clean, _ = panel.mm(SEED, sims, QS, 0, 4)
    finally:
        panel.close()
    want, wok = oracle_rows(O, d, sims, QS, 4, fail_mask=mask)
    assert list(ok) == list(wok) == [1, 1, 1, 0, 1]
    good, worst = close_mm(rows, want, len(QS))
    assert good, worst
    assert np.isnan(rows[3]).all()
    assert not np.allclose(rows[1], clean[1])  # the shifted pairing changes the pass


def test_mm_point_pass_failure(ob, O, N):
    """More than half of group B's point-pass fits failing fails the point pass (ok = 0, NaN row),
    which QuantileDecompositionBuilder::run reports as NalgebraError (:231-236, ob_builder.cpp)."""
    d = mm_data(1200, 2, seed=6)
    sims = 16
    mask = np.zeros((2, sims), np.uint8)
    mask[1, :9] = 1 << 7  # the point pass (rep 2^32 - 1): 9 of 16 fail, 7 < 8 survive
    panel = ob.Panel(d["xa"], d["ya"], d["xb"], d["yb"])
    try:
        panel.debug_mm_fail(mask)
        rows, ok = panel.mm(SEED, sims, QS, 0, 2)
    finally:
        panel.close()
    want, wok = oracle_rows(O, d, sims, QS, 2, fail_mask=mask)
    assert list(ok) == list(wok) == [0, 1, 1]
    good, worst = close_mm(rows, want, len(QS))
    assert good, worst


def _golden_mm():
    import json
    import os

    with open(os.path.join(os.path.dirname(os.path.abspath(__file__)), "golden", "mm_sims.json")) as f:
        return json.load(f)["cases"]


@pytest.mark.parametrize("case", range(2))
def test_mm_many_simulations_match_golden(ob, case):
    """configs[4]'s simulation count (1000) and 2500: the finish kernel's LDS bitonic sort then
    holds several fitted values per thread (256 threads, sort width 1024 / 4096). Rows vs the
    oracle's (HiGHS-exact fits, MM-1 draws) committed by tests/golden/make_mm_sims.py."""
    c = _golden_mm()[case]
    d = mm_data(c["rows"], c["predictors"], seed=c["data_seed"])
    panel = ob.Panel(d["xa"], d["ya"], d["xb"], d["yb"])
    try:
        rows, ok = panel.mm(c["seed"], c["simulations"], c["quantiles"], 0, c["replicates"])
    finally:
        panel.close()
    assert list(ok) == c["ok"] == [1] * (1 + c["replicates"])
    good, worst = close_mm(rows, np.array(c["pass_rows"]), len(c["quantiles"]))
    assert good, worst


def _qr_objective(x, y, c, beta, tau):
    r = y - x @ beta
    return float(np.sum(c * np.where(r >= 0, tau * r, (tau - 1.0) * r)))


def test_mm_degenerate_lp_reaches_the_optimum(ob, O):
    """Integer-valued covariates (years of education, whole years of experience) and an outcome
    on a 0.5 grid: many rows tie, the QR LP is degenerate and its optimal face is not a point.
    HiGHS (the oracle) returns a vertex of that face, Clarabel (the reference, an IPM) and the
    engine's IPM a point inside it, so the coefficients need not agree. What every optimum shares
    is the objective sum_i c_i rho_tau(y_i - x_i beta) (quantile_regression.rs:22-129): the
    engine's must equal HiGHS's for every fit, point pass and a resample, to the IPM's stopping
    rule (1e-9 relative)."""
    rng = np.random.default_rng(8)
    d = {}
    for g, ng in (("a", 400), ("b", 360)):
        edu = rng.integers(8, 21, ng).astype(float)
        exp_ = rng.integers(0, 41, ng).astype(float)
        y = np.round(2.0 * (1.0 + 0.08 * edu + 0.02 * exp_ + rng.standard_t(4, ng) * 0.4)) / 2.0
        d["x" + g], d["y" + g] = np.column_stack([edu, exp_]), y
    sims = 24
    panel = ob.Panel(d["xa"], d["ya"], d["xb"], d["yb"])
    try:
        fits = {rep: panel.debug_mm_betas(SEED, sims, rep) for rep in (O.MM_POINT_REP, 3)}
    finally:
        panel.close()
    xs = [O.with_intercept(d["xa"]), O.with_intercept(d["xb"])]
    ys = [d["ya"], d["yb"]]
    ties = 0
    for rep, (betas, done) in fits.items():
        assert done.all(), (rep, done)
        for g in (0, 1):
            n = len(ys[g])
            c = np.ones(n) if rep == O.MM_POINT_REP else np.bincount(O.resample_indices(SEED, rep, g, n), minlength=n)
            for s in range(sims):
                tau = O.mm_tau(SEED, rep, s)
                bh = O.qr_exact(xs[g], ys[g], c.astype(np.int64), tau)
                fh = _qr_objective(xs[g], ys[g], c, bh, tau)
                fe = _qr_objective(xs[g], ys[g], c, betas[g, s], tau)
                assert abs(fe - fh) <= 1e-9 * (1.0 + abs(fh)), (rep, g, s, tau, fe, fh)
                # residual signs: no row of positive count lies strictly beyond the optimum's
                # balance -- the share of the count below the fit is at most tau
                r = ys[g] - xs[g] @ betas[g, s]
                tol = 1e-7 * (1.0 + np.abs(ys[g]))
                assert c[r < -tol].sum() <= tau * c.sum() + 1e-9 and c[r > tol].sum() <= (1 - tau) * c.sum() + 1e-9
                ties += int(np.abs(bh - betas[g, s]).max() > 1e-6)
    print(f"degenerate fits whose engine coefficients differ from the HiGHS vertex: {ties} of {4 * sims}")


def test_mm_after_async_boot_on_a_side_stream(ob):
    """an asynchronous boot on a user stream, followed at once by mm() on the same panel
    (the context stream): MM rewrites the count images and flags the boot may still be reading, so
    the engine orders it after the boot (engine_order / engine_mark). Both results must equal the
    same calls made one after the other."""
    import torch

    d = mm_data(400_000, 15, seed=31)
    panel = ob.Panel(d["xa"], d["ya"], d["xb"], d["yb"])
    try:
        n = 8000
        want_rows, want_ok = panel.boot(SEED, 100, n, 0)
        want_mm, want_mok = panel.mm(SEED, 16, QS, 0, 2)
        dev = torch.device("cuda", 0)
        rows = torch.empty((n, panel.row_len), dtype=torch.float64, device=dev)
        ok = torch.empty(n, dtype=torch.uint8, device=dev)
        side = torch.cuda.Stream(device=dev)
        panel.boot_device(SEED, 100, n, rows.data_ptr(), ok.data_ptr(), 0, stream=side.cuda_stream)
        got_mm, got_mok = panel.mm(SEED, 16, QS, 0, 2)  # no host sync in between
        side.synchronize()
        assert np.array_equal(rows.cpu().numpy(), want_rows) and np.array_equal(ok.cpu().numpy(), want_ok)
        assert np.array_equal(got_mok, want_mok)
        assert np.array_equal(got_mm, want_mm, equal_nan=True)
        # and the other way round: a boot on the side stream right after mm() waits for it
        got_mm2, _ = panel.mm(SEED, 16, QS, 2, 2)
        panel.boot_device(SEED, 100, n, rows.data_ptr(), ok.data_ptr(), 0, stream=side.cuda_stream)
        side.synchronize()
        assert np.array_equal(rows.cpu().numpy(), want_rows)
    finally:
        panel.close()


def test_mm_count_overflow_raises_and_leaves_boot_flag(ob):
    """the Machado-Mata run reads the overflow word engine_counts writes (d_flags[2]),
    ORed over every segment, and does not clear the boot calls' word. With the overflow forced
    (option debug_count_overflow) mm() and debug_counts() raise OB_E_OVERFLOW; with it unset the
    same calls succeed, and an async boot issued before mm() still reports clean."""
    import torch

    N = ob._native
    d = mm_data(4000, 3, seed=33)
    panel = ob.Panel(d["xa"], d["ya"], d["xb"], d["yb"])
    try:
        with N.option("debug_count_overflow", 1):
            with pytest.raises(N.OaxacaError) as e:
                panel.mm(SEED, 16, QS, 0, 3)
            assert e.value.code == N.OB_E_OVERFLOW
            with pytest.raises(N.OaxacaError) as e:
                panel.debug_counts(SEED, 0, 4, 0)
            assert e.value.code == N.OB_E_OVERFLOW
            # the point pass alone draws no counts, so it cannot overflow
            panel.mm(SEED, 16, QS, 0, 0)
        rows, ok = panel.mm(SEED, 16, QS, 0, 2)
        assert ok.all()
        dev = torch.device("cuda", 0)
        brow = torch.empty((64, panel.row_len), dtype=torch.float64, device=dev)
        bok = torch.empty(64, dtype=torch.uint8, device=dev)
        panel.boot_device(SEED, 0, 64, brow.data_ptr(), bok.data_ptr(), 0)
        panel.mm(SEED, 16, QS, 0, 1)
        panel.sync()  # collects the boot's flag: clean
    finally:
        panel.close()
