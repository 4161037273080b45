"""Parity of the HIP engine (through the C ABI) with the oracle on the same OBRS-3 stream.

Tolerance (SURVEY.md §8c, f64 throughout): |engine - oracle| <= 1e-6 * max(|oracle|, |total_gap|)
element-wise; observed differences are ~1e-9 relative (summation order only). Failure masks
(replicates the reference would drop) must be identical. All tests need an MI355X."""
import json
import os

import numpy as np
import pytest

pytestmark = pytest.mark.gpu
ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
KAT = json.load(open(os.path.join(ROOT, "tests", "golden", "reference_kat.json")))
RTOL = 1e-6
SEED = 0x0B5EED


def close(a, b, gap_scale, rtol=RTOL):
    a, b = np.asarray(a, float), np.asarray(b, float)
    scale = np.maximum(np.abs(b), abs(gap_scale))
    bad = ~(np.abs(a - b) <= rtol * scale)
    bad &= ~(np.isnan(a) & np.isnan(b))
    return not bad.any(), (np.abs(a - b) / np.maximum(scale, 1e-300)).max() if a.size else 0.0


def make(O, ob, n, p, weighted, seed=11, extra_cols=None, norm=None, n_num=None):
    d = O.synthetic_panel(n, p, weighted, seed=seed)
    xa, xb = d["xa"], d["xb"]
    if extra_cols is not None:
        xa = np.hstack([xa, extra_cols[0]])
        xb = np.hstack([xb, extra_cols[1]])
    panel = ob.Panel(xa, d["ya"], xb, d["yb"], d["wa"], d["wb"], n_num=n_num, norm=norm)
    k = xa.shape[1] + 1
    cfg = O.PassConfig(k, xa.shape[1] if n_num is None else n_num, 0, weighted, norm)
    args = [O.with_intercept(xa), d["ya"], d["wa"], O.with_intercept(xb), d["yb"], d["wb"]]
    return panel, cfg, args


CONFIGS = [  # (rows, predictors, weighted)
    (777, 0, False), (777, 1, True), (1500, 3, False), (4000, 5, True), (20001, 5, False),
    (3000, 20, True), (9000, 20, False), (2600, 40, True),
]


@pytest.mark.parametrize("n,p,weighted", CONFIGS)
@pytest.mark.parametrize("ref", [0, 1, 2, 3])
def test_point_estimate_parity(O, ob, n, p, weighted, ref):
    panel, cfg, args = make(O, ob, n, p, weighted)
    cfg.c.ref_mode = O.REF_FROM_ENUM[ref]
    row, res = panel.point_estimate(ref, residuals=True)
    rc, orow, ores = O.single_pass(cfg, *args, residuals=True)
    assert rc == 0
    good, err = close(row, orow, orow[5])
    assert good, f"max rel err {err}"
    assert np.allclose(res, ores, rtol=1e-6, atol=1e-6 * np.abs(args[4]).max())


@pytest.mark.parametrize("n,p,weighted", CONFIGS)
@pytest.mark.parametrize("ref", [0, 2, 3, 5])
def test_replicate_rows_parity(O, ob, n, p, weighted, ref):
    reps = 70 if n * p < 100_000 else 40
    panel, cfg, args = make(O, ob, n, p, weighted)
    cfg.c.ref_mode = O.REF_FROM_ENUM[ref]
    rows, ok = panel.boot(SEED, 3, reps, ref)
    orows, ook = O.boot_ref(cfg, *args, SEED, 3, reps, full=False)
    assert np.array_equal(ok, ook)
    m = ok.astype(bool)
    good, err = close(rows[m], orows[m], np.abs(orows[m, 5]).max())
    assert good, f"max rel err {err}"


def test_identities_hold_per_replicate(O, ob):
    panel, cfg, args = make(O, ob, 8000, 8, True)
    rows, ok = panel.boot(SEED, 0, 300, 2)
    lay = ob.row_layout(panel.k, panel.n_base)
    assert ok.all()
    tf = rows[:, 0] + rows[:, 1]
    assert np.allclose(rows[:, 2] + rows[:, 3] + rows[:, 4], tf, rtol=1e-10, atol=1e-10)
    assert np.allclose(rows[:, lay["detailed_explained"]].sum(1), rows[:, 0], rtol=1e-9, atol=1e-10)
    assert np.allclose(rows[:, lay["detailed_unexplained"]].sum(1), rows[:, 1], rtol=1e-9, atol=1e-10)
    assert np.allclose(tf, rows[:, 5], rtol=1e-8, atol=1e-9)  # OLS with intercept fits the (weighted) means


def test_rare_category_failures_match(O, ob):
    """An all-zero dummy after resampling is an exact zero Cholesky pivot -> dropped replicate."""
    n = 1200
    rng = np.random.default_rng(4)
    da = np.zeros((n // 2, 1))
    da[[5, 99]] = 1.0  # present twice in group A only
    db = np.zeros((n - n // 2, 1))
    db[rng.choice(n - n // 2, 40, replace=False)] = 1.0
    panel, cfg, args = make(O, ob, n, 3, False, extra_cols=(da, db))
    rows, ok = panel.boot(SEED, 0, 200, 0)
    orows, ook = O.boot_ref(cfg, *args, SEED, 0, 200, full=False)
    assert np.array_equal(ok, ook)
    assert 5 < (ok == 0).sum() < 80
    assert np.isnan(rows[~ok.astype(bool)]).all()
    m = ok.astype(bool)
    assert close(rows[m], orows[m], 1.0)[0]


def test_normalized_categorical_parity(O, ob):
    n = 6000
    rng = np.random.default_rng(8)
    lev_a = rng.integers(0, 4, n // 2)
    lev_b = rng.integers(0, 4, n - n // 2)
    dum = lambda lv: np.column_stack([lv == j for j in (1, 2, 3)]).astype(float)
    # names: intercept, x1..x3, sec_1, sec_2, sec_3 ; pooled: intercept, x1..x3, IND, sec_1..sec_3
    norm = {"start": [0, 3], "idx": [4, 5, 6], "m": [4], "pstart": [0, 3], "pidx": [5, 6, 7], "has_base": [1]}
    for ref in (0, 1, 2, 3):
        panel, cfg, args = make(O, ob, n, 3, True, extra_cols=(dum(lev_a), dum(lev_b)), norm=norm, n_num=3)
        cfg.c.ref_mode = O.REF_FROM_ENUM[ref]
        rc, orow = O.single_pass(cfg, *args)
        assert rc == 0 and close(panel.point_estimate(ref), orow, orow[5])[0]
        rows, ok = panel.boot(SEED, 0, 50, ref)
        orows, ook = O.boot_ref(cfg, *args, SEED, 0, 50, full=False)
        assert np.array_equal(ok, ook)
        assert close(rows, orows, np.abs(orows[:, 5]).max())[0]


def test_deterministic_and_shard_invariant(ob, O):
    panel, _, _ = make(O, ob, 5000, 6, True)
    r1, o1 = panel.boot(SEED, 0, 300, 2)
    r2, o2 = panel.boot(SEED, 0, 300, 2)
    assert np.array_equal(r1, r2) and np.array_equal(o1, o2)
    a, _ = panel.boot(SEED, 0, 100, 2)
    b, _ = panel.boot(SEED, 100, 200, 2)
    assert np.array_equal(np.vstack([a, b]), r1)  # replicate ids, not launch shape, define results
    c, _ = panel.boot(SEED + 1, 0, 100, 2)
    assert not np.array_equal(c, a)


def test_segment_boundary(ob, O):
    """More than one 16384-replicate segment in one call."""
    panel, _, _ = make(O, ob, 600, 2, False)
    rows, ok = panel.boot(SEED, 0, 16500, 0)
    t = panel.timing()
    assert t["gram_launches"] == 2 and t["gram_ms"] > 0
    mid, _ = panel.boot(SEED, 16370, 40, 0)
    assert np.array_equal(rows[16370:16410], mid)
    assert ok.all()


def test_device_api_with_torch_stream(ob, O):
    import torch

    panel, _, _ = make(O, ob, 3000, 4, True)
    rows_h, ok_h = panel.boot(SEED, 5, 128, 1)
    dev = torch.device("cuda", 0)
    rows = torch.empty((128, panel.row_len), dtype=torch.float64, device=dev)
    ok = torch.empty(128, dtype=torch.uint8, device=dev)
    s = torch.cuda.Stream(device=dev)
    with torch.cuda.stream(s):
        panel.boot_device(SEED, 5, 128, rows.data_ptr(), ok.data_ptr(), 1, stream=s.cuda_stream)
    panel.sync()
    assert np.array_equal(rows.cpu().numpy(), rows_h) and np.array_equal(ok.cpu().numpy(), ok_h)


# ------------------------------------------------------------------------------------------
# builder level (OaxacaBuilder / OaxacaBlinder) vs OracleBuilder
# ------------------------------------------------------------------------------------------
def compare_results(r, o, gap_tol=None):
    scale = abs(o["total_gap"])
    assert abs(r.total_gap - o["total_gap"]) <= 1e-9 * max(1.0, scale)
    assert r.n_a == o["n_a"] and r.n_b == o["n_b"] and r.n_failed == o["n_failed"]
    for tname in ("aggregate", "detailed_explained", "detailed_unexplained"):
        got, want = getattr(r.two_fold, tname), o["two_fold"][tname]
        assert [c.name for c in got] == [c["name"] for c in want]
        for c, w in zip(got, want):
            for f in ("estimate", "std_err", "p_value", "ci_lower", "ci_upper"):
                a, b = getattr(c, f), w[f]
                if f == "p_value":
                    assert a == b, (tname, c.name, f, a, b)  # sign counts are exact
                else:
                    assert (np.isnan(a) and np.isnan(b)) or abs(a - b) <= RTOL * max(abs(b), scale, 1e-12), (
                        tname, c.name, f, a, b)
    for c, w in zip(r.three_fold.aggregate, o["three_fold"]["aggregate"]):
        assert c.name == w["name"] and abs(c.estimate - w["estimate"]) <= RTOL * max(abs(w["estimate"]), scale)
        assert abs(c.std_err - w["std_err"]) <= RTOL * max(abs(w["std_err"]), scale)
    assert np.allclose(r.residuals, o["residuals"], rtol=1e-6, atol=1e-9 * max(1.0, scale))
    assert np.allclose(r.beta_star, o["beta_star"], rtol=1e-6, atol=1e-9)


def synthetic_frame(n, seed=9, weighted=True):
    rng = np.random.default_rng(seed)
    g = np.where(rng.random(n) < 0.45, "M", "F")
    edu = np.clip(np.round(rng.normal(13, 2.5, n)), 8, 20)
    exp_ = rng.uniform(0, 40, n)
    sector = rng.choice(["agri", "manu", "serv", "tech"], n, p=[0.1, 0.3, 0.4, 0.2])
    region = rng.choice(["n", "s", "e"], n)
    y = (1.0 + 0.08 * edu + 0.03 * exp_ + (g == "M") * 0.2 + (sector == "tech") * 0.3 + rng.normal(0, 0.5, n))
    f = {"wage": y.tolist(), "gender": g.tolist(), "education": edu.tolist(), "experience": exp_.tolist(),
         "sector": sector.tolist(), "region": region.tolist()}
    if weighted:
        f["w"] = rng.uniform(0.5, 2.0, n).tolist()
    return f


@pytest.mark.parametrize("ref", [0, 1, 2, 3, 4, 5])
def test_builder_run_matches_oracle(ob, O, ref):
    f = synthetic_frame(5000)
    b = (ob.OaxacaBuilder(f, "wage", "gender", "F").predictors(["education", "experience"])
         .categorical_predictors(["sector", "region"]).normalize(["sector"]).weights("w")
         .bootstrap_reps(200).reference_coefficients(ref).seed(SEED))
    o = (O.OracleBuilder(f, "wage", "gender", "F")
         .set(["education", "experience"], ["sector", "region"], ["sector"], 200, ref, "w", SEED))
    compare_results(b.run(), o.run())


def test_decompose_quantile_matches_oracle(ob, O):
    f = synthetic_frame(3000, weighted=False)
    for q in (0.1, 0.5, 0.9):
        b = (ob.OaxacaBuilder(f, "wage", "gender", "F").predictors(["education", "experience"])
             .bootstrap_reps(100).reference_coefficients(1).seed(SEED))
        o = O.OracleBuilder(f, "wage", "gender", "F").set(["education", "experience"], reps=100, ref_mode=1, seed=SEED)
        compare_results(b.decompose_quantile(q), o.decompose_quantile(q))


@pytest.mark.parametrize("weighted,ref", [(False, 1), (True, 2), (True, 0)])
def test_decompose_quantiles_multi_tau(ob, O, weighted, ref):
    """one run serves several quantiles; each equals the single-quantile
    run bitwise (same OBRS-3 stream, same per-pair MFMA columns) and the oracle within tolerance."""
    f = synthetic_frame(4000, seed=21, weighted=weighted)
    taus = (0.1, 0.5, 0.9)

    def builder():
        b = (ob.OaxacaBuilder(f, "wage", "gender", "F").predictors(["education", "experience"])
             .categorical_predictors(["sector"]).bootstrap_reps(150).reference_coefficients(ref).seed(SEED))
        return b.weights("w") if weighted else b

    multi = builder().decompose_quantiles(taus)
    assert len(multi) == len(taus)
    for t, q in enumerate(taus):
        single = builder().decompose_quantile(q)
        assert multi[t].total_gap == single.total_gap
        for tab in ("two_fold", "three_fold"):
            for cm, cs in zip(getattr(multi[t], tab).aggregate, getattr(single, tab).aggregate):
                assert (cm.name, cm.estimate, cm.std_err, cm.ci_lower, cm.ci_upper) == \
                       (cs.name, cs.estimate, cs.std_err, cs.ci_lower, cs.ci_upper)
        o = (O.OracleBuilder(f, "wage", "gender", "F")
             .set(["education", "experience"], ["sector"], [], 150, ref, "w" if weighted else None, SEED))
        compare_results(multi[t], o.decompose_quantile(q))


def test_multi_outcome_panel_rows_bitwise(ob, O):
    """Panel with an (n, 3) outcome block: each outcome's rows equal a one-outcome panel's."""
    d = O.synthetic_panel(6000, 6, True, seed=5)
    rng = np.random.default_rng(3)
    ya = np.column_stack([d["ya"], d["ya"] ** 2 / 10, rng.normal(size=d["ya"].size)])
    yb = np.column_stack([d["yb"], d["yb"] ** 2 / 10, rng.normal(size=d["yb"].size)])
    multi = ob.Panel(d["xa"], ya, d["xb"], yb, d["wa"], d["wb"])
    assert multi.n_y == 3
    rows, ok = multi.boot(SEED, 40, 300, 2)
    pe = multi.point_estimate(2)
    for t in range(3):
        one = ob.Panel(d["xa"], ya[:, t], d["xb"], yb[:, t], d["wa"], d["wb"])
        r1, ok1 = one.boot(SEED, 40, 300, 2)
        assert np.array_equal(rows[t], r1, equal_nan=True) and np.array_equal(ok[t], ok1)
        assert np.array_equal(pe[t], one.point_estimate(2))


@pytest.mark.parametrize("mode", ["GroupB", "GroupA", "Pooled", "Weighted"])
def test_reference_integration_runs(ob, mode):  # tests/integration_test.rs:105-144
    k = KAT["integration_frame"]
    f = {"wage": k["wage"], "education": k["education"], "gender": k["gender"]}
    b = (ob.OaxacaBuilder(f, "wage", "gender", "F").predictors(["education"]).bootstrap_reps(5)
         .reference_coefficients(ob.ReferenceCoefficients[mode]))
    r = b.run()
    assert abs(r.total_gap - 10.0) < 1e-9
    assert abs(r.explained().estimate + r.unexplained().estimate - r.total_gap) < 1e-9
    assert r.n_a == 10 and r.n_b == 10
    assert "Two-Fold Decomposition" in r.summary()


def test_reference_categorical_normalize_run(ob):  # tests/integration_test.rs:146-163
    k = KAT["integration_categorical"]
    f = {kk: k[kk] for kk in ("wage", "education", "gender", "union")}
    r = (ob.OaxacaBuilder(f, "wage", "gender", "F").predictors(["education"]).categorical_predictors(["union"])
         .normalize(["union"]).bootstrap_reps(5).run())
    assert abs(r.total_gap - 10.0) < 1e-9
    assert abs(r.explained().estimate + r.unexplained().estimate - r.total_gap) < 1e-9
    assert r.n_a == 10 and r.n_b == 10


def test_python_surface_fit(ob):  # python.rs:193-276 via OaxacaBlinder
    k = KAT["integration_frame"]
    m = ob.OaxacaBlinder({"wage": k["wage"], "education": k["education"], "gender": k["gender"]},
                         "wage", "gender", "F", ["education"], bootstrap_reps=50, seed=1)
    r = m.fit()
    assert abs(r.total_gap - 10.0) < 1e-9 and len(r.two_fold.aggregate) == 2
    assert r.two_fold.detailed_selection == []
    assert "total gap is 10.0000" in r.interpret()
    rq = m.fit_quantile(0.5)
    assert np.isfinite(rq.total_gap)
    js = json.loads(r.to_json())
    assert "total_gap" in js and "aggregate" in js["two_fold"]


def test_reference_weights_nulls_rif(ob):
    k = KAT["weights"]
    f = {kk: k[kk] for kk in ("outcome", "group", "weight", "x")}
    r = ob.OaxacaBuilder(f, "outcome", "group", "B").predictors(["x"]).bootstrap_reps(0).run()
    assert abs(r.total_gap - k["gap_unweighted"]) < k["tol"]
    r = ob.OaxacaBuilder(f, "outcome", "group", "B").predictors(["x"]).weights("weight").bootstrap_reps(0).run()
    assert abs(r.total_gap - k["gap_weighted"]) < k["tol"]
    k = KAT["nulls"]
    r = (ob.OaxacaBuilder({kk: k[kk] for kk in ("outcome", "group", "education")}, "outcome", "group", "B")
         .predictors(["education"]).run())
    assert r.n_a == 3 and r.n_b == 3
    k = KAT["rif"]
    r = (ob.OaxacaBuilder({kk: k[kk] for kk in ("wage", "group", "education")}, "wage", "group", "F")
         .predictors(["education"]).bootstrap_reps(10).decompose_quantile(0.9))
    assert r.total_gap > 0.0


def test_reference_budget(ob):  # tests/optimize_budget_test.rs
    k = KAT["budget"]
    f = {kk: k[kk] for kk in ("wage", "education", "group")}
    r = ob.OaxacaBuilder(f, "wage", "group", "B").predictors(["education"]).run()
    assert abs(r.total_gap - 16.0) < 1e-9
    adj = r.optimize_budget(5.0, 10.0)
    assert len(adj) == 1 and abs(adj[0].adjustment - 5.0) < 1e-9 and abs(adj[0].original_residual + 5.0) < 1e-9
    adj = r.optimize_budget(100.0, 15.0)
    assert len(adj) == 2 and abs(sum(a.adjustment for a in adj) - 6.0) < 1e-9
    assert sorted(round(a.adjustment, 9) for a in adj) == [1.0, 5.0]
    assert r.optimize_budget(100.0, 20.0) == []
    m = ob.OaxacaBlinder(f, "wage", "group", "B", ["education"])
    assert len(m.optimize_budget(5.0, 10.0)) == 1


def test_reference_cotton_neumark(ob):  # tests/features_test.rs:14-35
    k = KAT["reference_groups"]
    f = {kk: k[kk] for kk in ("wage", "education", "experience", "gender")}
    for mode in (ob.ReferenceCoefficients.Cotton, ob.ReferenceCoefficients.Neumark):
        r = (ob.OaxacaBuilder(f, "wage", "gender", "F").predictors(["education", "experience"])
             .reference_coefficients(mode).run())
        assert r.total_gap > 0.0


def test_from_formula_and_csv_frame(ob):  # builder.rs:139-160 + tests/data/wage.csv
    k = KAT["wage_csv"]
    f = {kk: k[kk] for kk in ("wage", "education", "gender", "sector")}
    r = ob.OaxacaBuilder.from_formula(f, "wage ~ education + C(sector)", "gender", "F").bootstrap_reps(2).run()
    assert [c.name for c in r.two_fold.detailed_explained] == ["__ob_intercept__", "education", "sector_B"]


def test_errors_on_gpu(ob, N):
    base = {"y": [1.0, 2.0, 3.0, 4.0, 5.0, 6.0, 7.0, 8.0], "g": ["a"] * 4 + ["b"] * 4,
            "x": [1.0, 2.0, 3.0, 4.0, 1.0, 2.0, 3.0, 4.0]}
    f = dict(base, x2=[2.0, 4.0, 6.0, 8.0, 2.0, 4.0, 6.0, 8.0])  # x2 = 2 x: singular
    with pytest.raises(N.OaxacaError) as e:
        ob.OaxacaBuilder(f, "y", "g", "b").predictors(["x", "x2"]).run()
    assert e.value.code == N.OB_E_LINALG and "Failed to perform Cholesky decomposition" in str(e.value)
    f = dict(base, x2=[1.0, 0.0, 2.0, 5.0, 1.0, 0.0, 3.0, 5.0], x3=[0.0, 1.0, 1.0, 2.0, 2.0, 1.0, 0.0, 3.0])
    with pytest.raises(N.OaxacaError) as e:  # n = 4 <= k = 4
        ob.OaxacaBuilder(f, "y", "g", "b").predictors(["x", "x2", "x3"]).run()
    assert e.value.code == N.OB_E_INSUFFICIENT and "Insufficient data for OLS calculation" in str(e.value)
    f = dict(base, w=[1.0, 1.0, -1.0, 1.0, 1.0, 1.0, 1.0, 1.0])
    with pytest.raises(N.OaxacaError) as e:
        ob.OaxacaBuilder(f, "y", "g", "b").predictors(["x"]).weights("w").run()
    assert e.value.code == N.OB_E_GROUP and "Weights cannot be negative" in str(e.value)
    with pytest.raises(N.OaxacaError) as e:
        ob.OaxacaBuilder(base, "y", "g", "zzz").predictors(["x"]).run()
    assert e.value.code == N.OB_E_GROUP and "One group has no data" in str(e.value)
    with pytest.raises(N.OaxacaError) as e:
        ob.OaxacaBuilder(base, "y", "g", "b").predictors(["x"]).heckman_selection("s", ["x"]).run()
    assert e.value.code == N.OB_E_COLUMN


def test_sharded_fit_two_ranks_on_one_gpu(ob, O, tmp_path):
    """fit_sharded with 2 gloo ranks sharing GPU 0 == single-process run."""
    import subprocess
    import sys

    script = tmp_path / "w.py"
    script.write_text(f"""
import importlib, os, sys, json
sys.path.insert(0, {ROOT!r}); sys.path.insert(0, {os.path.join(ROOT, 'tests')!r})
import torch, torch.distributed as dist
dist.init_process_group("gloo")
ob = importlib.import_module("oaxaca-blinder-rs_amd")
D = importlib.import_module("oaxaca-blinder-rs_amd.distributed")
from test_gpu_parity import synthetic_frame
f = synthetic_frame(4000)
b = (ob.OaxacaBuilder(f, "wage", "gender", "F").predictors(["education", "experience"])
     .categorical_predictors(["sector"]).weights("w").bootstrap_reps(333).reference_coefficients(2).seed(7).device(0))
r = D.fit_sharded(b)
if dist.get_rank() == 0:
    json.dump({{"se": [c.std_err for c in r.two_fold.aggregate], "lo": [c.ci_lower for c in r.two_fold.aggregate]}},
              open({str(tmp_path / 'out.json')!r}, "w"))
dist.destroy_process_group()
""")
    env = dict(os.environ, MASTER_ADDR="127.0.0.1")
    subprocess.run([sys.executable, "-m", "torch.distributed.run", "--nproc-per-node", "2", "--master-addr",
                    "127.0.0.1", "--master-port", "29533", str(script)], check=True, env=env, timeout=600)
    got = json.load(open(tmp_path / "out.json"))
    f = synthetic_frame(4000)
    r = (ob.OaxacaBuilder(f, "wage", "gender", "F").predictors(["education", "experience"])
         .categorical_predictors(["sector"]).weights("w").bootstrap_reps(333).reference_coefficients(2).seed(7).run())
    assert got["se"] == [c.std_err for c in r.two_fold.aggregate]
    assert got["lo"] == [c.ci_lower for c in r.two_fold.aggregate]


def test_full_size_panel_properties(ob, O):
    """BASELINE configs[1] shape (1M x 20, WLS): point estimate vs oracle, 4 replicates vs the
    oracle's reference algorithm, identities and determinism on 512 replicates."""
    d = O.synthetic_panel(1_000_000, 20, True)
    panel = ob.Panel(d["xa"], d["ya"], d["xb"], d["yb"], d["wa"], d["wb"])
    cfg = O.PassConfig(21, 20, 0, True)
    xa, xb = O.with_intercept(d["xa"]), O.with_intercept(d["xb"])
    rc, orow = O.single_pass(cfg, xa, d["ya"], d["wa"], xb, d["yb"], d["wb"])
    assert rc == 0 and close(panel.point_estimate(0), orow, orow[5])[0]
    rows, ok = panel.boot(SEED, 0, 512, 0)
    assert ok.all()
    orows, ook = O.boot_ref(cfg, xa, d["ya"], d["wa"], xb, d["yb"], d["wb"], SEED, 100, 4, threads=4, full=False)
    assert ook.all() and close(rows[100:104], orows, abs(orow[5]))[0]
    assert np.allclose(rows[:, 2] + rows[:, 3] + rows[:, 4], rows[:, 0] + rows[:, 1], rtol=1e-10, atol=1e-12)
    assert np.allclose(rows[:, 0] + rows[:, 1], rows[:, 5], rtol=1e-8, atol=1e-10)
    rows2, _ = panel.boot(SEED, 0, 512, 0)
    assert np.array_equal(rows, rows2)
    # the bootstrap spread is a real sampling distribution: SE of total_gap ~ sd(y)/sqrt(n)*sqrt(2)
    se_gap = rows[:, 5].std(ddof=1)
    sd = np.sqrt((d["ya"].var() + d["yb"].var()) / 2)
    assert 0.5 < se_gap / (sd * np.sqrt(2 / 500_000)) < 2.0


@pytest.mark.parametrize("n", [40960 * 256, 40961 * 256 + 77, 24_000_001])
def test_large_groups_and_the_limit(ob, O, N, n):
    """Large groups: 10,485,760 rows (40,960 tiles, the largest flat level-1 tree), 40,962 tiles
    (level 1 as two subtrees under level 1, partial tail) and 24,000,001 rows (93,751 tiles, D = 17,
    three subtrees under level 2; past the i8 Gram's 2^24-row range, so the f64 MFMA Gram runs).
    Bootstrap rows match the oracle's reference algorithm; 2^28 + 1 rows are refused up front."""
    rng = np.random.default_rng(3)
    x = rng.normal(size=(n, 1))
    y = 1.0 + 0.5 * x[:, 0] + rng.normal(size=n)
    xb, yb = x[:4096] + 0.1, y[:4096] - 0.2
    panel = ob.Panel(x, y, xb, yb)
    try:
        rows, ok = panel.boot(SEED, 0, 2, 0)
        assert panel.timing()["gram_path"] == (1 if n >= 1 << 24 else 2)
    finally:
        panel.close()
    cfg = O.PassConfig(2, 1, 0, False)
    orows, ook = O.boot_ref(cfg, O.with_intercept(x), y, None, O.with_intercept(xb), yb, None, SEED, 0, 2,
                            threads=8, full=False)
    assert ok.all() and ook.all() and close(rows, orows, abs(orows[0, 5]))[0]
    if n == 40960 * 256:
        big = (1 << 28) + 1
        with pytest.raises(N.OaxacaError) as e:
            ob.Panel(np.empty((big, 1)), np.empty(big), xb, yb)
        assert e.value.code == N.OB_E_UNSUPPORTED


@pytest.mark.parametrize("na,nb", [(65536, 256), (65537, 300), (131372, 1000), (200000, 70000), (257, 65535)])
def test_level1_tree_shapes_match_oracle(ob, O, na, nb):
    """Level 1's fair-bit tree at its shape edges: 256 tiles (the largest LDS-only
    tree, no padding), 257 tiles (first m1-direct tree, half of round 0 rejected, 1-row tail),
    one tile, partial tails, several rejection rounds and the direct draws; rows vs the oracle."""
    rng = np.random.default_rng(na + nb)
    xa = rng.normal(size=(na, 1))
    ya = 1.0 + 0.5 * xa[:, 0] + rng.normal(size=na)
    xb = rng.normal(size=(nb, 1)) + 0.1
    yb = 0.8 + 0.4 * xb[:, 0] + rng.normal(size=nb)
    panel = ob.Panel(xa, ya, xb, yb)
    try:
        rows, ok = panel.boot(SEED, 5, 4, 0)
    finally:
        panel.close()
    cfg = O.PassConfig(2, 1, 0, False)
    orows, ook = O.boot_ref(cfg, O.with_intercept(xa), ya, None, O.with_intercept(xb), yb, None, SEED, 5, 4,
                            threads=8, full=False)
    assert ok.all() and ook.all() and close(rows, orows, abs(orows[0, 5]))[0]


def test_double_buffered_resample_bitwise(ob, O):
    """Option rs_double: two m1 / count-image buffers, so each boot segment's level 1 and counts run
    under the previous segment's Gram (ob_engine.hpp). The kernels and their inputs are unchanged,
    so the rows equal the one-buffer run bitwise: single calls, calls enqueued back to back on the
    device API with one sync, a two-segment call, and a point estimate and a debug-counts call (both
    on the first buffer) between boots."""
    import torch

    panel, _, _ = make(O, ob, 5000, 6, True)
    small, _, _ = make(O, ob, 600, 2, False)
    with ob._native.option("rs_double", 0):
        want = [panel.boot(SEED, r0, 300, 2) for r0 in (0, 300, 600)]
        pe = panel.point_estimate(2)
        cnt = panel.debug_counts(SEED, 7, 64, 1)
        long_rows, long_ok = small.boot(SEED, 0, 16500, 0)
    with ob._native.option("rs_double", 1):
        got = [panel.boot(SEED, r0, 300, 2) for r0 in (0, 300, 600)]
        for (a, oa), (b, obb) in zip(want, got):
            assert np.array_equal(a, b) and np.array_equal(oa, obb)
        dev = torch.device("cuda", 0)
        rows = torch.empty((900, panel.row_len), dtype=torch.float64, device=dev)
        ok = torch.empty(900, dtype=torch.uint8, device=dev)
        for i, r0 in enumerate((0, 300, 600)):
            panel.boot_device(SEED, r0, 300, rows[300 * i:].data_ptr(), ok[300 * i:].data_ptr(), 2)
        panel.sync()
        assert np.array_equal(rows.cpu().numpy(), np.vstack([w[0] for w in want]))
        assert np.array_equal(ok.cpu().numpy(), np.concatenate([w[1] for w in want]))
        b0 = panel.boot(SEED, 0, 300, 2)
        assert np.array_equal(panel.point_estimate(2), pe)
        assert all(np.array_equal(x, y) for x, y in zip(panel.debug_counts(SEED, 7, 64, 1), cnt))
        b1 = panel.boot(SEED, 300, 300, 2)
        assert np.array_equal(b0[0], want[0][0]) and np.array_equal(b1[0], want[1][0])
        r2, o2 = small.boot(SEED, 0, 16500, 0)
        assert np.array_equal(r2, long_rows) and np.array_equal(o2, long_ok)


def test_pieced_resample_bitwise(ob, O):
    """Option rs_pieces: level 1 and the count kernel of a segment in replicate pieces, each piece's
    counts beside the next piece's level 1 (ob_engine.hip engine_boot). Same kernels on the same
    (replicate, tile) units, so the rows equal the one-launch run bitwise, with and without the
    double-buffered resample, across a two-segment call and a partial last batch."""
    panel, _, _ = make(O, ob, 7000, 5, True)
    small, _, _ = make(O, ob, 600, 2, False)
    with ob._native.option("rs_pieces", 1), ob._native.option("rs_double", 0):
        want = panel.boot(SEED, 11, 777, 3)
        want_long = small.boot(SEED, 0, 16500, 0)
        cnt = panel.debug_counts(SEED, 11, 128, 0)
    for pieces in (2, 3, 5, 8):
        for dbl in (0, 1):
            with ob._native.option("rs_pieces", pieces), ob._native.option("rs_double", dbl):
                got = panel.boot(SEED, 11, 777, 3)
                assert np.array_equal(got[0], want[0]) and np.array_equal(got[1], want[1]), (pieces, dbl)
                got2 = panel.boot(SEED, 11, 777, 3)  # back to back on the same buffers
                assert np.array_equal(got2[0], want[0]), (pieces, dbl)
    with ob._native.option("rs_pieces", 4):
        r, o = small.boot(SEED, 0, 16500, 0)
        assert np.array_equal(r, want_long[0]) and np.array_equal(o, want_long[1])
        assert all(np.array_equal(x, y) for x, y in zip(panel.debug_counts(SEED, 11, 128, 0), cnt))


def test_tail_stream_bitwise_and_ordered(ob, O):
    """Option tail_stream: the Gram on an engine stream, reduce / exceptions / solve on another, the
    caller's stream waiting for them at the end of the call, so the next segment's Gram runs under
    this one's tail (two partial buffers). Rows bitwise as on one stream; a copy the caller enqueues
    between two calls that reuse one rows buffer still sees the first call's rows (the tail waits
    for the caller's stream); calls alternate between two torch streams; with and without rs_double."""
    import torch

    panel, _, _ = make(O, ob, 6000, 5, True)
    small, _, _ = make(O, ob, 600, 2, False)
    with ob._native.option("tail_stream", 0), ob._native.option("rs_double", 0):
        want = [panel.boot(SEED, r0, 256, 2) for r0 in (0, 256, 512)]
        want_long = small.boot(SEED, 0, 16500, 0)
    dev = torch.device("cuda", 0)
    for dbl in (0, 1):
        with ob._native.option("tail_stream", 1), ob._native.option("rs_double", dbl):
            got = [panel.boot(SEED, r0, 256, 2) for r0 in (0, 256, 512)]
            for (a, oa), (b, obb) in zip(want, got):
                assert np.array_equal(a, b) and np.array_equal(oa, obb), dbl
            rows = torch.empty((256, panel.row_len), dtype=torch.float64, device=dev)
            ok = torch.empty(256, dtype=torch.uint8, device=dev)
            copies = []
            streams = [torch.cuda.Stream(device=dev), torch.cuda.Stream(device=dev)]
            for i, r0 in enumerate((0, 256, 512)):
                st = streams[i % 2]
                if i:
                    st.wait_stream(streams[(i - 1) % 2])  # the caller orders its own streams
                with torch.cuda.stream(st):
                    panel.boot_device(SEED, r0, 256, rows.data_ptr(), ok.data_ptr(), 2, stream=st.cuda_stream)
                    copies.append((rows.clone(), ok.clone()))  # enqueued on st after the call
            panel.sync()
            torch.cuda.synchronize()
            for (c, co), (w, wo) in zip(copies, want):
                assert np.array_equal(c.cpu().numpy(), w) and np.array_equal(co.cpu().numpy(), wo), dbl
            r, o = small.boot(SEED, 0, 16500, 0)
            assert np.array_equal(r, want_long[0]) and np.array_equal(o, want_long[1]), dbl
