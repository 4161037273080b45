"""The C ABI library loads, exports exactly what include/oaxaca_boot.h declares, and its host-only
entry points (bootstrap_stats, aggregate, RIF, get_data_matrices, error mapping) agree with the
oracle. No GPU compute here."""
import json
import os
import re

import numpy as np
import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
KAT = json.load(open(os.path.join(ROOT, "tests", "golden", "reference_kat.json")))


def _header_functions():
    text = open(os.path.join(ROOT, "include", "oaxaca_boot.h")).read()
    text = re.sub(r"/\*.*?\*/", "", text, flags=re.S)
    return set(re.findall(r"\b(ob_[a-z0-9_]+)\s*\(", text))


def test_header_and_exports_agree(N):
    declared = _header_functions()
    assert declared == set(N.EXPORTED)
    lib = N.lib()
    for name in declared:
        assert hasattr(lib, name), name


def test_symbols_in_dynamic_table(N):
    import subprocess

    out = subprocess.run(["nm", "-D", "--defined-only", N.LIB_PATH], capture_output=True, text=True).stdout
    syms = {l.split()[-1] for l in out.splitlines() if " T " in l}
    assert set(N.EXPORTED) <= syms


def test_no_gpu_fails_loudly(N):
    """Without a visible GPU the engine refuses to start (no CPU fallback)."""
    if N.device_count() > 0:
        pytest.skip("a GPU is visible")
    import ctypes as C

    ctx = C.c_void_p()
    rc = N.lib().ob_ctx_create(0, C.byref(ctx))
    assert rc == N.OB_E_HIP
    assert "no HIP device" in N.lib().ob_last_error().decode()


def test_bootstrap_stats_matches_oracle(ob, O):
    rng = np.random.default_rng(1)
    for n in (0, 1, 2, 5, 39, 40, 41, 1000, 10007):
        v = rng.normal(0.3, 1.0, n)
        v[: n // 7] = 0.0
        a, b = ob.bootstrap_stats(v), O.bootstrap_stats(v)
        for x, y in zip((a[0], a[1], *a[2]), (b[0], b[1], *b[2])):
            assert (np.isnan(x) and np.isnan(y)) or abs(x - y) <= 1e-12 * max(1.0, abs(y))
    for vals, p in KAT["p_values"]["cases"]:
        assert abs(ob.bootstrap_stats(vals)[1] - p) < 1e-9


def test_aggregate_matches_per_column(ob, O):
    rng = np.random.default_rng(2)
    rows = rng.normal(size=(5000, 9))
    ok = (rng.random(5000) > 0.1).astype(np.uint8)
    cols = [0, 3, 8]
    out = ob.aggregate(rows, ok, cols)
    for j, c in enumerate(cols):
        se, p, (lo, hi) = O.bootstrap_stats(rows[ok.astype(bool), c])
        assert np.allclose(out[j], [se, p, lo, hi], rtol=1e-12, atol=0)


def test_rif_matches_oracle(ob, O):
    rng = np.random.default_rng(3)
    for n in (0, 1, 2, 3, 10, 1001):
        y = np.round(rng.normal(20, 5, n), 1)
        for tau in (0.1, 0.5, 0.9):
            a, b = ob.rif(y, tau), O.rif(y, tau)
            assert np.allclose(a, b, rtol=1e-12, atol=1e-12)
    y = np.full(50, 3.0)  # zero spread fallback (rif.rs:51-57)
    assert np.allclose(ob.rif(y, 0.5), O.rif(y, 0.5))


def _frames():
    k = KAT["integration_categorical"]
    yield ({"wage": k["wage"], "education": k["education"], "gender": k["gender"], "union": k["union"]},
           "wage", "gender", "F", ["education"], ["union"])
    n = KAT["nulls"]
    yield ({"outcome": n["outcome"], "group": n["group"], "education": n["education"]},
           "outcome", "group", "B", ["education"], [])
    # third group ignored, integer predictor cast to f64, categorical level absent from one group
    yield ({"y": [1.0, 2.0, 3.5, 4.0, 5.0, 6.5, 7.0, 8.0, 9.0],
            "g": ["b", "a", "a", "c", "a", "b", "b", "c", "a"],
            "age": [30, 40, 35, 50, 22, 41, 39, 44, 28],
            "sector": ["x", "y", "x", "z", "y", "x", "y", "z", "x"]},
           "y", "g", "b", ["age"], ["sector"])


@pytest.mark.parametrize("case", list(range(3)))
def test_get_data_matrices_matches_oracle(ob, O, case):
    frame, y, g, ref, preds, cats = list(_frames())[case]
    b = ob.OaxacaBuilder(frame, y, g, ref).predictors(preds).categorical_predictors(cats)
    xa, ya, xb, yb, names = b.get_data_matrices()
    ob_ = O.OracleBuilder(frame, y, g, ref).set(predictors=preds, categorical=cats)
    oxa, oya, oxb, oyb, onames = ob_.get_data_matrices()
    assert names == onames
    assert np.array_equal(xa, oxa) and np.array_equal(xb, oxb)
    assert np.array_equal(ya, oya) and np.array_equal(yb, oyb)


def test_errors_mirror_reference(ob, N):
    f = {"wage": [1.0, 2.0, 3.0], "g": ["a", "a", "a"], "x": [1.0, 2.0, 3.0]}
    with pytest.raises(N.OaxacaError) as e:  # clean_dataframe (builder.rs:773-778)
        ob.OaxacaBuilder(f, "wage", "g", "a").predictors(["nope"]).get_data_matrices()
    assert e.value.code == N.OB_E_COLUMN and "Column not found: nope" in str(e.value)
    with pytest.raises(N.OaxacaError) as e:  # split_groups (builder.rs:67-71)
        ob.OaxacaBuilder(f, "wage", "g", "a").predictors(["x"]).get_data_matrices()
    assert e.value.code == N.OB_E_GROUP and "Not enough groups" in str(e.value)
    f2 = {"wage": [1.0, 2.0], "g": [1, 2], "x": [1.0, 2.0]}
    with pytest.raises(N.OaxacaError) as e:  # `.str()?` on a non-string group column
        ob.OaxacaBuilder(f2, "wage", "g", "1").predictors(["x"]).get_data_matrices()
    assert e.value.code == N.OB_E_POLARS
    f3 = {"wage": [1, 2, 3, 4], "g": ["a", "b", "a", "b"], "x": [1.0, 2.0, 3.0, 4.0]}
    with pytest.raises(N.OaxacaError) as e:  # outcome must be Float64 (builder.rs:308)
        ob.OaxacaBuilder(f3, "wage", "g", "a").predictors(["x"]).get_data_matrices()
    assert e.value.code == N.OB_E_POLARS


def test_formula_parser(ob, N):  # formula.rs:12-58 (tests at formula.rs:63-88)
    assert ob.parse_formula("wage ~ education + experience") == ("wage", ["education", "experience"], [])
    assert ob.parse_formula("wage ~ education + C(sector) + factor(region)") == (
        "wage", ["education"], ["sector", "region"])
    for bad in ("wage education", "~ education", "wage ~ "):
        with pytest.raises(N.OaxacaError):
            ob.parse_formula(bad)


def test_row_layout(ob):
    lay = ob.row_layout(21, 2)
    assert lay["len"] == 6 + 2 * 23 + 5 * 21
    assert lay["beta_star"].stop == lay["len"]


def _write(tmp_path, name, text):
    p = tmp_path / name
    p.write_text(text)
    return str(p)


def test_read_csv_reference_wage_file(ob, tmp_path):
    """tests/data/wage.csv of the reference (golden transcription), read as the CLI's
    LazyCsvReader would: floats for wage/education, strings for gender/sector."""
    k = KAT["wage_csv"]
    cols = ["wage", "education", "gender", "sector"]
    lines = [",".join(cols)] + [",".join(f"{k[c][i]:.1f}" if c in ("wage", "education") else str(k[c][i])
                                        for c in cols) for i in range(len(k["wage"]))]
    f = ob.read_csv(_write(tmp_path, "wage.csv", "\n".join(lines) + "\n"))
    assert list(f) == cols
    assert f["wage"].dtype == np.float64 and np.allclose(f["wage"], k["wage"])
    assert f["gender"] == list(k["gender"]) and f["sector"] == list(k["sector"])
    # the frame feeds the builder's host path (get_data_matrices needs no GPU)
    xa, ya, xb, yb, names = (ob.OaxacaBuilder(f, "wage", "gender", "F").predictors(["education"])
                             .categorical_predictors(["sector"]).get_data_matrices())
    assert names == ["__ob_intercept__", "education", "sector_B"]
    assert len(ya) + len(yb) == len(k["wage"])


def test_read_csv_inference_nulls_quotes(ob, tmp_path):
    text = ('a,b,c,d,e\n'
            '1,2.5,x,,"q,1"\n'
            '2,,y,,"say ""hi"""\r\n'
            '3,4,,,z\n')
    f = ob.read_csv(_write(tmp_path, "t.csv", text))
    assert f["a"].dtype == np.int64 and list(f["a"]) == [1, 2, 3]
    assert f["b"].dtype == np.float64 and isinstance(f["b"], np.ma.MaskedArray)
    assert list(np.ma.getmaskarray(f["b"])) == [False, True, False] and f["b"][2] == 4.0
    assert f["c"] == ["x", "y", None]
    assert f["d"] == [None, None, None]          # all-null inference window -> str column
    assert f["e"] == ["q,1", 'say "hi"', "z"]


def test_read_csv_errors(ob, N, tmp_path):
    with pytest.raises(N.OaxacaError) as e:
        ob.read_csv(str(tmp_path / "missing.csv"))
    assert e.value.code == 1
    rows = "\n".join(["v"] + [str(i) for i in range(150)] + ["1.5"]) + "\n"  # i64 inferred from 100 rows
    with pytest.raises(N.OaxacaError) as e:
        ob.read_csv(_write(tmp_path, "late.csv", rows))
    assert "could not parse" in str(e.value)
    with pytest.raises(N.OaxacaError):
        ob.read_csv(_write(tmp_path, "ragged.csv", "a,b\n1,2\n3\n"))


def test_read_csv_large_parallel(ob, tmp_path):
    rng = np.random.default_rng(1)
    n = 120_000
    x = rng.normal(size=n)
    g = rng.integers(0, 2, n)
    p = tmp_path / "big.csv"
    with open(p, "w") as fh:
        fh.write("x,g\n")
        fh.writelines(f"{v!r},{gg}\n" for v, gg in zip(x.tolist(), g.tolist()))
    f = ob.read_csv(str(p))
    assert np.array_equal(f["x"], x) and np.array_equal(f["g"], g)
