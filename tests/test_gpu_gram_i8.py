"""The exact integer-sliced Gram (ob_gram_i8.hip) against the f64 MFMA Gram (ob_gram_kernel).

Both compute G_r = sum_i c_ri v_i v_i^T (v = sqrt(w) [1, x, y], ols.rs:68-78) for the same
OBRS-3 counts. The i8 path's only approximation is the 54-bit fixed-point split of each pair
product relative to its chunk's power of two (rounding <= 2^-55 of the chunk's largest regular
|P| per row); rows whose magnitude dwarfs their chunk's ("exception rows": some |v_c| >= 2^B x
the chunk's geometric-mean scale of column c, or non-finite) are summed in f64 instead
(DESIGN.md §5.0). So the two Grams must agree to 1e-12 of the natural scale sqrt(G_aa G_bb) of
every entry -- also for replicates that miss a 1e8x sentinel row -- and the rows the engine
returns (default path: i8) must equal the f64 path's rows to 1e-9 relative and the oracle's
(builder.rs:816-839 over gathered rows) to 1e-6.
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


def test_i8_gram_six_slices(ob, O):
    """Tiles whose pairs all have a narrow magnitude range run 6 of the 7 digit slices
    (oz_nsl_kernel); their Gram still agrees with the f64 Gram to 1e-12 of sqrt(G_aa G_bb).
    A heavy-tailed column keeps the tiles holding its pairs on 7 slices."""
    d = O.synthetic_panel(400_000, 20, True, seed=5)
    rng = np.random.default_rng(5)
    for heavy in (False, True):
        xa, xb = d["xa"].copy(), d["xb"].copy()
        if heavy:
            xa[:, 4] = np.exp(rng.normal(0.0, 1.5, xa.shape[0]))
            xb[:, 4] = np.exp(rng.normal(0.0, 1.5, xb.shape[0]))
        panel = ob.Panel(xa, d["ya"], xb, d["yb"], d["wa"], d["wb"])
        try:
            g64 = panel.debug_gram(SEED, 3, 64, path=1)
            g8 = panel.debug_gram(SEED, 3, 64, path=2)
            t = panel.timing()
            assert t["gram_path"] == 2 and t["oz_tiles"] > 0
            if heavy:
                assert 0 < t["oz_tiles6"] < t["oz_tiles"], (t["oz_tiles6"], t["oz_tiles"])
            else:
                assert t["oz_tiles6"] == t["oz_tiles"], (t["oz_tiles6"], t["oz_tiles"])
            assert _check_gram(g8, g64, 22) < 1e-12
        finally:
            panel.close()


def test_i8_rows_equal_f64_rows(ob, O):
    """Default (i8) rows vs the f64 MFMA Gram's rows (option gram_path = 1), all reference modes,
    with dummies."""
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
            with ob._native.option("gram_path", 1):
                r64, ok64 = panel.boot(SEED, 0, 200, ref)
                assert panel.timing()["gram_path"] == 1
            assert np.array_equal(ok8, ok64)
            gap = np.abs(r64[:, 5:6])
            assert np.all(np.abs(r8 - r64) <= 1e-9 * np.maximum(np.abs(r64), gap)), ref
    finally:
        panel.close()


def test_i8_gram_widest_panel(ob, O):
    """p = 120 predictors (k1 = 122, 7,503 pairs: the engine's widest panel) on the default i8
    path: the digit preparation's per-pair LDS is tiled over pair blocks, so the panel
    runs the i8 Gram instead of failing, and agrees with the f64 Gram to 1e-12 of sqrt(G_aa G_bb)."""
    d = O.synthetic_panel(3000, 120, True, seed=120)
    panel = ob.Panel(d["xa"], d["ya"], d["xb"], d["yb"], d["wa"], d["wb"])
    try:
        g8 = panel.debug_gram(SEED, 0, 64, path=0)
        assert panel.timing()["gram_path"] == 2
        g64 = panel.debug_gram(SEED, 0, 64, path=1)  # f64 MFMA Gram: one staged sub-tile at k1 > 101
        assert _check_gram(g8, g64, 122) < 1e-12
        row = panel.point_estimate(0)  # the unit Gram (ob_gram_kernel<.., true>) at the same width
    finally:
        panel.close()
    cfg = O.PassConfig(121, 120, 0, True)
    rc, orow = O.single_pass(cfg, O.with_intercept(d["xa"]), d["ya"], d["wa"], O.with_intercept(d["xb"]), d["yb"],
                             d["wb"])
    assert rc == 0
    scale = np.maximum(np.abs(orow), abs(orow[5]))
    assert np.all(np.abs(row - orow) <= 1e-6 * scale)


# ---- exception rows: sentinels, heavy tails, non-finite values ---------------------------------
def _halve(chunks):
    """Each chunk split in two: the chunking a 2x chunk target would give (64 instead of 32)."""
    out = []
    for g, t0, t1 in chunks:
        m = (t0 + t1) // 2
        out += [(g, t0, m), (g, m, t1)] if t1 - t0 > 1 else [(g, t0, t1)]
    return out


def _exception_rule(xa, ya, wa, xb, yb, wb, chunks, bits_min=8, cap=4096):
    """numpy restatement of oz_scale/oz_dev/oz_choose/oz_collect (ob_gram_i8.hip) over the chunk
    table `chunks` [(group, first tile, end tile)] (the engine's, from ob_debug_chunks): per
    (chunk, column) s_c = floor(mean frexp exponent of the nonzero finite v_c + 0.5); per row d =
    max_c min(ex - s_c, 126) (127 if some v_c is not finite); B = the smallest bits >= 8 leaving
    <= 4096 rows with d > B. Returns (B, sorted [(group, row)])."""
    def vmat(x, y, w):
        one = np.ones((x.shape[0], 1))
        v = np.hstack([one, x, y.reshape(len(y), -1)])
        return v * np.sqrt(w)[:, None] if w is not None else v
    vs = [vmat(xa, ya, wa), vmat(xb, yb, wb)]
    devs = [np.full(v.shape[0], -128, dtype=np.int64) for v in vs]
    for g, t0, t1 in chunks:
        v = vs[g][t0 * 256: t1 * 256]
        with np.errstate(invalid="ignore"):
            ex = np.frexp(np.where(np.isfinite(v), v, 0.0))[1].astype(np.int64)
        nz = (v != 0) & np.isfinite(v)
        s = np.where(nz.any(0), np.floor(np.where(nz, ex, 0).sum(0) / np.maximum(nz.sum(0), 1) + 0.5), 0)
        dev = np.where(nz, np.minimum(ex - s.astype(np.int64), 126), -128).max(1)
        dev = np.where((~np.isfinite(v)).any(1), 127, np.maximum(dev, -128))
        devs[g][t0 * 256: t1 * 256] = dev
    allv = np.concatenate(devs)
    b = bits_min
    while (allv > b).sum() > cap and b < 126:
        b += 1
    return b, [(g, int(r)) for g in (0, 1) for r in np.nonzero(devs[g] > b)[0]]


def _sentinel_panel(O, n, p, seed):
    d = O.synthetic_panel(n, p, True, seed=seed)
    rng = np.random.default_rng(seed)
    xa, xb, ya, yb = d["xa"].copy(), d["xb"].copy(), d["ya"].copy(), d["yb"].copy()
    wa = np.exp(rng.normal(0.0, 1.0, len(ya)))  # log-normal survey weights
    wb = np.exp(rng.normal(0.0, 1.0, len(yb)))
    med = float(np.median(np.abs(xa[:, 1])))
    for r, f in ((1000, 1e6), (1001, 1e7), (1002, 1e8)):  # three sentinels in one chunk of A
        xa[r, 1] = f * med
    xb[4000, 2] = 99_999_999.0  # a top-coded covariate in B
    yb[9000] = 1e9              # and an outcome sentinel
    return xa, ya, wa, xb, yb, wb


def test_exception_rows_follow_the_rule(ob, O):
    """The engine's exception list is exactly the numpy restatement of its rule."""
    xa, ya, wa, xb, yb, wb = _sentinel_panel(O, 120_000, 6, 3)
    panel = ob.Panel(xa, ya, xb, yb, wa, wb)
    try:
        panel.debug_gram(SEED, 0, 64, path=2)
        bits, rows = panel.debug_gram_exceptions()
        b_ref, rows_ref = _exception_rule(xa, ya, wa, xb, yb, wb, panel.debug_chunks())
        assert bits == b_ref == 8 and rows == rows_ref, (bits, rows[:10], rows_ref[:10])
        assert {(0, 1000), (0, 1001), (0, 1002), (1, 4000), (1, 9000)} <= set(rows)
        assert panel.timing()["oz_exceptions"] == len(rows)
    finally:
        panel.close()


def test_exception_rule_depends_on_the_chunking(ob, O):
    """A block of rows scaled by 2^16 that fills a little over half of a chunk at the engine's
    chunking (and all of the first chunk after halving): the exception list the engine returns is
    the rule's over the engine's own chunk table, and the rule over the halved table gives a
    different list -- so the restatement above cannot pass on a stale chunking."""
    d = O.synthetic_panel(120_000, 4, True, seed=21)
    xa = d["xa"].copy()
    chunks = None
    panel = None
    try:
        panel = ob.Panel(d["xa"], d["ya"], d["xb"], d["yb"], d["wa"], d["wb"])
        chunks = panel.debug_chunks()
        panel.close()
        g, t0, t1 = chunks[0]
        assert g == 0 and t1 - t0 >= 4
        hi = (t0 + t1) // 2 * 256  # rows [0, hi) of the first chunk of A: the first half-chunk
        xa[:hi, 1] *= 2.0 ** 16
        panel = ob.Panel(xa, d["ya"], d["xb"], d["yb"], d["wa"], d["wb"])
        assert panel.debug_chunks() == chunks
        panel.debug_gram(SEED, 0, 64, path=2)
        bits, rows = panel.debug_gram_exceptions()
    finally:
        if panel is not None:
            panel.close()
    want = _exception_rule(xa, d["ya"], d["wa"], d["xb"], d["yb"], d["wb"], chunks)
    assert (bits, rows) == want, (bits, len(rows), want[0], len(want[1]))
    stale = _exception_rule(xa, d["ya"], d["wa"], d["xb"], d["yb"], d["wb"], _halve(chunks))
    assert stale != want, "the panel does not discriminate the chunking"


def test_sentinels_gram_exact_for_replicates_missing_them(ob, O):
    """Sentinel rows 1e6-1e8 x the median in one chunk, log-normal weights: the i8 Gram equals
    the f64 Gram to 1e-12 of sqrt(G_aa G_bb) on every replicate -- including the ~37 % that do
    not draw a given sentinel, where a chunk-wide exponent would lose up to 1e-5."""
    xa, ya, wa, xb, yb, wb = _sentinel_panel(O, 200_000, 8, 5)
    panel = ob.Panel(xa, ya, xb, yb, wa, wb)
    try:
        reps = 256
        g64 = panel.debug_gram(SEED, 0, reps, path=1)
        g8 = panel.debug_gram(SEED, 0, reps, path=2)
        assert panel.timing()["gram_path"] == 2 and panel.timing()["oz_exceptions"] >= 5
        worst = _check_gram(g8, g64, 8 + 2)
        assert worst < 1e-12
        na = len(ya)
        drew = np.array([np.isin([1000, 1001, 1002], O.resample_indices(SEED, r, 0, na)) for r in range(reps)])
        assert (~drew[:, 2]).sum() > 50 and (~drew.any(1)).sum() > 0  # replicates missing the 1e8 row, and all three
    finally:
        panel.close()


@pytest.mark.parametrize("ref", [0, 2])
def test_sentinels_rows_and_stats_match_oracle(ob, O, ref):
    """Rows and SE / CI / p of every reported component vs the oracle's gathered-row algorithm
    (builder.rs:816-839, ols.rs:68-89) over 256 replicates, 1e-6 mixed tolerance."""
    xa, ya, wa, xb, yb, wb = _sentinel_panel(O, 200_000, 8, 5)
    panel = ob.Panel(xa, ya, xb, yb, wa, wb)
    try:
        rows, ok = panel.boot(SEED, 0, 256, ref)
        assert panel.timing()["gram_path"] == 2
    finally:
        panel.close()
    cfg = O.PassConfig(9, 8, O.REF_FROM_ENUM[ref], True)
    orows, ook = O.boot_ref(cfg, O.with_intercept(xa), ya, wa, O.with_intercept(xb), yb, wb, SEED, 0, 256,
                            full=False)
    assert np.array_equal(ok, ook)
    gap = abs(float(np.nanmedian(orows[:, 5])))
    m = ook.astype(bool)
    scale = np.maximum(np.abs(orows[m]), gap)
    assert np.all(np.abs(rows[m] - orows[m]) <= 1e-6 * scale)
    st = ob.aggregate(rows, ok, np.arange(6 + 2 * 9, dtype=np.int32))
    for j in range(6 + 2 * 9):
        se, pv, (lo, hi) = O.bootstrap_stats(orows[m, j])
        for got, want in ((st[j, 0], se), (st[j, 2], lo), (st[j, 3], hi)):
            assert abs(got - want) <= 1e-6 * max(abs(want), gap), (j, got, want)
        assert st[j, 1] == pv


def test_heavy_tailed_covariate_matches_oracle(ob, O):
    """A Pareto(1.2) income-like covariate (many rows far above the geometric mean: B rises only if
    more than 4096 would be exceptions) and log-normal weights: rows vs the oracle at 1e-6."""
    d = O.synthetic_panel(150_000, 5, True, seed=9)
    rng = np.random.default_rng(9)
    xa, xb = d["xa"].copy(), d["xb"].copy()
    xa[:, 3] = rng.pareto(1.2, len(xa)) * 1e4 + 1e3
    xb[:, 3] = rng.pareto(1.2, len(xb)) * 1e4 + 1e3
    wa, wb = np.exp(rng.normal(0, 1.5, len(xa))), np.exp(rng.normal(0, 1.5, len(xb)))
    panel = ob.Panel(xa, d["ya"], xb, d["yb"], wa, wb)
    try:
        rows, ok = panel.boot(SEED, 0, 128, 0)
        bits, exc = panel.debug_gram_exceptions()
        assert (bits, exc) == _exception_rule(xa, d["ya"], wa, xb, d["yb"], wb, panel.debug_chunks())
    finally:
        panel.close()
    cfg = O.PassConfig(6, 5, 0, True)
    orows, ook = O.boot_ref(cfg, O.with_intercept(xa), d["ya"], wa, O.with_intercept(xb), d["yb"], wb, SEED, 0, 128,
                            full=False)
    assert np.array_equal(ok, ook) and ok.all()
    gap = abs(float(np.median(orows[:, 5])))
    assert np.all(np.abs(rows - orows) <= 1e-6 * np.maximum(np.abs(orows), gap))


def test_nonfinite_rows_touch_only_replicates_that_draw_them(ob, O):
    """NaN in a predictor of one row of A and inf in the outcome of one row of B (strtod lets both
    through the CSV reader): exception rows, so a replicate that does not draw them is finite and
    equal to the oracle's gathered-row result, and one that does gets the reference's NaN / failed
    Cholesky (ok = 0 iff a pivot is NaN, ob_oracle.c orc_cholesky)."""
    d = O.synthetic_panel(20_000, 4, True, seed=12)
    xa, yb = d["xa"].copy(), d["yb"].copy()
    xa[777, 2] = np.nan
    yb[4321] = np.inf
    panel = ob.Panel(xa, d["ya"], d["xb"], yb, d["wa"], d["wb"])
    try:
        rows, ok = panel.boot(SEED, 0, 200, 0)
        bits, exc = panel.debug_gram_exceptions()
        assert (0, 777) in exc and (1, 4321) in exc
    finally:
        panel.close()
    cfg = O.PassConfig(5, 4, 0, True)
    orows, ook = O.boot_ref(cfg, O.with_intercept(xa), d["ya"], d["wa"], O.with_intercept(d["xb"]), yb, d["wb"],
                            SEED, 0, 200, full=False)
    assert np.array_equal(ok, ook)
    drew_a = np.array([777 in set(O.resample_indices(SEED, r, 0, len(xa))) for r in range(200)])
    assert drew_a.any() and (~drew_a).any()
    assert not ok[drew_a].any()  # a NaN pivot fails the Cholesky, as in the reference
    fin = np.isfinite(orows)
    assert np.array_equal(fin, np.isfinite(rows))
    gap = abs(float(np.nanmedian(orows[:, 5])))
    assert np.all(np.abs(rows[fin] - orows[fin]) <= 1e-6 * np.maximum(np.abs(orows[fin]), gap))


@pytest.mark.parametrize("n,p,weighted,heavy,reps", [
    (400_000, 20, True, False, 300),  # configs[1]-like: every column-tile pair on six slices
    (400_000, 20, True, True, 70),    # a heavy-tailed column: seven-slice tiles, one tile per pass
    (20001, 5, False, False, 131),    # 28 pairs: one column tile, the pair's second tile absent
    (9000, 14, True, False, 64),      # 136 pairs: five column tiles, the last pair lone
    (2600, 40, False, False, 200),    # 903 pairs: 29 column tiles
])
def test_wide_tile_gram_bitwise(ob, O, n, p, weighted, heavy, reps):
    """The two i8 Gram kernels (option gram_tile: 1 = 8 waves x 32 pairs, oz_gram_kernel; 2 = 4
    waves x 64 pairs with AGPR accumulators, oz_gram_w_kernel; 3 = that wide tile with each chunk's
    sub-tiles split over two blocks whose int64 slice-group sums meet in oz_split_combine_kernel)
    form the same exact integer slice sums and combine them with the same two roundings, so their
    Grams are bitwise equal, partial replicate tiles (reps % 256 != 0) and dead batches included."""
    d = O.synthetic_panel(n, p, weighted, seed=n + p + 7)
    xa, xb = d["xa"].copy(), d["xb"].copy()
    if heavy:
        rng = np.random.default_rng(9)
        xa[:, 4] = np.exp(rng.normal(0.0, 1.5, xa.shape[0]))
        xb[:, 4] = np.exp(rng.normal(0.0, 1.5, xb.shape[0]))
    panel = ob.Panel(xa, d["ya"], xb, d["yb"], d["wa"], d["wb"])
    try:
        got = {}
        for tile in (1, 2, 3):
            with ob._native.option("gram_tile", tile):
                got[tile] = panel.debug_gram(SEED, 5, reps, path=2)
                t = panel.timing()
                assert t["gram_path"] == 2 and t["oz_wide"] == tile - 1
        if heavy:
            assert 0 < t["oz_tiles6"] < t["oz_tiles"]
        assert np.array_equal(got[1], got[2], equal_nan=True)
        assert np.array_equal(got[1], got[3], equal_nan=True)
    finally:
        panel.close()
