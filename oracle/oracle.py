"""TEST INFRASTRUCTURE ONLY -- the CPU restatement of the reference bootstrap path.

Imported by tests/, ``__graft_entry__.smoke()`` and bench.py's ``cpu_baseline`` leg, and only
there, as the checker. The product package never imports it.

Two layers:
* ``liboboracle.so`` (ob_oracle.c): Philox/OBRS-3 resampling, ols() with nalgebra's Cholesky
  order, run_single_pass, the reference-algorithm bootstrap driver (gather every column, full
  X^T X per replicate, Rayon-like threads), bootstrap_stats, RIF.
* ``OracleBuilder`` below: builder.rs's frame logic (clean_dataframe, create_dummies_manual,
  split_groups, prepare_data, run, process_component/process_detailed_components,
  decompose_quantile, get_data_matrices) restated in numpy, independent of the product's C++.

Pinning: tests/test_oracle_kat.py checks this restatement against every known-answer test the
reference holds for the path. Bootstrap SE/CI/p parity is defined on the shared
OBRS-3 stream (the reference's resampling is unseeded, builder.rs:822-827).
"""
from __future__ import annotations

import ctypes as C
import math
import os
import subprocess

import numpy as np

HERE = os.path.dirname(os.path.abspath(__file__))
LIB_PATH = os.path.join(HERE, "liboboracle.so")

REF = {"group_a": 0, "group_b": 1, "pooled": 2, "weighted": 3, "cotton": 3, "neumark": 2}
# product enum values (ReferenceCoefficients) -> oracle modes
REF_FROM_ENUM = {0: 0, 1: 1, 2: 2, 3: 3, 4: 3, 5: 2}

ORC_OK, ORC_E_INSUFFICIENT, ORC_E_CHOLESKY, ORC_E_NEGWEIGHT, ORC_E_GROUP = 0, 1, 2, 3, 4


def build(force: bool = False) -> str:
    if force or not os.path.exists(LIB_PATH) or (
            os.path.getmtime(LIB_PATH) < os.path.getmtime(os.path.join(HERE, "ob_oracle.c"))):
        subprocess.check_call(["make", "-s", "-C", HERE], stdout=subprocess.DEVNULL)
    return LIB_PATH


class _Cfg(C.Structure):
    _fields_ = [("k", C.c_int), ("pool_pos", C.c_int), ("ref_mode", C.c_int), ("weighted", C.c_int),
                ("n_norm", C.c_int), ("norm_start", C.POINTER(C.c_int)), ("norm_idx", C.POINTER(C.c_int)),
                ("norm_m", C.POINTER(C.c_int)), ("pooled_start", C.POINTER(C.c_int)),
                ("pooled_idx", C.POINTER(C.c_int)), ("has_base", C.POINTER(C.c_int))]


_lib = None


def lib():
    global _lib
    if _lib is None:
        build()
        L = C.CDLL(LIB_PATH)
        D, U32, I64 = C.POINTER(C.c_double), C.POINTER(C.c_uint32), C.c_int64
        L.orc_philox4x32_10.argtypes = [U32, U32, U32]
        L.orc_level1_counts.argtypes = [C.c_uint64, C.c_uint32, C.c_uint32, C.c_uint32, U32]
        L.orc_resample_indices.argtypes = [C.c_uint64, C.c_uint32, C.c_uint32, C.c_uint32, U32]
        L.orc_ols.argtypes = [D, D, I64, C.c_int, D, D, D, C.c_int]
        L.orc_ols.restype = C.c_int
        L.orc_row_len.argtypes = [C.c_int, C.c_int]
        L.orc_row_len.restype = C.c_int
        L.orc_n_base.argtypes = [C.POINTER(_Cfg)]
        L.orc_n_base.restype = C.c_int
        L.orc_single_pass.argtypes = [C.POINTER(_Cfg), D, D, D, I64, D, D, D, I64, D, D, C.c_int]
        L.orc_single_pass.restype = C.c_int
        L.orc_boot_ref.argtypes = [C.POINTER(_Cfg), D, D, D, I64, D, D, D, I64, C.c_uint64, C.c_uint32,
                                   C.c_uint32, C.c_int, C.c_int, D, C.POINTER(C.c_uint8)]
        L.orc_binomial_half.argtypes = [C.c_uint32, C.c_uint64, C.c_uint32, C.c_uint32, C.c_uint32, C.c_uint32]
        L.orc_binomial_half.restype = C.c_uint32
        L.orc_bootstrap_stats.argtypes = [D, I64, D]
        L.orc_rif.argtypes = [D, I64, C.c_double, D]
        _lib = L
    return _lib


def _d(a):
    return None if a is None else a.ctypes.data_as(C.POINTER(C.c_double))


# ---------------------------------------------------------------------------------------------
# numeric layer
# ---------------------------------------------------------------------------------------------
def philox(ctr, key):
    c = (C.c_uint32 * 4)(*[int(x) & 0xFFFFFFFF for x in ctr])
    k = (C.c_uint32 * 2)(*[int(x) & 0xFFFFFFFF for x in key])
    o = (C.c_uint32 * 4)()
    lib().orc_philox4x32_10(c, k, o)
    return list(o)


def level1_counts(seed, rep, g, n):
    m = np.zeros(max((n + 255) // 256, 1), dtype=np.uint32)
    lib().orc_level1_counts(seed & (2**64 - 1), rep, g, n, m.ctypes.data_as(C.POINTER(C.c_uint32)))
    return m[: (n + 255) // 256]


def binomial_half(c, seed, rep, g=0, k=0, rl=0):
    """One OBRS-2 level-1 split of c draws (popcount below 4096 draws; Knuth-Yao B(2^j, 1/2)
    samples + popcount bits from 4096 up); rl = (round << 5) + level."""
    return int(lib().orc_binomial_half(c, seed & (2**64 - 1), rep, g, k, rl))


def resample_indices(seed, rep, g, n):
    out = np.zeros(max(n, 1), dtype=np.uint32)
    lib().orc_resample_indices(seed & (2**64 - 1), rep, g, n, out.ctypes.data_as(C.POINTER(C.c_uint32)))
    return out[:n]


def ols(y, x, w=None, full=True):
    """math/ols.rs:44-144 -> (rc, beta, residuals); x is (n, k) including the intercept."""
    x = np.asfortranarray(x, dtype=np.float64)
    y = np.ascontiguousarray(y, dtype=np.float64)
    w = None if w is None else np.ascontiguousarray(w, dtype=np.float64)
    n, k = x.shape
    beta = np.zeros(k)
    res = np.zeros(max(n, 1))
    rc = lib().orc_ols(_d(y), _d(x), n, k, _d(w), _d(beta), _d(res), 1 if full else 0)
    return rc, beta, res[:n]


class PassConfig:
    """orc_cfg; keeps its arrays alive."""

    def __init__(self, k, n_num, ref_mode, weighted, norm=None):
        self._keep = []
        self.c = _Cfg()
        self.c.k, self.c.pool_pos, self.c.ref_mode, self.c.weighted = k, 1 + n_num, ref_mode, 1 if weighted else 0
        norm = norm or {"start": [0], "idx": [], "m": [], "pstart": [0], "pidx": [], "has_base": []}
        arrs = {}
        for key in ("start", "idx", "m", "pstart", "pidx", "has_base"):
            a = np.ascontiguousarray(np.asarray(norm[key], dtype=np.int32).reshape(-1))
            if a.size == 0:
                a = np.zeros(1, dtype=np.int32)
            arrs[key] = a
            self._keep.append(a)
        self.c.n_norm = len(norm["m"])
        P = C.POINTER(C.c_int)
        self.c.norm_start = arrs["start"].ctypes.data_as(P)
        self.c.norm_idx = arrs["idx"].ctypes.data_as(P)
        self.c.norm_m = arrs["m"].ctypes.data_as(P)
        self.c.pooled_start = arrs["pstart"].ctypes.data_as(P)
        self.c.pooled_idx = arrs["pidx"].ctypes.data_as(P)
        self.c.has_base = arrs["has_base"].ctypes.data_as(P)
        self.k = k
        self.n_base = lib().orc_n_base(C.byref(self.c))
        self.row_len = lib().orc_row_len(k, self.n_base)


def single_pass(cfg: PassConfig, xa, ya, wa, xb, yb, wb, residuals=False):
    """run_single_pass on prepared matrices (x incl. intercept) -> (rc, row[, resid_b])."""
    xa, xb = np.asfortranarray(xa, dtype=np.float64), np.asfortranarray(xb, dtype=np.float64)
    ya, yb = np.ascontiguousarray(ya, dtype=np.float64), np.ascontiguousarray(yb, dtype=np.float64)
    wa = None if wa is None else np.ascontiguousarray(wa, dtype=np.float64)
    wb = None if wb is None else np.ascontiguousarray(wb, dtype=np.float64)
    row = np.full(cfg.row_len, np.nan)
    res = np.zeros(max(len(yb), 1))
    rc = lib().orc_single_pass(C.byref(cfg.c), _d(xa), _d(ya), _d(wa), len(ya), _d(xb), _d(yb), _d(wb), len(yb),
                               _d(row), _d(res), 1)
    return (rc, row, res[: len(yb)]) if residuals else (rc, row)


def boot_ref(cfg: PassConfig, xa, ya, wa, xb, yb, wb, seed, first_rep, n_reps, threads=None, full=True):
    """Reference-algorithm bootstrap (builder.rs:816-839) on the OBRS-3 stream -> (rows, ok)."""
    xa, xb = np.asfortranarray(xa, dtype=np.float64), np.asfortranarray(xb, dtype=np.float64)
    ya, yb = np.ascontiguousarray(ya, dtype=np.float64), np.ascontiguousarray(yb, dtype=np.float64)
    wa = None if wa is None else np.ascontiguousarray(wa, dtype=np.float64)
    wb = None if wb is None else np.ascontiguousarray(wb, dtype=np.float64)
    rows = np.full((n_reps, cfg.row_len), np.nan)
    ok = np.zeros(n_reps, dtype=np.uint8)
    threads = threads or min(os.cpu_count() or 1, 16)
    if n_reps:
        lib().orc_boot_ref(C.byref(cfg.c), _d(xa), _d(ya), _d(wa), len(ya), _d(xb), _d(yb), _d(wb), len(yb),
                           seed & (2**64 - 1), first_rep, n_reps, 1 if full else 0, threads, _d(rows),
                           ok.ctypes.data_as(C.POINTER(C.c_uint8)))
    return rows, ok


def bootstrap_stats(values):
    """inference.rs:4-34 -> (std_err, p_value, (lo, hi))"""
    v = np.ascontiguousarray(values, dtype=np.float64)
    out = np.zeros(4)
    lib().orc_bootstrap_stats(_d(v), len(v), _d(out))
    return out[0], out[1], (out[2], out[3])


def rif(y, tau):
    y = np.ascontiguousarray(y, dtype=np.float64)
    out = np.zeros(max(len(y), 1))
    lib().orc_rif(_d(y), len(y), float(tau), _d(out))
    return out[: len(y)]


# ---------------------------------------------------------------------------------------------
# frame layer (builder.rs restated over dict-of-columns frames)
# ---------------------------------------------------------------------------------------------
class OracleError(RuntimeError):
    def __init__(self, kind, msg):
        super().__init__(msg)
        self.kind = kind


def _col(frame, name):
    if name not in frame:
        raise OracleError("ColumnNotFound", f"Column not found: {name}")
    return frame[name]


def _is_null(v):
    return v is None


def _kind(values):
    present = [v for v in values if v is not None]
    if present and all(isinstance(v, str) for v in present):
        return "str"
    if present and all(isinstance(v, (int, np.integer)) and not isinstance(v, bool) for v in present):
        return "i64"
    return "f64"


class OracleBuilder:
    """builder.rs:37-757 over ``{name: list}`` frames (None = null)."""

    def __init__(self, frame, outcome, group, reference_group):
        self.frame = {k: list(v) for k, v in frame.items()}
        self.outcome, self.group, self.reference_group = outcome, group, reference_group
        self.predictors, self.categorical, self.normalize_vars = [], [], []
        self.reps, self.ref_mode, self.weights, self.seed = 20, 0, None, 0x0B5EED
        self.selection, self.selection_predictors = None, []

    def heckman(self, outcome, predictors):  # builder.rs:238-246
        self.selection, self.selection_predictors = outcome, list(predictors)
        return self

    # setters mirror builder.rs:165-246
    def set(self, predictors=(), categorical=(), normalize=(), reps=20, ref_mode=0, weights=None, seed=0x0B5EED):
        self.predictors, self.categorical, self.normalize_vars = list(predictors), list(categorical), list(normalize)
        self.reps, self.ref_mode, self.weights, self.seed = reps, ref_mode, weights, seed
        return self

    def clean_dataframe(self, frame):  # builder.rs:760-784
        cols = [self.outcome, self.group] + self.predictors + self.categorical + ([self.weights] if self.weights else [])
        if self.selection:
            cols += [self.selection] + self.selection_predictors
        for c in cols:
            _col(frame, c)
        n = len(next(iter(frame.values()))) if frame else 0
        keep = [i for i in range(n) if all(not _is_null(frame[c][i]) for c in cols)]
        return {k: [v[i] for i in keep] for k, v in frame.items()}

    def create_dummies(self, values, name):  # builder.rs:380-418
        if _kind(values) != "str":
            raise OracleError("PolarsError", "invalid series dtype: expected `String`")
        levels = sorted(set(v for v in values if v is not None))
        if not levels:
            raise OracleError("InvalidGroupVariable", f"Could not get reference category for {name}")
        dummies = {f"{name}_{lv}": [1.0 if v == lv else 0.0 for v in values] for lv in levels[1:]}
        return dummies, len(levels), f"{name}_{levels[0]}"

    def split_groups(self, frame):  # builder.rs:61-102
        g = frame[self.group]
        if _kind(g) != "str":
            raise OracleError("PolarsError", "invalid series dtype: expected `String`")
        levels = sorted(set(v for v in g if v is not None))
        if len(levels) < 2:
            raise OracleError("InvalidGroupVariable", "Invalid group variable: Not enough groups for comparison")
        b = self.reference_group
        a = levels[1] if levels[0] == b else levels[0]
        ia = [i for i, v in enumerate(g) if v == a]
        ib = [i for i, v in enumerate(g) if v == b]
        return ia, ib, a

    def prepare_data(self, frame, rows, dummy_names, extra=()):  # builder.rs:294-378
        y = frame[self.outcome]
        if _kind(y) != "f64":
            raise OracleError("PolarsError", "invalid series dtype: expected `Float64`")
        names = ["__ob_intercept__"] + self.predictors + list(extra) + list(dummy_names)
        x = np.zeros((len(rows), len(names)))
        x[:, 0] = 1.0
        for j, nm in enumerate(names[1:], start=1):
            if nm in frame:
                x[:, j] = [float(frame[nm][i]) for i in rows]
        yv = np.array([float(y[i]) for i in rows])
        w = np.array([float(frame[self.weights][i]) for i in rows]) if self.weights else None
        return x, yv, w, names

    def _stage(self):
        df = self.clean_dataframe(self.frame)
        dummy_names, counts, bases = [], {}, {}
        for cat in self.categorical:
            d, m, base = self.create_dummies(df[cat], cat)
            counts[cat], bases[cat] = m, base
            dummy_names += list(d)
            df.update(d)
        return df, dummy_names, counts, bases

    def _norm_lists(self, names, pooled_names, counts, bases):
        st, idx, m, pst, pidx, has, base_names = [0], [], [], [0], [], [], []
        for var in self.normalize_vars:
            pre = var + "_"
            idx += [i for i, nm in enumerate(names) if nm.startswith(pre)]
            pidx += [i for i, nm in enumerate(pooled_names) if nm.startswith(pre)]
            st.append(len(idx))
            pst.append(len(pidx))
            m.append(counts.get(var, -1))
            has.append(1 if var in bases else 0)
            if var in bases:
                base_names.append(bases[var])
        return {"start": st, "idx": idx, "m": m, "pstart": pst, "pidx": pidx, "has_base": has}, base_names

    def prepared(self):
        """Everything run() computes before the replicate loop."""
        df, dummy_names, counts, bases = self._stage()
        ia, ib, _ = self.split_groups(df)
        if not ia or not ib:
            raise OracleError("InvalidGroupVariable", "Invalid group variable: One group has no data")
        xa, ya, wa, names = self.prepare_data(df, ia, dummy_names)
        xb, yb, wb, _ = self.prepare_data(df, ib, dummy_names)
        pooled = ["__ob_intercept__"] + self.predictors + ["__ob_group_indicator__"] + dummy_names
        norm, base_names = self._norm_lists(names, pooled, counts, bases)
        cfg = PassConfig(len(names), len(self.predictors), REF_FROM_ENUM[self.ref_mode], self.weights is not None,
                         norm if self.normalize_vars else None)
        return dict(xa=xa, ya=ya, wa=wa, xb=xb, yb=yb, wb=wb, names=names, detail_names=names + base_names,
                    cfg=cfg, norm=norm if self.normalize_vars else None)

    def point(self, prep):
        rc, row, res = single_pass(prep["cfg"], prep["xa"], prep["ya"], prep["wa"], prep["xb"], prep["yb"],
                                   prep["wb"], residuals=True)
        if rc != ORC_OK:
            raise OracleError({1: "InsufficientData", 2: "NalgebraError", 3: "InvalidGroupVariable",
                               4: "InvalidGroupVariable"}[rc], f"single pass failed ({rc})")
        return row, res

    def boot_rows(self, prep, first_rep, n_reps, threads=None, full=False):
        return boot_ref(prep["cfg"], prep["xa"], prep["ya"], prep["wa"], prep["xb"], prep["yb"], prep["wb"],
                        self.seed, first_rep, n_reps, threads=threads, full=full)

    def aggregate(self, prep, point_row, rows, ok, resid):
        """builder.rs:841-950 -> dict shaped like OaxacaResults."""
        k = prep["cfg"].k
        kd = k + prep["cfg"].n_base
        good = rows[ok.astype(bool)]

        def comp(name, point, vals):
            se, p, (lo, hi) = bootstrap_stats(vals)
            t = point / se if abs(se) > 1e-9 else 0.0
            return dict(name=name, estimate=point, std_err=se, t_stat=t, p_value=p, ci_lower=lo, ci_upper=hi)

        def detailed(base):
            out = []
            names = prep["detail_names"]
            for i in range(kd):
                cols = [base + q for q in range(kd) if names[q] == names[i]]
                vals = good[:, cols].reshape(-1) if len(good) else np.zeros(0)
                out.append(comp(names[i], point_row[base + i], vals))
            return out

        tail = 6 + 2 * kd
        return dict(
            total_gap=point_row[5],
            two_fold=dict(aggregate=[comp("explained", point_row[0], good[:, 0]),
                                     comp("unexplained", point_row[1], good[:, 1])],
                          detailed_explained=detailed(6), detailed_unexplained=detailed(6 + kd), detailed_selection=[]),
            three_fold=dict(aggregate=[comp(n, point_row[2 + i], good[:, 2 + i])
                                       for i, n in enumerate(("endowments", "coefficients", "interaction"))],
                            detailed=[]),
            n_a=len(prep["ya"]), n_b=len(prep["yb"]), residuals=resid,
            xa_mean=point_row[tail + 2 * k: tail + 3 * k], xb_mean=point_row[tail + 3 * k: tail + 4 * k],
            beta_star=point_row[tail + 4 * k: tail + 5 * k], n_failed=int(len(ok) - ok.sum()))

    def _heckman_groups(self, df, rows, dummy_names):  # estimation.rs:177-260 for one group
        x, y, w, names = self.prepare_data(df, rows, dummy_names)
        sel = df[self.selection]
        if _kind(sel) != "f64":
            raise OracleError("PolarsError", "invalid series dtype: expected `Float64`")
        zsel = np.ones((len(rows), 1 + len(self.selection_predictors)))
        for j, nm in enumerate(self.selection_predictors, start=1):
            zsel[:, j] = [float(df[nm][i]) for i in rows]
        return dict(x=x, y=y, w=w, zsel=zsel, s=np.array([float(sel[i]) for i in rows])), names

    def run_heckman(self):
        """run() with .heckman_selection(): every pass through heckman_single_pass, replicates
        gathered by the OBRS-3 index stream."""
        df, dummy_names, _, _ = self._stage()
        ia, ib, _ = self.split_groups(df)
        if not ia or not ib:
            raise OracleError("InvalidGroupVariable", "Invalid group variable: One group has no data")
        ga, names = self._heckman_groups(df, ia, dummy_names)
        gb, _ = self._heckman_groups(df, ib, dummy_names)
        weighted = self.weights is not None
        point = heckman_single_pass(ga, gb, self.ref_mode, weighted)
        k1, ks = len(names) + 1, ga["zsel"].shape[1]
        rows, ok = np.full((self.reps, len(point)), np.nan), np.zeros(self.reps, dtype=np.uint8)
        for r in range(self.reps):
            take = []
            for gi, g in enumerate((ga, gb)):
                idx = resample_indices(self.seed, r, gi, len(g["y"]))
                take.append({kk: (None if v is None else v[idx]) for kk, v in g.items()})
            try:
                rows[r] = heckman_single_pass(take[0], take[1], self.ref_mode, weighted)
                ok[r] = 1
            except OracleError:
                pass
        good = rows[ok.astype(bool)]

        def comp(name, pt, vals):
            se, p, (lo, hi) = bootstrap_stats(vals)
            return dict(name=name, estimate=pt, std_err=se, t_stat=pt / se if abs(se) > 1e-9 else 0.0, p_value=p,
                        ci_lower=lo, ci_upper=hi)

        dnames = names + ["IMR"]
        snames = ["__ob_intercept__"] + self.selection_predictors
        base_sel = 6 + 2 * k1 + 5 * k1
        det = lambda base: [comp(dnames[i], point[base + i], good[:, base + i] if len(good) else np.zeros(0))
                            for i in range(k1)]
        n_b_sel = int((gb["s"] == 1.0).sum())
        tail = 6 + 2 * k1
        return dict(
            total_gap=point[5],
            two_fold=dict(aggregate=[comp("explained", point[0], good[:, 0]),
                                     comp("unexplained", point[1], good[:, 1])],
                          detailed_explained=det(6), detailed_unexplained=det(6 + k1),
                          detailed_selection=[comp(snames[i], point[base_sel + i], good[:, base_sel + i])
                                              for i in range(ks)]),
            three_fold=dict(aggregate=[comp(nm, point[2 + i], good[:, 2 + i])
                                       for i, nm in enumerate(("endowments", "coefficients", "interaction"))],
                            detailed=[]),
            n_a=len(ga["y"]), n_b=len(gb["y"]), residuals=np.zeros(n_b_sel),
            xa_mean=point[tail + 2 * k1: tail + 3 * k1], xb_mean=point[tail + 3 * k1: tail + 4 * k1],
            beta_star=point[tail + 4 * k1: tail + 5 * k1], n_failed=int(len(ok) - ok.sum()), rows=rows, ok=ok)

    def run(self, threads=None):
        if self.selection:
            return self.run_heckman()
        prep = self.prepared()
        point_row, resid = self.point(prep)
        rows, ok = self.boot_rows(prep, 0, self.reps, threads=threads)
        return self.aggregate(prep, point_row, rows, ok, resid)

    def decompose_quantile(self, q, threads=None):  # builder.rs:711-757
        df = self.clean_dataframe(self.frame)
        ia, ib, _ = self.split_groups(df)
        y = df[self.outcome]
        ra = rif([y[i] for i in ia], q)
        rb = rif([y[i] for i in ib], q)
        order = ia + ib
        mod = {k: [v[i] for i in order] for k, v in df.items()}
        mod[self.outcome] = list(ra) + list(rb)
        nb = OracleBuilder(mod, self.outcome, self.group, self.reference_group)
        nb.set(self.predictors, self.categorical, self.normalize_vars, self.reps, self.ref_mode, self.weights, self.seed)
        return nb.run(threads=threads)

    def get_data_matrices(self):  # builder.rs:252-291
        df, dummy_names, _, _ = self._stage()
        ia, ib, _ = self.split_groups(df)
        saved, self.weights = self.weights, None
        try:
            xa, ya, _, names = self.prepare_data(df, ia, dummy_names)
            xb, yb, _, _ = self.prepare_data(df, ib, dummy_names)
        finally:
            self.weights = saved
        return xa, ya, xb, yb, names


# ---------------------------------------------------------------------------------------------
# Heckman two-step (estimation.rs:114-260, heckman.rs:38-108, math/probit.rs:25-170) and the
# selection terms of run_single_pass (builder.rs:477-534). statrs Normal(0, 1): cdf(z) =
# 0.5 erfc(-z / sqrt 2), pdf(z) = exp(-z^2 / 2) / sqrt(2 pi).
# ---------------------------------------------------------------------------------------------
def _ncdf(z):
    from scipy.special import erfc

    return 0.5 * erfc(-np.asarray(z, dtype=float) / math.sqrt(2.0))


def _npdf(z):
    z = np.asarray(z, dtype=float)
    return np.exp(-0.5 * z * z) / math.sqrt(2.0 * math.pi)


def _chol_solve_nalgebra(m, b):
    """nalgebra Cholesky (fails iff a pivot is 0, negative or NaN) + solve; None on failure."""
    k = m.shape[0]
    a = np.array(m, dtype=float, order="F")
    for j in range(k):
        for c in range(j):
            a[j:, j] += -a[j, c] * a[j:, c]
        d = a[j, j]
        if not (d != 0.0 and d >= 0.0):
            return None
        a[j, j] = math.sqrt(d)
        a[j + 1:, j] /= a[j, j]
    x = np.array(b, dtype=float)
    for i in range(k):
        x[i] = x[i] / a[i, i]
        x[i + 1:] -= x[i] * a[i + 1:, i]
    for i in range(k - 1, -1, -1):
        x[i] = (x[i] - a[i + 1:, i] @ x[i + 1:]) / a[i, i]
    return x


def probit(y, x, max_iter=100, tol=1e-6, full=False):  # math/probit.rs:25-170 (Fisher scoring from 0)
    k = x.shape[1]
    beta = np.zeros(k)
    converged, it = False, 0
    for it in range(1, max_iter + 1):
        z = x @ beta
        phi = _npdf(z)
        big = np.clip(_ncdf(z), 1e-10, 1.0 - 1e-10)
        lam = np.where(y > 0.5, phi / big, -phi / (1.0 - big))
        w = np.sqrt(phi * phi / (big * (1.0 - big))) ** 2  # sqrt_w squared, as the reference
        g = x.T @ lam
        h = -(x.T * w) @ x - 1e-9 * np.eye(k)
        step = _chol_solve_nalgebra(-h, g)
        if step is None:  # LU fallback (probit.rs:124-137)
            step = -np.linalg.solve(h, g)
        beta = beta + step
        if np.linalg.norm(step) < tol:
            converged = True
            break
    return dict(coefficients=beta, converged=converged, iterations=it) if full else beta


def heckman_two_step(y_sel, x_sel, y_out, x_out, x_sel_sub):  # heckman.rs:38-108
    gamma = probit(y_sel, x_sel)
    zg = x_sel_sub @ gamma
    phi, big = _npdf(zg), _ncdf(zg)
    imr = np.where(big < 1e-10, 0.0, phi / np.where(big < 1e-10, 1.0, big))
    x_aug = np.column_stack([x_out, imr])
    rc, coef, _ = ols(y_out, x_aug)
    if rc != ORC_OK:
        raise OracleError({1: "InsufficientData", 2: "NalgebraError"}[rc], f"heckman ols failed ({rc})")
    delta = float(np.mean(-imr * (imr + zg)))
    return dict(gamma=gamma, beta=coef[:-1], theta=coef[-1], imr=imr, imr_mean=float(imr.mean()), delta=delta)


def heckman_single_pass(ga, gb, ref_mode, weighted):
    """One Heckman decomposition pass. ga/gb: dict(x (n x K with intercept), y, w, zsel (n x Ks with
    intercept), s). Returns the row [aggregates | detailed K+1 | detailed K+1 | beta_a, beta_b,
    xa_mean, xb_mean, beta_star (K+1 each) | selection components (Ks)]."""
    res, means, zmean = [], [], []
    for g in (ga, gb):
        sel = g["s"] == 1.0
        if not sel.any():
            raise OracleError("InvalidGroupVariable", "No observed outcomes in group")
        r = heckman_two_step(g["s"], g["zsel"], g["y"][sel], g["x"][sel], g["zsel"][sel])
        res.append(r)
        means.append(np.append(g["x"][sel].mean(axis=0), r["imr_mean"]))
        zmean.append(g["zsel"].mean(axis=0))
    ba = np.append(res[0]["beta"], res[0]["theta"])
    bb = np.append(res[1]["beta"], res[1]["theta"])
    if ref_mode == 0:
        bs = ba
    elif ref_mode == 1:
        bs = bb
    elif ref_mode in (3, 4):
        na = ga["w"].sum() if weighted else len(ga["y"])
        nb = gb["w"].sum() if weighted else len(gb["y"])
        if na + nb == 0.0:
            raise OracleError("InvalidGroupVariable", "No data in groups for weighted coefficients.")
        wa_ = na / (na + nb)
        bs = ba * wa_ + bb * (1.0 - wa_)
    else:
        raise OracleError("Unsupported", "Heckman with pooled coefficients (the reference panics)")
    xa, xb = means
    dx, db = xa - xb, ba - bb
    expl = float(dx @ bs)
    unexpl = float((xa @ ba - xb @ bb) - expl)
    row = [expl, unexpl, float(dx @ bb), float(xb @ db), float(dx @ db)]
    if weighted:
        gap = ga["y"] @ ga["w"] / ga["w"].sum() - gb["y"] @ gb["w"] / gb["w"].sum()
    else:
        gap = ga["y"].mean() - gb["y"].mean()
    row.append(float(gap))
    row += list(dx * bs) + list(xa * (ba - bs) + xb * (bs - bb))
    row += list(ba) + list(bb) + list(xa) + list(xb) + list(bs)
    th, de, gm = (res[0]["theta"], res[0]["delta"], res[0]["gamma"]) if ref_mode == 0 else \
        (res[1]["theta"], res[1]["delta"], res[1]["gamma"])
    row += list(th * de * gm * (zmean[0] - zmean[1]))
    return np.array(row)


def heckman_row_len(k, ks):
    return 6 + 2 * (k + 1) + 5 * (k + 1) + ks


# ---------------------------------------------------------------------------------------------
# Machado-Mata (quantile_decomposition.rs:21-445, math/quantile_regression.rs:22-129)
# QR is solved exactly with HiGHS (scipy) on the dual LP  max y'a  s.t.  X'a = (1 - tau) X'c,
# 0 <= a <= c (c = resample counts); the equality multipliers are beta. The reference solves the
# primal LP with Clarabel's interior-point method (default tolerances ~1e-8); for a unique
# optimum both give the same beta up to that tolerance (its own tests use 1e-4). The draws follow
# MM-1 (csrc/ob_spec.h) in place of the reference's unseeded thread_rng.
# ---------------------------------------------------------------------------------------------
TAG_MMT, TAG_MMR, MM_POINT_REP = 0x4D4D5431, 0x4D4D5231, 0xFFFFFFFF


def mm_tau(seed, rep, s):  # MM-1 tau_s (quantile_decomposition.rs:215-219)
    x, y, _, _ = philox([s, rep, 0, TAG_MMT], [seed & 0xFFFFFFFF, seed >> 32])
    t = 0.01 + 0.98 * (((x >> 5) * 67108864.0 + (y >> 6)) * (1.0 / 9007199254740992.0))
    return t if t < 0.99 else 0.98999999999999999


def mm_pick(seed, rep, g, i, n):  # MM-1 position of pick i (quantile_decomposition.rs:246-247)
    thresh = (2**32 - n) % n
    j = 0
    while True:
        w = philox([i, rep, g, TAG_MMR + (j >> 2)], [seed & 0xFFFFFFFF, seed >> 32])
        for h in range(4):
            m = w[h] * n
            if (m & 0xFFFFFFFF) >= thresh:
                return m >> 32
        j += 4


def qr_exact(x, y, c, tau):
    """solve_qr (quantile_regression.rs:22-129) on the rows with c > 0; None where it fails."""
    from scipy.optimize import linprog

    act = c > 0
    xa, ya, ca = x[act], y[act], c[act].astype(float)
    if not np.all(np.isfinite(xa)) or not np.all(np.isfinite(ya)):
        return None
    res = linprog(-ya, A_eq=xa.T, b_eq=(1.0 - tau) * (xa.T @ ca), bounds=list(zip(np.zeros(len(ca)), ca)),
                  method="highs")
    if res.status != 0:
        return None
    return -np.asarray(res.eqlin.marginals, dtype=float)


def empirical_quantile(v, q):  # quantile_decomposition.rs:164-171
    if len(v) == 0:
        return 0.0
    v = np.sort(np.asarray(v, dtype=float))
    return float(v[min(int(len(v) * q), len(v) - 1)])


def mm_single_pass(xa, ya, ca, xb, yb, cb, seed, rep, sims, quantiles, fail_mask=None):
    """run_single_pass (quantile_decomposition.rs:173-279) on count-weighted groups; returns the
    row [gap, characteristics, coefficients] per target quantile. fail_mask[g][s] bit (rep & 7)
    drops fit (g, s) as a failed solve_qr (Err, :221-229) -- the engine's ob_debug_mm_fail."""
    taus = [mm_tau(seed, rep, s) for s in range(sims)]

    def dropped(g, s):
        return fail_mask is not None and s < len(fail_mask[g]) and (int(fail_mask[g][s]) >> (rep & 7)) & 1

    # filter_map keeps the successful fits in simulation order, independently per group
    ba = [b for s, b in enumerate(qr_exact(xa, ya, ca, t) for t in taus) if b is not None and not dropped(0, s)]
    bb = [b for s, b in enumerate(qr_exact(xb, yb, cb, t) for t in taus) if b is not None and not dropped(1, s)]
    if len(ba) < sims // 2 or len(bb) < sims // 2:
        raise OracleError("NalgebraError", "Failed to estimate a sufficient number of quantile regressions.")
    num = min(len(ba), len(bb))
    cuma, cumb = np.cumsum(ca), np.cumsum(cb)
    yaa, ybb, yab = [], [], []
    for i in range(num):
        ra = int(np.searchsorted(cuma, mm_pick(seed, rep, 0, i, len(ya)), side="right"))
        rb = int(np.searchsorted(cumb, mm_pick(seed, rep, 1, i, len(yb)), side="right"))
        yaa.append(float(xa[ra] @ ba[i]))
        ybb.append(float(xb[rb] @ bb[i]))
        yab.append(float(xa[ra] @ bb[i]))
    row = []
    for q in quantiles:
        qaa, qbb, qab = empirical_quantile(yaa, q), empirical_quantile(ybb, q), empirical_quantile(yab, q)
        row += [qaa - qbb, qab - qbb, qaa - qab]
    return np.array(row)


class OracleQuantileDecomposition:
    """QuantileDecompositionBuilder (quantile_decomposition.rs:21-445) over {name: list} frames."""

    def __init__(self, frame, outcome, group, reference_group):
        self.frame = {k: list(v) for k, v in frame.items()}
        self.outcome, self.group, self.reference_group = outcome, group, reference_group
        self.predictors, self.categorical = [], []
        self.quantiles, self.simulations, self.reps, self.seed = [0.1, 0.25, 0.5, 0.75, 0.9], 200, 20, 0x0B5EED

    def set(self, predictors=(), categorical=(), quantiles=None, simulations=200, reps=20, seed=0x0B5EED):
        self.predictors, self.categorical = list(predictors), list(categorical)
        if quantiles is not None:
            self.quantiles = list(quantiles)
        self.simulations, self.reps, self.seed = simulations, reps, seed
        return self

    def _groups(self):
        g = self.frame[self.group]
        levels = sorted(set(v for v in g if v is not None))
        b = self.reference_group
        a = levels[0] if levels and levels[0] != b else (levels[1] if len(levels) > 1 else "")
        return a, b

    def _design(self, rows, dummies):  # prepare_data (quantile_decomposition.rs:96-141)
        y = self.frame[self.outcome]
        if _kind(y) != "f64":
            raise OracleError("PolarsError", "invalid series dtype: expected `Float64`")
        if any(y[i] is None for i in rows):
            raise OracleError("InvalidGroupVariable", "Null outcome encountered")
        cols = [[1.0] * len(rows)]
        for nm in self.predictors:
            cols.append([np.nan if self.frame[nm][i] is None else float(self.frame[nm][i]) for i in rows])
        for nm in dummies:
            cols.append([dummies[nm][i] for i in rows])
        return np.array(cols, dtype=float).T, np.array([float(y[i]) for i in rows])

    def prepared(self):
        dummies = {}
        for cat in self.categorical:  # create_dummies_manual (quantile_decomposition.rs:143-161)
            vals = self.frame[cat]
            if _kind(vals) != "str":
                raise OracleError("PolarsError", "invalid series dtype: expected `String`")
            for lv in sorted(set(v for v in vals if v is not None))[1:]:
                dummies[f"{cat}_{lv}"] = [np.nan if v is None else (1.0 if v == lv else 0.0) for v in vals]
        a, b = self._groups()
        g = self.frame[self.group]
        ia = [i for i, v in enumerate(g) if v == a]
        ib = [i for i, v in enumerate(g) if v == b]
        if len(ia) < 2 or len(ib) < 2:
            raise OracleError("InvalidGroupVariable", "One group has insufficient data")
        xa, ya = self._design(ia, dummies)
        xb, yb = self._design(ib, dummies)
        return xa, ya, xb, yb

    def run(self):
        xa, ya, xb, yb = self.prepared()
        one_a, one_b = np.ones(len(ya), dtype=np.int64), np.ones(len(yb), dtype=np.int64)
        point = mm_single_pass(xa, ya, one_a, xb, yb, one_b, self.seed, MM_POINT_REP, self.simulations,
                               self.quantiles)
        rows = np.full((self.reps, len(point)), np.nan)
        ok = np.zeros(self.reps, dtype=np.uint8)
        for r in range(self.reps):
            ca = np.bincount(resample_indices(self.seed, r, 0, len(ya)), minlength=len(ya))
            cb = np.bincount(resample_indices(self.seed, r, 1, len(yb)), minlength=len(yb))
            try:
                rows[r] = mm_single_pass(xa, ya, ca, xb, yb, cb, self.seed, r, self.simulations, self.quantiles)
                ok[r] = 1
            except OracleError:
                pass
        good = rows[ok.astype(bool)]
        out = {}
        for qi, q in enumerate(self.quantiles):
            det = {}
            for k, nm in enumerate(("Total Gap", "Characteristics", "Coefficients")):
                pt = point[3 * qi + k]
                se, p, (lo, hi) = bootstrap_stats(good[:, 3 * qi + k] if len(good) else np.zeros(0))
                det[nm] = dict(name=nm, estimate=pt, std_err=se, t_stat=pt / se if abs(se) > 1e-9 else 0.0,
                               p_value=p, ci_lower=lo, ci_upper=hi)
            out[f"q{int(q * 100.0)}"] = det
        a, b = self._groups()
        g = self.frame[self.group]
        return dict(results_by_quantile=out, n_a=sum(v == a for v in g), n_b=sum(v == b for v in g), point=point,
                    rows=rows, ok=ok)


# ---------------------------------------------------------------------------------------------
# synthetic wage panel, deterministic from a seed
# ---------------------------------------------------------------------------------------------
def synthetic_panel(n, p, weighted, seed=20260424):
    """Groups A ('M') and B ('F'), n/2 rows each. x1 education, x2 experience, x3 = x2^2/100,
    x4.. ~ N(0,1) (+0.2 in A); y = [1, x] beta_g + N(0, 0.5^2), beta_A = beta_B + 0.05.
    Returns dict(xa, ya, wa, xb, yb, wb) with predictor-only x (no intercept column)."""
    rng = np.random.default_rng(seed)
    out = {}
    na = n // 2
    nb = n - na
    beta_b = np.concatenate([[5.0, 0.08, 0.03, -0.04], 0.1 * np.ones(max(p - 3, 0))])[: p + 1]
    for g, ng in (("a", na), ("b", nb)):
        x = np.empty((ng, p))
        if p >= 1:
            x[:, 0] = np.clip(np.round(rng.normal(13.0, 2.5, ng)), 8, 20)
        if p >= 2:
            x[:, 1] = rng.uniform(0.0, 40.0, ng)
        if p >= 3:
            x[:, 2] = x[:, 1] ** 2 / 100.0
        if p >= 4:
            x[:, 3:] = rng.normal(0.2 if g == "a" else 0.0, 1.0, (ng, p - 3))
        beta = beta_b + (0.05 if g == "a" else 0.0)
        y = beta[0] + x @ beta[1:] + rng.normal(0.0, 0.5, ng)
        out["x" + g] = x
        out["y" + g] = y
        out["w" + g] = rng.uniform(0.5, 2.0, ng) if weighted else None
    return out


def with_intercept(x):
    return np.hstack([np.ones((x.shape[0], 1)), x])


def rel_close(a, b, rtol, scale=None):
    """Mixed tolerance |a-b| <= rtol * max(|b|, scale)."""
    a, b = np.asarray(a, dtype=float), np.asarray(b, dtype=float)
    s = np.abs(b) if scale is None else np.maximum(np.abs(b), scale)
    return np.all(np.abs(a - b) <= rtol * np.maximum(s, 1e-300)) or np.allclose(a, b, rtol=rtol, atol=0)


if __name__ == "__main__":
    print(philox([0, 0, 0, 0], [0, 0]))
    print(math.pi)
