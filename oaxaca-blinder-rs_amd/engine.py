"""Hot-path binding: the two groups' design resident in HBM (``ob_panel``) and the bootstrap
replicate kernel sequence (``ob_boot_run``). This is the layer a Rust ``run()`` would call in
place of builder.rs:808-847; ``api.OaxacaBuilder`` drives it for frame inputs.
"""
from __future__ import annotations

import ctypes as C

import numpy as np

from . import _native as N
from .api import ReferenceCoefficients


def row_layout(k: int, n_base: int = 0) -> dict:
    """Offsets of the per-replicate row (include/oaxaca_boot.h OB_ROW_*)."""
    kd = k + n_base
    t = 6 + 2 * kd
    return {"explained": 0, "unexplained": 1, "endowments": 2, "coefficients": 3, "interaction": 4,
            "total_gap": 5, "detailed_explained": slice(6, 6 + kd), "detailed_unexplained": slice(6 + kd, 6 + 2 * kd),
            "beta_a": slice(t, t + k), "beta_b": slice(t + k, t + 2 * k), "xa_mean": slice(t + 2 * k, t + 3 * k),
            "xb_mean": slice(t + 3 * k, t + 4 * k), "beta_star": slice(t + 4 * k, t + 5 * k),
            "len": t + 5 * k}


def _dp(a):
    return None if a is None else a.ctypes.data_as(C.POINTER(C.c_double))


def _ip(a):
    return a.ctypes.data_as(C.POINTER(C.c_int32))


class Panel:
    """Two-group design (predictors only; intercept implicit) copied into HBM.

    ``xa``/``xb``: (n_g, p) arrays; ``n_num`` numeric predictors precede dummy columns (the
    pooled group indicator is inserted after them); ``norm`` optionally carries the
    normalization lists (dict with start, idx, m, pstart, pidx, has_base). ``ya``/``yb`` may be
    (n_g, n_y) blocks of several outcomes (RIF multi-tau): every replicate then yields n_y rows
    from one Gram pass, and ``point_estimate``/``boot`` return an outcome axis first.
    """

    def __init__(self, xa, ya, xb, yb, wa=None, wb=None, n_num=None, norm=None, device=None, ctx=None):
        xa = np.asarray(xa, dtype=np.float64)
        xb = np.asarray(xb, dtype=np.float64)
        if xa.ndim != 2 or xb.ndim != 2 or xa.shape[1] != xb.shape[1]:
            raise ValueError("xa/xb must be 2-D with the same number of columns")
        self.p = xa.shape[1]
        self._xa = np.asfortranarray(xa)
        self._xb = np.asfortranarray(xb)
        ya = np.asarray(ya, dtype=np.float64)
        yb = np.asarray(yb, dtype=np.float64)
        self.n_y = 1 if ya.ndim == 1 else ya.shape[1]
        if (yb.ndim == 1 and self.n_y != 1) or (yb.ndim == 2 and yb.shape[1] != self.n_y):
            raise ValueError("ya/yb must carry the same number of outcomes")
        self._ya = np.asfortranarray(ya.reshape(ya.shape[0], self.n_y))  # ld = n_g, as x
        self._yb = np.asfortranarray(yb.reshape(yb.shape[0], self.n_y))
        if len(self._ya) != xa.shape[0] or len(self._yb) != xb.shape[0]:
            raise ValueError("y length mismatch")
        weighted = wa is not None
        if weighted != (wb is not None):
            raise ValueError("weights must be given for both groups or neither")
        self._wa = None if wa is None else np.ascontiguousarray(wa, dtype=np.float64)
        self._wb = None if wb is None else np.ascontiguousarray(wb, dtype=np.float64)
        d = N.ob_panel_desc()
        d.p = self.p
        d.n_num = self.p if n_num is None else int(n_num)
        d.weighted = 1 if weighted else 0
        d.n_y = self.n_y
        d.a = N.ob_group_desc(xa.shape[0], _dp(self._xa), max(xa.shape[0], 1), _dp(self._ya), _dp(self._wa))
        d.b = N.ob_group_desc(xb.shape[0], _dp(self._xb), max(xb.shape[0], 1), _dp(self._yb), _dp(self._wb))
        self._norm_keep = []
        if norm:
            arrs = [np.ascontiguousarray(norm[k], dtype=np.int32)
                    for k in ("start", "idx", "m", "pstart", "pidx", "has_base")]
            self._norm_keep = arrs
            d.n_norm = len(arrs[2])
            (d.norm_start, d.norm_idx, d.norm_m, d.pooled_start, d.pooled_idx, d.has_base) = [_ip(a) for a in arrs]
        self._h = C.c_void_p()
        self._ctx = ctx if ctx is not None else N.context(device)
        N.check(N.lib().ob_panel_create(self._ctx, C.byref(d), C.byref(self._h)))
        self.k = N.lib().ob_panel_k(self._h)
        self.n_base = N.lib().ob_panel_n_base(self._h)
        self.row_len = N.lib().ob_panel_row_len(self._h)
        self.layout = row_layout(self.k, self.n_base)
        self.n_a, self.n_b = xa.shape[0], xb.shape[0]

    def point_estimate(self, ref=ReferenceCoefficients.GroupA, residuals=False):
        row = np.empty((self.n_y, self.row_len))
        res = np.empty((self.n_y, self.n_b)) if residuals else None
        N.check(N.lib().ob_point_estimate(self._h, int(ref), _dp(row), _dp(res)))
        if self.n_y == 1:
            row = row[0]
            res = None if res is None else res[0]
        return (row, res) if residuals else row

    def boot(self, seed: int, first_rep: int, n_reps: int, ref=ReferenceCoefficients.GroupA):
        rows = np.empty((self.n_y, n_reps, self.row_len))
        ok = np.zeros((self.n_y, n_reps), dtype=np.uint8)
        if n_reps:
            N.check(N.lib().ob_boot_run(self._h, seed & ((1 << 64) - 1), first_rep, n_reps, int(ref), _dp(rows),
                                        ok.ctypes.data_as(C.POINTER(C.c_uint8))))
        return (rows[0], ok[0]) if self.n_y == 1 else (rows, ok)

    def mm(self, seed: int, simulations: int, quantiles, first_rep: int = 0, n_reps: int = 0, with_point=True):
        """Machado-Mata passes (ob_mm_run): rows [gap, characteristics, coefficients] per quantile,
        the point pass first when ``with_point``; ok = 0 where a pass failed."""
        q = np.ascontiguousarray(quantiles, dtype=np.float64)
        m = int(bool(with_point)) + n_reps
        rows = np.empty((m, 3 * q.size))
        ok = np.zeros(m, dtype=np.uint8)
        N.check(N.lib().ob_mm_run(self._h, seed & ((1 << 64) - 1), int(simulations), _dp(q), int(q.size), first_rep,
                                  n_reps, int(bool(with_point)), _dp(rows), ok.ctypes.data_as(C.POINTER(C.c_uint8))))
        return rows, ok

    def debug_mm_betas(self, seed: int, simulations: int, rep: int):
        """ob_debug_mm_betas: the 2 x simulations QR coefficient vectors of one MM pass (rep =
        OB_MM_POINT_REP = 2^32 - 1 for the point pass): (betas [2, S, K], converged [2, S])."""
        b = np.empty((2, int(simulations), self.k))
        done = np.zeros((2, int(simulations)), dtype=np.uint8)
        N.check(N.lib().ob_debug_mm_betas(self._h, seed & ((1 << 64) - 1), int(simulations), int(rep), _dp(b),
                                          done.ctypes.data_as(C.POINTER(C.c_uint8))))
        return b, done

    def debug_mm_fail(self, mask=None):
        """ob_debug_mm_fail: mask[g][s] bit (rep & 7) forces fit (g, s) of pass rep to fail."""
        m = np.ascontiguousarray(np.zeros((2, 0)) if mask is None else mask, dtype=np.uint8)
        N.check(N.lib().ob_debug_mm_fail(self._h, m.ctypes.data_as(C.POINTER(C.c_uint8)), m.shape[1]))

    def boot_device(self, seed: int, first_rep: int, n_reps: int, rows_ptr: int, ok_ptr: int,
                    ref=ReferenceCoefficients.GroupA, stream: int | None = None):
        N.check(N.lib().ob_boot_run_device(self._h, seed & ((1 << 64) - 1), first_rep, n_reps, int(ref),
                                           C.c_void_p(rows_ptr), C.c_void_p(ok_ptr), C.c_void_p(stream or 0)))

    def boot_sharded(self, seed: int, first_rep: int, n_reps: int, ref=ReferenceCoefficients.GroupA):
        """This rank's shard of [first_rep, first_rep + n_reps) plus the RCCL all-gather
        (ob_boot_run_sharded): every rank returns all rows. Collective over the panel's rank ctx."""
        rows = np.empty((self.n_y, n_reps, self.row_len))
        ok = np.zeros((self.n_y, n_reps), dtype=np.uint8)
        if n_reps:
            N.check(N.lib().ob_boot_run_sharded(self._h, seed & ((1 << 64) - 1), first_rep, n_reps, int(ref), _dp(rows),
                                                ok.ctypes.data_as(C.POINTER(C.c_uint8))))
        return (rows[0], ok[0]) if self.n_y == 1 else (rows, ok)

    def boot_sharded_device(self, seed: int, first_rep: int, n_reps: int, rows_ptr: int, ok_ptr: int,
                            ref=ReferenceCoefficients.GroupA, stream: int | None = None):
        N.check(N.lib().ob_boot_run_sharded_device(self._h, seed & ((1 << 64) - 1), first_rep, n_reps, int(ref),
                                                   C.c_void_p(rows_ptr), C.c_void_p(ok_ptr), C.c_void_p(stream or 0)))

    def debug_counts(self, seed: int, first_rep: int, n_reps: int, group: int):
        """OBRS-3 counts as the Gram kernel consumes them (ob_debug_counts): (level-1 tile counts
        [n_reps, tiles], per-row counts [n_reps, n_g] uint8)."""
        ng = self.n_a if group == 0 else self.n_b
        tiles = -(-ng // 256)
        l1 = np.zeros((n_reps, tiles), dtype=np.uint32)
        rc = np.zeros((n_reps, ng), dtype=np.uint8)
        N.check(N.lib().ob_debug_counts(self._h, seed & ((1 << 64) - 1), first_rep, n_reps, group,
                                        l1.ctypes.data_as(C.POINTER(C.c_uint32)),
                                        rc.ctypes.data_as(C.POINTER(C.c_uint8))))
        return l1, rc

    def debug_gram(self, seed: int, first_rep: int, n_reps: int, path: int = 0):
        """Reduced extended Grams [n_reps, 2, e_pad] (ob_debug_gram): path 1 = f64 MFMA,
        2 = exact integer-sliced i8 MFMA, 0 = the engine's default."""
        e_pad = -(-((self.k + self.n_y) * (self.k + self.n_y + 1) // 2) // 16) * 16
        g = np.empty((n_reps, 2, e_pad))
        N.check(N.lib().ob_debug_gram(self._h, int(path), seed & ((1 << 64) - 1), first_rep, n_reps, _dp(g)))
        return g

    def debug_chunks(self):
        """The panel's row chunking (ob_debug_chunks): [(group, first tile, end tile), ...]."""
        n = C.c_int32(0)
        N.check(N.lib().ob_debug_chunks(self._h, None, 0, C.byref(n)))
        t = np.zeros(3 * n.value, dtype=np.uint32)
        N.check(N.lib().ob_debug_chunks(self._h, t.ctypes.data_as(C.POINTER(C.c_uint32)), n.value, C.byref(n)))
        return [tuple(int(v) for v in t[3 * c: 3 * c + 3]) for c in range(n.value)]

    def set_gather_columns(self, cols=None):
        """Row columns the sharded entry points gather (ob_panel_set_gather_columns); None = all."""
        c = np.ascontiguousarray([] if cols is None else cols, dtype=np.int32)
        N.check(N.lib().ob_panel_set_gather_columns(self._h, _ip(c), len(c)))

    def component_columns(self):
        """The row columns the aggregation reads: two-fold, three-fold, total gap, detailed."""
        return list(range(6 + 2 * (self.k + self.n_base)))

    def debug_shard_sim(self, world: int, self_rank: int, seed: int, first_rep: int, n_reps: int,
                        ref=ReferenceCoefficients.GroupA):
        """ob_debug_shard_sim: a `world`-rank sharded run simulated on this GPU, as rank
        `self_rank` receives it."""
        rows = np.empty((self.n_y, n_reps, self.row_len))
        ok = np.zeros((self.n_y, n_reps), dtype=np.uint8)
        if n_reps:
            N.check(N.lib().ob_debug_shard_sim(self._h, world, self_rank, seed & ((1 << 64) - 1), first_rep, n_reps,
                                               int(ref), _dp(rows), ok.ctypes.data_as(C.POINTER(C.c_uint8))))
        return (rows[0], ok[0]) if self.n_y == 1 else (rows, ok)

    def debug_gram_exceptions(self):
        """The i8 Gram's exception rows (ob_debug_gram_exceptions): (bits, [(group, row), ...])."""
        bits, n = C.c_int32(0), C.c_int32(0)
        buf = np.zeros(4096, dtype=np.uint32)
        N.check(N.lib().ob_debug_gram_exceptions(self._h, C.byref(bits), C.byref(n),
                                                 buf.ctypes.data_as(C.POINTER(C.c_uint32)), len(buf)))
        ent = buf[: n.value]
        return bits.value, [(int(e >> 31), int(e & 0x7FFFFFFF)) for e in ent]

    def sync(self):
        N.check(N.lib().ob_panel_sync(self._h))

    def timing(self) -> dict:
        t = N.ob_timing()
        N.check(N.lib().ob_panel_last_timing(self._h, C.byref(t)))
        return {f: getattr(t, f) for f, _ in N.ob_timing._fields_}

    def close(self):
        if self._h:
            N.lib().ob_panel_destroy(self._h)
            self._h = None

    def __del__(self):
        try:
            self.close()
        except Exception:
            pass


def boot_multi(panels, seed: int, first_rep: int, n_reps: int, ref=ReferenceCoefficients.GroupA):
    """One process, several GPUs (ob_boot_run_multi): panels[i] (same design, distinct devices)
    runs shard i; the shards are all-gathered over an RCCL clique of those devices."""
    p0 = panels[0]
    rows = np.empty((p0.n_y, n_reps, p0.row_len))
    ok = np.zeros((p0.n_y, n_reps), dtype=np.uint8)
    hs = (C.c_void_p * len(panels))(*[p._h for p in panels])
    if n_reps:
        N.check(N.lib().ob_boot_run_multi(hs, len(panels), seed & ((1 << 64) - 1), first_rep, n_reps, int(ref),
                                          _dp(rows), ok.ctypes.data_as(C.POINTER(C.c_uint8))))
    return (rows[0], ok[0]) if p0.n_y == 1 else (rows, ok)


def bootstrap_stats(values, point_estimate: float = 0.0):
    """inference.rs:4-34 -> (std_err, p_value, (ci_lower, ci_upper)) via the native routine."""
    v = np.ascontiguousarray(values, dtype=np.float64)
    out = np.empty(4)
    N.check(N.lib().ob_bootstrap_stats(_dp(v), len(v), float(point_estimate), _dp(out)))
    return out[0], out[1], (out[2], out[3])


def aggregate(rows, ok, cols):
    """ob_aggregate: bootstrap_stats of each row column over ok rows -> (n_cols, 4) array of
    (std_err, p_value, ci_lower, ci_upper)."""
    rows = np.ascontiguousarray(rows, dtype=np.float64)
    ok = np.ascontiguousarray(ok, dtype=np.uint8)
    cols = np.ascontiguousarray(cols, dtype=np.int32)
    out = np.empty((len(cols), 4))
    N.check(N.lib().ob_aggregate(_dp(rows), ok.ctypes.data_as(C.POINTER(C.c_uint8)), len(ok), rows.shape[1],
                                 _ip(cols), len(cols), _dp(out)))
    return out


def rif(y, quantile: float):
    """math/rif.rs:14-88 via the native routine."""
    y = np.ascontiguousarray(y, dtype=np.float64)
    out = np.empty_like(y)
    N.check(N.lib().ob_rif(_dp(y), len(y), float(quantile), _dp(out)))
    return out
