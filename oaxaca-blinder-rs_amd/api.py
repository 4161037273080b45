"""Python surface of the engine, mirroring the reference's public API for the bootstrap path:

* ``OaxacaBuilder``  -- builder.rs:37-757 (setters, run, decompose_quantile, get_data_matrices)
* ``OaxacaBlinder``  -- the pyo3 class declared in python.rs:193-276 (fit, fit_quantile,
  optimize_budget); ``bootstrap_reps`` defaults to 100 and the reference coefficients to the
  builder default GroupA, as there.
* ``OaxacaResults`` / ``TwoFoldResults`` / ``DecompositionDetail`` / ``ComponentResult`` --
  types.rs:8-47,160-180 (field names and order are the API).

Every compute call goes through the C ABI into the HIP engine; there is no CPU path.
"""
from __future__ import annotations

import ctypes as C
import enum
import json
from dataclasses import dataclass, field

import numpy as np

from . import _native as N
from .frame import Frame


class ReferenceCoefficients(enum.IntEnum):
    """decomposition.rs:5-20"""
    GroupA = 0
    GroupB = 1
    Pooled = 2
    Weighted = 3
    Cotton = 4
    Neumark = 5


@dataclass
class ComponentResult:
    name: str
    estimate: float
    std_err: float
    t_stat: float
    p_value: float
    ci_lower: float
    ci_upper: float

    def __repr__(self):
        return f"ComponentResult(name={self.name}, estimate={self.estimate})"


@dataclass
class TwoFoldResults:
    aggregate: list
    detailed_explained: list
    detailed_unexplained: list
    detailed_selection: list


@dataclass
class DecompositionDetail:
    aggregate: list
    detailed: list


@dataclass
class BudgetAdjustment:
    index: int
    original_residual: float
    adjustment: float


@dataclass
class OaxacaResults:
    total_gap: float
    two_fold: TwoFoldResults
    three_fold: DecompositionDetail
    n_a: int
    n_b: int
    residuals: np.ndarray
    xa_mean: np.ndarray = field(repr=False)
    xb_mean: np.ndarray = field(repr=False)
    beta_star: np.ndarray = field(repr=False)
    n_failed: int = 0

    def explained(self):
        return next((c for c in self.two_fold.aggregate if c.name == "explained"), None)

    def unexplained(self):
        return next((c for c in self.two_fold.aggregate if c.name == "unexplained"), None)

    def get_summary_table(self):
        return [(c.name, c) for c in self.two_fold.aggregate]

    def get_detailed_table(self):
        m = {}
        for c in self.two_fold.detailed_explained:
            m.setdefault(c.name, [0.0, 0.0])[0] = c.estimate
        for c in self.two_fold.detailed_unexplained:
            m.setdefault(c.name, [0.0, 0.0])[1] = c.estimate
        return [(k, v[0], v[1]) for k, v in m.items()]

    def optimize_budget(self, budget: float, target_gap: float):
        """types.rs:98-156 (greedy raises for the most negative group-B residuals)."""
        if self.total_gap <= target_gap:
            return []
        needed = (self.total_gap - target_gap) * self.n_b
        eff = min(budget, needed)
        cand = sorted(((i, r) for i, r in enumerate(self.residuals) if r < 0.0), key=lambda t: t[1])
        out, spent = [], 0.0
        for idx, res in cand:
            if spent >= eff:
                break
            raise_ = min(-res, eff - spent)
            if raise_ > 1e-9:
                out.append(BudgetAdjustment(idx, float(res), float(raise_)))
                spent += raise_
        return out

    def to_json(self) -> str:
        def comp(c):
            return c.__dict__

        def fix(v):  # serde_json writes non-finite floats as null
            return v if isinstance(v, str) or np.isfinite(v) else None

        d = {
            "total_gap": self.total_gap,
            "two_fold": {k: [{kk: fix(vv) for kk, vv in comp(c).items()} for c in getattr(self.two_fold, k)]
                         for k in ("aggregate", "detailed_explained", "detailed_unexplained", "detailed_selection")},
            "three_fold": {k: [{kk: fix(vv) for kk, vv in comp(c).items()} for c in getattr(self.three_fold, k)]
                           for k in ("aggregate", "detailed")},
            "n_a": self.n_a,
            "n_b": self.n_b,
            "residuals": [fix(float(v)) for v in self.residuals],
        }
        return json.dumps(d)

    def summary(self) -> str:
        """display.rs:9-82 (plain-text tables)."""
        lines = ["Oaxaca-Blinder Decomposition Results", "=" * 40,
                 f"Group A (Advantaged): {self.n_a} observations",
                 f"Group B (Reference):  {self.n_b} observations",
                 f"Total Gap: {self.total_gap:.4f}", ""]

        def table(title, comps, first="Component"):
            lines.append(title)
            lines.append(f"{first:<28} {'Estimate':>10} {'Std. Err.':>10} {'p-value':>8}  95% CI")
            for c in comps:
                lines.append(f"{c.name:<28} {c.estimate:>10.4f} {c.std_err:>10.4f} {c.p_value:>8.4f}"
                             f"  [{c.ci_lower:.3f}, {c.ci_upper:.3f}]")
            lines.append("")

        table("Two-Fold Decomposition", self.two_fold.aggregate)
        table("Detailed Decomposition (Explained)", self.two_fold.detailed_explained, "Variable")
        table("Detailed Decomposition (Unexplained)", self.two_fold.detailed_unexplained, "Variable")
        text = "\n".join(lines)
        print(text)
        return text

    def interpret(self) -> str:
        """python.rs:155-185"""
        e = self.explained().estimate if self.explained() else 0.0
        u = self.unexplained().estimate if self.unexplained() else 0.0
        t = self.total_gap
        return (f"The total gap is {t:.4f}. \n{e / t * 100:.1f}% of this gap is explained by differences in "
                f"endowments (observables), while {u / t * 100:.1f}% is unexplained (coefficients/discrimination).")


def _results_from_c(handle) -> OaxacaResults:
    lib = N.lib()

    def table(t):
        out = []
        for i in range(lib.ob_results_count(handle, t)):
            c = N.ob_component()
            N.check(lib.ob_results_component(handle, t, i, C.byref(c)))
            out.append(ComponentResult(c.name.decode(), c.estimate, c.std_err, c.t_stat, c.p_value,
                                       c.ci_lower, c.ci_upper))
        return out

    def vec(w):
        ptr = C.POINTER(C.c_double)()
        n = C.c_int64()
        N.check(lib.ob_results_vector(handle, w, C.byref(ptr), C.byref(n)))
        return np.ctypeslib.as_array(ptr, shape=(n.value,)).copy() if n.value else np.zeros(0)

    try:
        return OaxacaResults(
            total_gap=lib.ob_results_total_gap(handle),
            two_fold=TwoFoldResults(table(N.OB_TABLE_TWO_FOLD), table(N.OB_TABLE_DETAILED_EXPLAINED),
                                    table(N.OB_TABLE_DETAILED_UNEXPLAINED), table(N.OB_TABLE_DETAILED_SELECTION)),
            three_fold=DecompositionDetail(table(N.OB_TABLE_THREE_FOLD), []),
            n_a=int(lib.ob_results_n_a(handle)), n_b=int(lib.ob_results_n_b(handle)),
            residuals=vec(N.OB_VEC_RESIDUALS), xa_mean=vec(N.OB_VEC_XA_MEAN), xb_mean=vec(N.OB_VEC_XB_MEAN),
            beta_star=vec(N.OB_VEC_BETA_STAR), n_failed=int(lib.ob_results_n_failed(handle)))
    finally:
        lib.ob_results_free(handle)


def parse_formula(formula: str):
    """formula.rs:12-58: 'y ~ a + b + C(cat)' -> (outcome, predictors, categorical)."""
    parts = formula.split("~")
    if len(parts) != 2:
        raise N.OaxacaError(N.OB_E_GROUP, "Invalid group variable: Invalid formula format. Expected "
                                          f"'outcome ~ predictors', got '{formula}'")
    outcome = parts[0].strip()
    if not outcome:
        raise N.OaxacaError(N.OB_E_GROUP, "Invalid group variable: Outcome variable is missing")
    preds, cats = [], []
    for term in parts[1].split("+"):
        term = term.strip()
        if not term:
            continue
        if term.startswith("C(") and term.endswith(")"):
            cats.append(term[2:-1].strip())
        elif term.startswith("factor(") and term.endswith(")"):
            cats.append(term[7:-1].strip())
        else:
            preds.append(term)
    if not preds and not cats:
        raise N.OaxacaError(N.OB_E_GROUP, "Invalid group variable: No predictors specified")
    return outcome, preds, cats


def _strs(names):
    arr = (C.c_char_p * max(len(names), 1))(*[n.encode() for n in names])
    return C.cast(arr, C.POINTER(C.c_char_p)), arr


class OaxacaBuilder:
    """builder.rs:37-757. Defaults: bootstrap_reps 20, reference coefficients GroupA."""

    def __init__(self, dataframe, outcome: str, group: str, reference_group: str):
        self._frame = dataframe if isinstance(dataframe, Frame) else Frame(dataframe)
        self.outcome, self.group, self.reference_group = outcome, group, reference_group
        self._predictors: list[str] = []
        self._categorical: list[str] = []
        self._bootstrap_reps = 20
        self._ref = ReferenceCoefficients.GroupA
        self._normalize: list[str] = []
        self._weights: str | None = None
        self._selection: str | None = None
        self._selection_predictors: list[str] = []
        self._seed: int | None = None
        self._device: int | None = None
        self._ctx = None  # an explicit ob_ctx (distributed.fit_sharded's rank context)

    @classmethod
    def from_formula(cls, dataframe, formula: str, group: str, reference_group: str):
        outcome, preds, cats = parse_formula(formula)
        b = cls(dataframe, outcome, group, reference_group)
        b._predictors, b._categorical = preds, cats
        return b

    def predictors(self, names):
        self._predictors = [str(n) for n in names]
        return self

    def categorical_predictors(self, names):
        self._categorical = [str(n) for n in names]
        return self

    def bootstrap_reps(self, reps: int):
        self._bootstrap_reps = int(reps)
        return self

    def reference_coefficients(self, ref):
        self._ref = ReferenceCoefficients(ref)
        return self

    def normalize(self, names):
        self._normalize = [str(n) for n in names]
        return self

    def weights(self, name: str):
        self._weights = name
        return self

    def heckman_selection(self, outcome: str, predictors):
        self._selection = outcome
        self._selection_predictors = list(predictors)
        return self

    def seed(self, seed: int | None):
        """Extension: fix the OBRS-3 stream (the reference is unseeded; None = fresh entropy)."""
        self._seed = None if seed is None else int(seed) & ((1 << 64) - 1)
        return self

    def device(self, device: int | None):
        self._device = device
        return self

    def _config(self):
        keep = []
        cfg = N.ob_builder_config()
        cfg.outcome, cfg.group, cfg.reference_group = (self.outcome.encode(), self.group.encode(),
                                                       self.reference_group.encode())
        for attr, names in (("predictors", self._predictors), ("categorical", self._categorical),
                            ("normalize", self._normalize)):
            ptr, arr = _strs(names)
            keep.append(arr)
            setattr(cfg, attr, ptr)
            setattr(cfg, "n_" + attr if attr != "categorical" else "n_categorical", len(names))
        cfg.n_predictors = len(self._predictors)
        cfg.n_normalize = len(self._normalize)
        cfg.weights = self._weights.encode() if self._weights else None
        cfg.selection_outcome = self._selection.encode() if self._selection else None
        ptr, arr = _strs(self._selection_predictors)
        keep.append(arr)
        cfg.selection_predictors = ptr
        cfg.n_selection_predictors = len(self._selection_predictors)
        cfg.bootstrap_reps = self._bootstrap_reps
        cfg.reference_coeffs = int(self._ref)
        cfg.has_seed = 0 if self._seed is None else 1
        cfg.seed = 0 if self._seed is None else self._seed
        return cfg, keep

    def get_data_matrices(self):
        """builder.rs:252-291 -> (X_A, y_A, X_B, y_B, names); X includes the intercept column."""
        lib = N.lib()
        cols, ncol, nrow = self._frame.as_c()
        cfg, keep = self._config()
        h = C.c_void_p()
        N.check(lib.ob_builder_data_matrices(cols, ncol, nrow, C.byref(cfg), C.byref(h)))
        try:
            na, nb, k = C.c_int64(), C.c_int64(), C.c_int32()
            N.check(lib.ob_matrices_dims(h, C.byref(na), C.byref(nb), C.byref(k)))
            ptrs = [C.POINTER(C.c_double)() for _ in range(4)]
            N.check(lib.ob_matrices_get(h, *[C.byref(p) for p in ptrs]))

            def mat(p, n, kk):
                if n * kk == 0:
                    return np.zeros((n, kk))
                return np.ctypeslib.as_array(p, shape=(kk, n)).T.copy()

            xa, xb = mat(ptrs[0], na.value, k.value), mat(ptrs[2], nb.value, k.value)
            ya = np.ctypeslib.as_array(ptrs[1], shape=(na.value,)).copy() if na.value else np.zeros(0)
            yb = np.ctypeslib.as_array(ptrs[3], shape=(nb.value,)).copy() if nb.value else np.zeros(0)
            names = [lib.ob_matrices_name(h, i).decode() for i in range(k.value)]
            return xa, ya, xb, yb, names
        finally:
            lib.ob_matrices_free(h)

    def run(self) -> OaxacaResults:
        """builder.rs:787-951 on the MI355X engine."""
        lib = N.lib()
        cols, ncol, nrow = self._frame.as_c()
        cfg, keep = self._config()
        h = C.c_void_p()
        N.check(lib.ob_builder_run(N.context(self._device), cols, ncol, nrow, C.byref(cfg), C.byref(h)))
        return _results_from_c(h)

    def decompose_quantile(self, quantile: float) -> OaxacaResults:
        """builder.rs:711-757: RIF-regression decomposition at ``quantile``."""
        lib = N.lib()
        cols, ncol, nrow = self._frame.as_c()
        cfg, keep = self._config()
        h = C.c_void_p()
        N.check(lib.ob_builder_decompose_quantile(N.context(self._device), cols, ncol, nrow, C.byref(cfg),
                                                  float(quantile), C.byref(h)))
        return _results_from_c(h)

    def decompose_quantiles(self, quantiles) -> list:
        """RIF decompositions at several quantiles in one run: one panel
        whose outcomes are the RIF columns, so every replicate's resample and Gram pass serve all
        quantiles. Element t equals ``decompose_quantile(quantiles[t])`` bitwise (same seed)."""
        lib = N.lib()
        taus = np.ascontiguousarray(quantiles, dtype=np.float64)
        if taus.ndim != 1 or taus.size == 0:
            raise ValueError("quantiles must be a non-empty 1-D sequence")
        cols, ncol, nrow = self._frame.as_c()
        cfg, keep = self._config()
        hs = (C.c_void_p * taus.size)()
        N.check(lib.ob_builder_decompose_quantiles(N.context(self._device), cols, ncol, nrow, C.byref(cfg),
                                                   taus.ctypes.data_as(C.POINTER(C.c_double)), int(taus.size),
                                                   C.cast(hs, C.POINTER(C.c_void_p))))
        return [_results_from_c(C.c_void_p(h)) for h in hs]

    def prepare(self) -> "PreparedRun":
        """clean/dummies/split/upload/point estimate once; replicate ranges run separately
        (the multi-GPU path in ``distributed.py``)."""
        lib = N.lib()
        cols, ncol, nrow = self._frame.as_c()
        cfg, keep = self._config()
        h = C.c_void_p()
        ctx = self._ctx if self._ctx is not None else N.context(self._device)
        N.check(lib.ob_builder_prepare(ctx, cols, ncol, nrow, C.byref(cfg), C.byref(h)))
        return PreparedRun(h, self._bootstrap_reps, N.resolve_device(self._device))


class PreparedRun:
    """An ``ob_prepared`` handle: panel resident in HBM + point estimate."""

    def __init__(self, handle, reps: int, device: int = 0):
        self._h = handle
        self.bootstrap_reps = reps
        self.device = device  # the GPU holding the panel
        self.row_len = N.lib().ob_prepared_row_len(handle)
        self.seed = int(N.lib().ob_prepared_seed(handle))

    def boot(self, first_rep: int, n_reps: int):
        rows = np.empty((n_reps, self.row_len), dtype=np.float64)
        ok = np.zeros(n_reps, dtype=np.uint8)
        if n_reps:
            N.check(N.lib().ob_prepared_boot(self._h, first_rep, n_reps,
                                             rows.ctypes.data_as(C.POINTER(C.c_double)),
                                             ok.ctypes.data_as(C.POINTER(C.c_uint8))))
        return rows, ok

    def boot_sharded(self, first_rep: int, n_reps: int):
        """ob_prepared_boot_sharded: this rank's shard + the engine's RCCL all-gather (a rank
        context) -> all rows on every rank."""
        rows = np.empty((n_reps, self.row_len), dtype=np.float64)
        ok = np.zeros(n_reps, dtype=np.uint8)
        if n_reps:
            N.check(N.lib().ob_prepared_boot_sharded(self._h, first_rep, n_reps,
                                                     rows.ctypes.data_as(C.POINTER(C.c_double)),
                                                     ok.ctypes.data_as(C.POINTER(C.c_uint8))))
        return rows, ok

    def boot_device(self, first_rep: int, n_reps: int, rows_ptr: int, ok_ptr: int, stream: int | None):
        """Enqueue replicates into device buffers (e.g. torch tensors' data_ptr()) on ``stream``."""
        N.check(N.lib().ob_prepared_boot_device(self._h, first_rep, n_reps, C.c_void_p(rows_ptr),
                                                C.c_void_p(ok_ptr), C.c_void_p(stream or 0)))

    def sync(self):
        N.check(N.lib().ob_panel_sync(N.lib().ob_prepared_panel(self._h)))

    def timing(self) -> dict:
        t = N.ob_timing()
        N.check(N.lib().ob_panel_last_timing(N.lib().ob_prepared_panel(self._h), C.byref(t)))
        return {f: getattr(t, f) for f, _ in N.ob_timing._fields_}

    def finish(self, rows: np.ndarray, ok: np.ndarray) -> OaxacaResults:
        rows = np.ascontiguousarray(rows, dtype=np.float64)
        ok = np.ascontiguousarray(ok, dtype=np.uint8)
        h = C.c_void_p()
        N.check(N.lib().ob_prepared_finish(self._h, rows.ctypes.data_as(C.POINTER(C.c_double)),
                                           ok.ctypes.data_as(C.POINTER(C.c_uint8)), len(ok), C.byref(h)))
        return _results_from_c(h)

    def close(self):
        if self._h:
            N.lib().ob_prepared_destroy(self._h)
            self._h = None

    def __del__(self):
        try:
            self.close()
        except Exception:
            pass


class OaxacaBlinder:
    """python.rs:193-276 (declared pyo3 surface). Errors surface as RuntimeError (OaxacaError)."""

    def __init__(self, dataframe, outcome, group, reference_group, predictors, categorical_predictors=(),
                 bootstrap_reps=100, weights=None, selection_outcome=None, selection_predictors=None, *,
                 seed=None, device=None):
        self.dataframe = dataframe if isinstance(dataframe, Frame) else Frame(dataframe)
        self.outcome, self.group, self.reference_group = outcome, group, reference_group
        self.predictors = list(predictors)
        self.categorical_predictors = list(categorical_predictors)
        self.bootstrap_reps = int(bootstrap_reps)
        self.weights = weights
        self.selection_outcome = selection_outcome
        self.selection_predictors = list(selection_predictors or [])
        self.seed = seed
        self.device = device

    def _create_builder(self) -> OaxacaBuilder:
        b = OaxacaBuilder(self.dataframe, self.outcome, self.group, self.reference_group)
        b.predictors(self.predictors).categorical_predictors(self.categorical_predictors)
        b.bootstrap_reps(self.bootstrap_reps).seed(self.seed).device(self.device)
        if self.weights:
            b.weights(self.weights)
        if self.selection_outcome:
            b.heckman_selection(self.selection_outcome, self.selection_predictors)
        return b

    def fit(self) -> OaxacaResults:
        return self._create_builder().run()

    def fit_quantile(self, quantile: float) -> OaxacaResults:
        return self._create_builder().decompose_quantile(quantile)

    def fit_quantiles(self, quantiles) -> list:
        """Several RIF quantiles sharing one bootstrap (``OaxacaBuilder.decompose_quantiles``)."""
        return self._create_builder().decompose_quantiles(quantiles)

    def optimize_budget(self, budget: float, target_gap: float):
        b = self._create_builder()
        b.bootstrap_reps(0)
        res = b.run()
        return [{"index": float(a.index), "original_residual": a.original_residual, "adjustment": a.adjustment}
                for a in res.optimize_budget(budget, target_gap)]


# ---------------------------------------------------------------------------------------------
# Machado-Mata (quantile_decomposition.rs:21-522)
# ---------------------------------------------------------------------------------------------
@dataclass
class QuantileDecompositionDetail:
    total_gap: ComponentResult
    characteristics_effect: ComponentResult
    coefficients_effect: ComponentResult


@dataclass
class QuantileDecompositionResults:
    """results_by_quantile: {"q10": QuantileDecompositionDetail, ...} (:448-460)."""
    results_by_quantile: dict
    n_a: int
    n_b: int
    n_failed: int = 0

    def summary(self) -> str:  # quantile_decomposition.rs:462-505
        lines = ["Machado-Mata Quantile Decomposition Results", "=" * 44,
                 f"Group A (Advantaged): {self.n_a} observations", f"Group B (Reference):  {self.n_b} observations"]
        for key in sorted(self.results_by_quantile):
            d = self.results_by_quantile[key]
            lines += ["", f"--- Decomposition for Quantile: {key} ---",
                      f"{'Component':<16} {'Estimate':>10} {'Std. Err.':>10} {'p-value':>10}  95% CI"]
            for c in (d.total_gap, d.characteristics_effect, d.coefficients_effect):
                lines.append(f"{c.name:<16} {c.estimate:>10.4f} {c.std_err:>10.4f} {c.p_value:>10.4f}  "
                             f"[{c.ci_lower:.3f}, {c.ci_upper:.3f}]")
        text = "\n".join(lines)
        print(text)
        return text


class QuantileDecompositionBuilder:
    """quantile_decomposition.rs:21-95. Defaults: quantiles {0.1, 0.25, 0.5, 0.75, 0.9},
    simulations 200, bootstrap_reps 20. Every quantile regression of a pass runs on the GPU
    (ob_mm.hip); draws follow MM-1 (csrc/ob_spec.h) from ``seed`` instead of an unseeded RNG."""

    def __init__(self, dataframe, outcome: str, group: str, reference_group: str):
        self._frame = dataframe if isinstance(dataframe, Frame) else Frame(dataframe)
        self.outcome, self.group, self.reference_group = outcome, group, reference_group
        self._predictors: list[str] = []
        self._categorical: list[str] = []
        self._quantiles = [0.1, 0.25, 0.5, 0.75, 0.9]
        self._simulations = 200
        self._bootstrap_reps = 20
        self._seed: int | None = None
        self._device: int | None = None

    def predictors(self, names):
        self._predictors = [str(n) for n in names]
        return self

    def categorical_predictors(self, names):
        self._categorical = [str(n) for n in names]
        return self

    def quantiles(self, qs):
        self._quantiles = [float(q) for q in qs]
        return self

    def simulations(self, n: int):
        self._simulations = int(n)
        return self

    def bootstrap_reps(self, reps: int):
        self._bootstrap_reps = int(reps)
        return self

    def seed(self, seed: int | None):
        self._seed = None if seed is None else int(seed) & (2**64 - 1)
        return self

    def device(self, device: int | None):
        self._device = device
        return self

    def run(self) -> QuantileDecompositionResults:
        """quantile_decomposition.rs:281-445 on the MI355X engine."""
        lib = N.lib()
        cols, ncol, nrow = self._frame.as_c()
        cfg = N.ob_qd_config()
        cfg.outcome, cfg.group, cfg.reference_group = (self.outcome.encode(), self.group.encode(),
                                                       self.reference_group.encode())
        pp, pa = _strs(self._predictors)
        cp, ca = _strs(self._categorical)
        qs = np.ascontiguousarray(self._quantiles, dtype=np.float64)
        cfg.predictors, cfg.n_predictors = pp, len(self._predictors)
        cfg.categorical, cfg.n_categorical = cp, len(self._categorical)
        cfg.quantiles, cfg.n_quantiles = qs.ctypes.data_as(C.POINTER(C.c_double)), int(qs.size)
        cfg.simulations, cfg.bootstrap_reps = self._simulations, self._bootstrap_reps
        cfg.has_seed = 0 if self._seed is None else 1
        cfg.seed = 0 if self._seed is None else self._seed
        h = C.c_void_p()
        N.check(lib.ob_quantile_decomposition_run(N.context(self._device), cols, ncol, nrow, C.byref(cfg),
                                                  C.byref(h)))
        try:
            n, na, nb = C.c_int32(), C.c_int64(), C.c_int64()
            N.check(lib.ob_qd_results_dims(h, C.byref(n), C.byref(na), C.byref(nb)))
            out = {}
            for i in range(n.value):
                key = C.c_char_p()
                comps = (N.ob_component * 3)()
                N.check(lib.ob_qd_results_get(h, i, C.byref(key), comps))
                cr = [ComponentResult(c.name.decode(), c.estimate, c.std_err, c.t_stat, c.p_value, c.ci_lower,
                                      c.ci_upper) for c in comps]
                out[key.value.decode()] = QuantileDecompositionDetail(*cr)
            return QuantileDecompositionResults(out, int(na.value), int(nb.value),
                                                int(lib.ob_qd_results_n_failed(h)))
        finally:
            lib.ob_qd_results_free(h)
            del pa, ca
