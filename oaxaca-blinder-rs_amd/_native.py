"""ctypes binding of ``liboaxaca_boot.so`` (the C ABI declared in ``include/oaxaca_boot.h``).

The library is built in-tree by ``__graft_entry__.build()`` (``make -C csrc``). There is no
fallback: if the library is missing, or no MI355X is visible when a compute entry point is
called, the call raises -- the bootstrap never silently runs on the CPU.
"""
from __future__ import annotations

import contextlib
import math
import ctypes as C
import os
import threading

_HERE = os.path.dirname(os.path.abspath(__file__))
# OB_LIB_PATH: an alternative build for A/B timing runs (tools/build_alt.sh); never set in tests.
LIB_PATH = os.environ.get("OB_LIB_PATH") or os.path.join(_HERE, "liboaxaca_boot.so")

OB_OK = 0
OB_E_POLARS, OB_E_COLUMN, OB_E_GROUP, OB_E_LINALG, OB_E_DIAG, OB_E_INSUFFICIENT = 1, 2, 3, 4, 5, 6
OB_E_HIP, OB_E_INVALID, OB_E_UNSUPPORTED, OB_E_OVERFLOW, OB_E_RCCL = 7, 8, 9, 10, 11

OB_COL_F64, OB_COL_I64, OB_COL_STR = 0, 1, 2
OB_TABLE_TWO_FOLD, OB_TABLE_DETAILED_EXPLAINED, OB_TABLE_DETAILED_UNEXPLAINED = 0, 1, 2
OB_TABLE_DETAILED_SELECTION, OB_TABLE_THREE_FOLD = 3, 4
OB_VEC_RESIDUALS, OB_VEC_XA_MEAN, OB_VEC_XB_MEAN, OB_VEC_BETA_STAR = 0, 1, 2, 3

# Every exported entry point of include/oaxaca_boot.h (tests/test_capi_host.py checks both ways).
EXPORTED = (
    "ob_last_error", "ob_version", "ob_device_count", "ob_ctx_create", "ob_ctx_destroy",
    "ob_panel_create", "ob_panel_destroy", "ob_panel_row_len", "ob_panel_k", "ob_panel_n_base", "ob_panel_n_y",
    "ob_point_estimate", "ob_boot_run", "ob_boot_run_device", "ob_panel_last_timing", "ob_panel_sync",
    "ob_bootstrap_stats", "ob_aggregate", "ob_rif",
    "ob_builder_prepare", "ob_prepared_row_len", "ob_prepared_n_y", "ob_prepared_seed", "ob_prepared_panel",
    "ob_prepared_boot", "ob_prepared_boot_device", "ob_prepared_finish", "ob_prepared_destroy",
    "ob_builder_run", "ob_builder_decompose_quantile", "ob_builder_decompose_quantiles",
    "ob_builder_data_matrices", "ob_csv_read", "ob_csv_dims", "ob_csv_column", "ob_csv_free",
    "ob_results_total_gap", "ob_results_n_a", "ob_results_n_b", "ob_results_n_failed",
    "ob_results_count", "ob_results_component", "ob_results_vector", "ob_results_free",
    "ob_matrices_dims", "ob_matrices_get", "ob_matrices_name", "ob_matrices_free",
    "ob_mm_run", "ob_quantile_decomposition_run", "ob_qd_results_dims", "ob_qd_results_get",
    "ob_qd_results_n_failed", "ob_qd_results_free",
    "ob_get_unique_id", "ob_ctx_create_rank", "ob_ctx_rank", "ob_boot_run_sharded", "ob_boot_run_sharded_device",
    "ob_boot_run_multi", "ob_debug_counts", "ob_prepared_boot_sharded", "ob_debug_gram",
    "ob_debug_gram_exceptions", "ob_panel_set_gather_columns", "ob_debug_shard_sim", "ob_debug_mm_fail",
    "ob_debug_chunks", "ob_debug_mm_betas", "ob_set_option", "ob_get_option", "ob_tuning_build",
    "ob_debug_normal",
)


class OaxacaError(RuntimeError):
    """Raised for any non-OB_OK return; ``code`` is the OB_E_* value (error.rs variants)."""

    def __init__(self, code: int, message: str):
        super().__init__(message)
        self.code = code


class ob_group_desc(C.Structure):
    _fields_ = [("n", C.c_int64), ("x", C.POINTER(C.c_double)), ("ldx", C.c_int64),
                ("y", C.POINTER(C.c_double)), ("w", C.POINTER(C.c_double))]


class ob_panel_desc(C.Structure):
    _fields_ = [("p", C.c_int32), ("n_num", C.c_int32), ("weighted", C.c_int32),
                ("a", ob_group_desc), ("b", ob_group_desc), ("n_norm", C.c_int32),
                ("norm_start", C.POINTER(C.c_int32)), ("norm_idx", C.POINTER(C.c_int32)),
                ("norm_m", C.POINTER(C.c_int32)), ("pooled_start", C.POINTER(C.c_int32)),
                ("pooled_idx", C.POINTER(C.c_int32)), ("has_base", C.POINTER(C.c_int32)),
                ("n_y", C.c_int32), ("heckman", C.c_int32), ("n_zsel", C.c_int32),
                ("za", C.POINTER(C.c_double)), ("zb", C.POINTER(C.c_double)),
                ("sa", C.POINTER(C.c_double)), ("sb", C.POINTER(C.c_double))]


class ob_timing(C.Structure):
    _fields_ = [("level1_ms", C.c_double), ("gram_ms", C.c_double), ("reduce_ms", C.c_double),
                ("solve_ms", C.c_double), ("gram_launches", C.c_int32), ("chunks", C.c_int32),
                ("blocks", C.c_int32), ("counts_ms", C.c_double),
                ("heckman_ms", C.c_double), ("probit_iterations", C.c_int32),
                ("mm_assemble_ms", C.c_double), ("mm_fit_rows", C.c_double), ("mm_iterations", C.c_int32),
                ("mm_ms", C.c_double), ("gather_ms", C.c_double), ("gram_path", C.c_int32),
                ("probit_ms", C.c_double), ("probit_launches", C.c_int32), ("heck_sums_ms", C.c_double),
                ("mm_reduced", C.c_int32), ("mm_retried", C.c_int64), ("prep_ms", C.c_double),
                ("oz_exceptions", C.c_int32), ("oz_bits", C.c_int32), ("oz_tiles6", C.c_int32),
                ("oz_tiles", C.c_int32), ("oz_wide", C.c_int32)]


class ob_unique_id(C.Structure):
    _fields_ = [("internal", C.c_uint8 * 128)]  # raw bytes (a c_char array would stop at NUL)


class ob_column(C.Structure):
    _fields_ = [("name", C.c_char_p), ("kind", C.c_int32), ("f64", C.POINTER(C.c_double)),
                ("i64", C.POINTER(C.c_int64)), ("str", C.POINTER(C.c_char_p)),
                ("valid", C.POINTER(C.c_uint8))]


class ob_builder_config(C.Structure):
    _fields_ = [("outcome", C.c_char_p), ("group", C.c_char_p), ("reference_group", C.c_char_p),
                ("predictors", C.POINTER(C.c_char_p)), ("n_predictors", C.c_int32),
                ("categorical", C.POINTER(C.c_char_p)), ("n_categorical", C.c_int32),
                ("normalize", C.POINTER(C.c_char_p)), ("n_normalize", C.c_int32),
                ("weights", C.c_char_p), ("selection_outcome", C.c_char_p),
                ("bootstrap_reps", C.c_uint64), ("reference_coeffs", C.c_int32),
                ("has_seed", C.c_int32), ("seed", C.c_uint64),
                ("selection_predictors", C.POINTER(C.c_char_p)), ("n_selection_predictors", C.c_int32)]


class ob_qd_config(C.Structure):
    _fields_ = [("outcome", C.c_char_p), ("group", C.c_char_p), ("reference_group", C.c_char_p),
                ("predictors", C.POINTER(C.c_char_p)), ("n_predictors", C.c_int32),
                ("categorical", C.POINTER(C.c_char_p)), ("n_categorical", C.c_int32),
                ("quantiles", C.POINTER(C.c_double)), ("n_quantiles", C.c_int32),
                ("simulations", C.c_int32), ("bootstrap_reps", C.c_uint64),
                ("has_seed", C.c_int32), ("seed", C.c_uint64)]


class ob_component(C.Structure):
    _fields_ = [("name", C.c_char_p), ("estimate", C.c_double), ("std_err", C.c_double),
                ("t_stat", C.c_double), ("p_value", C.c_double), ("ci_lower", C.c_double),
                ("ci_upper", C.c_double)]


_P = C.c_void_p
_D = C.POINTER(C.c_double)
_U8 = C.POINTER(C.c_uint8)
_SIGS = {
    "ob_last_error": (C.c_char_p, []),
    "ob_version": (C.c_char_p, []),
    "ob_device_count": (C.c_int, [C.POINTER(C.c_int)]),
    "ob_ctx_create": (C.c_int, [C.c_int, C.POINTER(_P)]),
    "ob_ctx_destroy": (None, [_P]),
    "ob_panel_create": (C.c_int, [_P, C.POINTER(ob_panel_desc), C.POINTER(_P)]),
    "ob_panel_destroy": (None, [_P]),
    "ob_panel_row_len": (C.c_int, [_P]),
    "ob_panel_k": (C.c_int, [_P]),
    "ob_panel_n_base": (C.c_int, [_P]),
    "ob_panel_n_y": (C.c_int, [_P]),
    "ob_point_estimate": (C.c_int, [_P, C.c_int, _D, _D]),
    "ob_boot_run": (C.c_int, [_P, C.c_uint64, C.c_uint64, C.c_uint64, C.c_int, _D, _U8]),
    "ob_boot_run_device": (C.c_int, [_P, C.c_uint64, C.c_uint64, C.c_uint64, C.c_int, _P, _P, _P]),
    "ob_panel_last_timing": (C.c_int, [_P, C.POINTER(ob_timing)]),
    "ob_panel_sync": (C.c_int, [_P]),
    "ob_bootstrap_stats": (C.c_int, [_D, C.c_int64, C.c_double, _D]),
    "ob_aggregate": (C.c_int, [_D, _U8, C.c_uint64, C.c_int32, C.POINTER(C.c_int32), C.c_int32, _D]),
    "ob_rif": (C.c_int, [_D, C.c_int64, C.c_double, _D]),
    "ob_builder_prepare": (C.c_int, [_P, C.POINTER(ob_column), C.c_int32, C.c_int64,
                                     C.POINTER(ob_builder_config), C.POINTER(_P)]),
    "ob_prepared_row_len": (C.c_int, [_P]),
    "ob_prepared_n_y": (C.c_int, [_P]),
    "ob_prepared_seed": (C.c_uint64, [_P]),
    "ob_prepared_panel": (_P, [_P]),
    "ob_prepared_boot": (C.c_int, [_P, C.c_uint64, C.c_uint64, _D, _U8]),
    "ob_prepared_boot_device": (C.c_int, [_P, C.c_uint64, C.c_uint64, _P, _P, _P]),
    "ob_prepared_finish": (C.c_int, [_P, _D, _U8, C.c_uint64, C.POINTER(_P)]),
    "ob_prepared_destroy": (None, [_P]),
    "ob_builder_run": (C.c_int, [_P, C.POINTER(ob_column), C.c_int32, C.c_int64,
                                 C.POINTER(ob_builder_config), C.POINTER(_P)]),
    "ob_builder_decompose_quantile": (C.c_int, [_P, C.POINTER(ob_column), C.c_int32, C.c_int64,
                                                C.POINTER(ob_builder_config), C.c_double, C.POINTER(_P)]),
    "ob_builder_decompose_quantiles": (C.c_int, [_P, C.POINTER(ob_column), C.c_int32, C.c_int64,
                                                 C.POINTER(ob_builder_config), _D, C.c_int32, C.POINTER(_P)]),
    "ob_builder_data_matrices": (C.c_int, [C.POINTER(ob_column), C.c_int32, C.c_int64,
                                           C.POINTER(ob_builder_config), C.POINTER(_P)]),
    "ob_csv_read": (C.c_int, [C.c_char_p, C.POINTER(_P)]),
    "ob_csv_dims": (C.c_int, [_P, C.POINTER(C.c_int64), C.POINTER(C.c_int32)]),
    "ob_csv_column": (C.c_int, [_P, C.c_int32, C.POINTER(ob_column)]),
    "ob_csv_free": (None, [_P]),
    "ob_results_total_gap": (C.c_double, [_P]),
    "ob_results_n_a": (C.c_int64, [_P]),
    "ob_results_n_b": (C.c_int64, [_P]),
    "ob_results_n_failed": (C.c_int64, [_P]),
    "ob_results_count": (C.c_int, [_P, C.c_int32]),
    "ob_results_component": (C.c_int, [_P, C.c_int32, C.c_int32, C.POINTER(ob_component)]),
    "ob_results_vector": (C.c_int, [_P, C.c_int32, C.POINTER(_D), C.POINTER(C.c_int64)]),
    "ob_results_free": (None, [_P]),
    "ob_matrices_dims": (C.c_int, [_P, C.POINTER(C.c_int64), C.POINTER(C.c_int64), C.POINTER(C.c_int32)]),
    "ob_matrices_get": (C.c_int, [_P, C.POINTER(_D), C.POINTER(_D), C.POINTER(_D), C.POINTER(_D)]),
    "ob_matrices_name": (C.c_char_p, [_P, C.c_int32]),
    "ob_matrices_free": (None, [_P]),
    "ob_mm_run": (C.c_int, [_P, C.c_uint64, C.c_int32, _D, C.c_int32, C.c_uint64, C.c_uint64, C.c_int32, _D, _U8]),
    "ob_quantile_decomposition_run": (C.c_int, [_P, C.POINTER(ob_column), C.c_int32, C.c_int64,
                                                C.POINTER(ob_qd_config), C.POINTER(_P)]),
    "ob_qd_results_dims": (C.c_int, [_P, C.POINTER(C.c_int32), C.POINTER(C.c_int64), C.POINTER(C.c_int64)]),
    "ob_qd_results_get": (C.c_int, [_P, C.c_int32, C.POINTER(C.c_char_p), C.POINTER(ob_component)]),
    "ob_qd_results_n_failed": (C.c_int64, [_P]),
    "ob_qd_results_free": (None, [_P]),
    "ob_get_unique_id": (C.c_int, [C.POINTER(ob_unique_id)]),
    "ob_ctx_create_rank": (C.c_int, [C.c_int, C.c_int, C.c_int, C.POINTER(ob_unique_id), C.POINTER(_P)]),
    "ob_ctx_rank": (C.c_int, [_P, C.POINTER(C.c_int), C.POINTER(C.c_int)]),
    "ob_boot_run_sharded": (C.c_int, [_P, C.c_uint64, C.c_uint64, C.c_uint64, C.c_int, _D, _U8]),
    "ob_boot_run_sharded_device": (C.c_int, [_P, C.c_uint64, C.c_uint64, C.c_uint64, C.c_int, _P, _P, _P]),
    "ob_boot_run_multi": (C.c_int, [C.POINTER(_P), C.c_int, C.c_uint64, C.c_uint64, C.c_uint64, C.c_int, _D, _U8]),
    "ob_debug_gram": (C.c_int, [_P, C.c_int, C.c_uint64, C.c_uint64, C.c_uint32, _D]),
    "ob_debug_mm_fail": (C.c_int, [_P, _U8, C.c_int32]),
    "ob_panel_set_gather_columns": (C.c_int, [_P, C.POINTER(C.c_int32), C.c_int32]),
    "ob_debug_shard_sim": (C.c_int, [_P, C.c_int, C.c_int, C.c_uint64, C.c_uint64, C.c_uint64, C.c_int, _D, _U8]),
    "ob_debug_gram_exceptions": (C.c_int, [_P, C.POINTER(C.c_int32), C.POINTER(C.c_int32),
                                           C.POINTER(C.c_uint32), C.c_int32]),
    "ob_prepared_boot_sharded": (C.c_int, [_P, C.c_uint64, C.c_uint64, _D, _U8]),
    "ob_debug_counts": (C.c_int, [_P, C.c_uint64, C.c_uint64, C.c_uint32, C.c_int, C.POINTER(C.c_uint32), _U8]),
    "ob_debug_chunks": (C.c_int, [_P, C.POINTER(C.c_uint32), C.c_int32, C.POINTER(C.c_int32)]),
    "ob_debug_mm_betas": (C.c_int, [_P, C.c_uint64, C.c_int32, C.c_uint64, _D, _U8]),
    "ob_set_option": (C.c_int, [C.c_char_p, C.c_double]),
    "ob_get_option": (C.c_int, [C.c_char_p, C.POINTER(C.c_double)]),
    "ob_tuning_build": (C.c_int, []),
    "ob_debug_normal": (C.c_int, [C.c_int, _D, C.c_int64, _D, _D]),
}

_lib = None
_lib_lock = threading.Lock()


def _share_torch_runtime():
    """PyTorch-ROCm bundles its own libamdhip64.so.7. Loading ours first would put two HIP
    runtimes in the process (torch's stream/allocations would then be foreign handles), so when
    torch is installed it is imported first and the engine binds to its runtime (same soname)."""
    if os.environ.get("OB_NO_TORCH") == "1":
        return
    try:
        import torch  # noqa: F401
    except ImportError:
        pass


def lib() -> C.CDLL:
    """Load the engine library once; raise loudly if it was not built."""
    global _lib
    if _lib is None:
        _share_torch_runtime()
    with _lib_lock:
        if _lib is None:
            if not os.path.exists(LIB_PATH):
                raise ImportError(
                    f"{LIB_PATH} is missing: build it with __graft_entry__.build() "
                    "(make -C oaxaca-blinder-rs_amd/csrc). There is no CPU fallback.")
            handle = C.CDLL(LIB_PATH)
            for name, (res, args) in _SIGS.items():
                fn = getattr(handle, name)
                fn.restype = res
                fn.argtypes = args
            _lib = handle
    return _lib


def check(rc: int) -> None:
    if rc != OB_OK:
        msg = lib().ob_last_error().decode("utf-8", "replace")
        raise OaxacaError(rc, msg)


_ctx_cache: dict = {}


def resolve_device(device: int | None = None) -> int:
    """The GPU a ``device=None`` call uses: OB_DEVICE, else LOCAL_RANK, else 0."""
    if device is None:
        device = int(os.environ.get("OB_DEVICE", os.environ.get("LOCAL_RANK", "0")))
    return int(device)


def context(device: int | None = None) -> C.c_void_p:
    """Process-wide ob_ctx for ``device`` (default: resolve_device())."""
    device = resolve_device(device)
    with _lib_lock:
        ctx = _ctx_cache.get(device)
    if ctx is None:
        ctx = C.c_void_p()
        check(lib().ob_ctx_create(device, C.byref(ctx)))
        with _lib_lock:
            _ctx_cache[device] = ctx
    return ctx


def unique_id() -> bytes:
    """ncclGetUniqueId through the engine (rank 0 calls it and broadcasts the 128 bytes)."""
    u = ob_unique_id()
    check(lib().ob_get_unique_id(C.byref(u)))
    return C.string_at(C.addressof(u), C.sizeof(u))


_rank_ctx_cache: dict = {}


def rank_context(device: int, rank: int, world: int, uid: bytes) -> C.c_void_p:
    """An ob_ctx that is rank ``rank`` of ``world`` on an RCCL communicator (ob_ctx_create_rank).
    Cached per (device, rank, world, uid); panels created in it run sharded."""
    key = (device, rank, world, bytes(uid))
    with _lib_lock:
        ctx = _rank_ctx_cache.get(key)
    if ctx is None:
        uid = bytes(uid)
        if len(uid) != C.sizeof(ob_unique_id):
            raise ValueError("a unique id is 128 bytes")
        u = ob_unique_id()
        C.memmove(C.addressof(u), uid, len(uid))
        ctx = C.c_void_p()
        check(lib().ob_ctx_create_rank(device, rank, world, C.byref(u), C.byref(ctx)))
        with _lib_lock:
            _rank_ctx_cache[key] = ctx
    return ctx


def ctx_rank(ctx) -> tuple:
    """(rank, world) of the engine's RCCL communicator in ``ctx`` (ob_ctx_rank; (0, 1) for a
    plain context)."""
    r, w = C.c_int(0), C.c_int(0)
    check(lib().ob_ctx_rank(ctx, C.byref(r), C.byref(w)))
    return r.value, w.value


def set_option(name: str, value) -> None:
    """ob_set_option: a process-wide engine switch (include/oaxaca_boot.h); None restores the default.
    The library reads no environment variable -- tests and tools set these explicitly."""
    check(lib().ob_set_option(name.encode(), float("nan") if value is None else float(value)))


def get_option(name: str):
    """ob_get_option: the value ob_set_option stored for ``name``, or None when it is unset."""
    v = C.c_double()
    check(lib().ob_get_option(name.encode(), C.byref(v)))
    return None if math.isnan(v.value) else v.value


@contextlib.contextmanager
def option(name: str, value):
    """set_option for the duration of a with-block, then back to the value it had before (so
    nested blocks and fixtures that already set the option keep their setting)."""
    prev = get_option(name)
    set_option(name, value)
    try:
        yield
    finally:
        set_option(name, prev)


def device_count() -> int:
    n = C.c_int(0)
    rc = lib().ob_device_count(C.byref(n))
    return n.value if rc == OB_OK else 0
