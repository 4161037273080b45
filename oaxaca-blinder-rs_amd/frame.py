"""Column frames for the C ABI (``ob_column``): the stand-in for the polars DataFrame that
``OaxacaBuilder::new`` receives (builder.rs:114). polars is not installed in this image, so a
frame is a ``dict`` of columns or a pandas DataFrame:

* ``float`` data -> Float64 column; ``int`` data -> Int64 (cast to f64 when used as a predictor,
  like ``to_ndarray::<Float64Type>``); ``str`` data -> String column.
* nulls: ``None`` entries of a list, masked entries of a ``numpy.ma.MaskedArray``, or pandas
  missing values (``pandas.isna``, the convention of ``polars.from_pandas``). A float NaN in a
  list or a plain ndarray is a value, not a null, as in polars.
"""
from __future__ import annotations

import ctypes as C

import numpy as np

from . import _native as N


class Frame:
    """Columns converted once to contiguous buffers; ``as_c()`` returns the ob_column array."""

    def __init__(self, data):
        self.columns: dict[str, tuple[int, object, np.ndarray | None]] = {}
        self.nrows = None
        for name, col in _iter_columns(data):
            kind, values, valid = _convert(col)
            n = len(values)
            if self.nrows is None:
                self.nrows = n
            elif n != self.nrows:
                raise ValueError(f"column '{name}' has {n} rows, expected {self.nrows}")
            self.columns[str(name)] = (kind, values, valid)
        if self.nrows is None:
            self.nrows = 0
        self._c = None
        self._keep = []

    def names(self):
        return list(self.columns)

    def as_c(self):
        if self._c is None:
            arr = (N.ob_column * max(len(self.columns), 1))()
            keep = []
            for i, (name, (kind, values, valid)) in enumerate(self.columns.items()):
                bname = name.encode()
                keep.append(bname)
                arr[i].name = bname
                arr[i].kind = kind
                if kind == N.OB_COL_F64:
                    arr[i].f64 = values.ctypes.data_as(C.POINTER(C.c_double))
                elif kind == N.OB_COL_I64:
                    arr[i].i64 = values.ctypes.data_as(C.POINTER(C.c_int64))
                else:
                    sarr = (C.c_char_p * max(len(values), 1))(*values)
                    keep.append(sarr)
                    arr[i].str = C.cast(sarr, C.POINTER(C.c_char_p))
                if valid is not None:
                    arr[i].valid = valid.ctypes.data_as(C.POINTER(C.c_uint8))
                keep.append(values)
                keep.append(valid)
            self._c = arr
            self._keep = keep
        return self._c, len(self.columns), self.nrows


def _iter_columns(data):
    if isinstance(data, Frame):
        raise TypeError("already a Frame")
    if hasattr(data, "columns") and hasattr(data, "__getitem__") and not isinstance(data, dict):
        for name in data.columns:  # pandas DataFrame
            yield name, data[name]
        return
    if isinstance(data, dict):
        yield from data.items()
        return
    raise TypeError("dataframe must be a dict of columns or a pandas DataFrame")


def _convert(col):
    valid = None
    try:
        import pandas as pd  # optional

        if isinstance(col, pd.Series):
            mask = col.isna().to_numpy()
            if col.dtype == object or pd.api.types.is_string_dtype(col.dtype):
                vals = [None if m else str(v) for v, m in zip(col.tolist(), mask)]
                return _strings(vals)
            if pd.api.types.is_integer_dtype(col.dtype) and not mask.any():
                return N.OB_COL_I64, np.ascontiguousarray(col.to_numpy(dtype=np.int64)), None
            vals = col.to_numpy(dtype=np.float64, na_value=0.0)
            valid = None if not mask.any() else (~mask).astype(np.uint8)
            return N.OB_COL_F64, np.ascontiguousarray(vals), valid
    except ImportError:
        pass
    if isinstance(col, np.ma.MaskedArray):
        mask = np.ma.getmaskarray(col)
        base = np.asarray(col.filled(0 if col.dtype.kind in "iuf" else ""))
        kind, vals, _ = _convert(base)
        if kind == N.OB_COL_STR:
            vals = [None if m else v for v, m in zip(vals, mask)]
            return N.OB_COL_STR, vals, None
        return kind, vals, (~mask).astype(np.uint8)
    if isinstance(col, np.ndarray):
        if col.dtype.kind == "f":
            return N.OB_COL_F64, np.ascontiguousarray(col, dtype=np.float64), None
        if col.dtype.kind in "iub":
            return N.OB_COL_I64, np.ascontiguousarray(col, dtype=np.int64), None
        if col.dtype.kind in "USO":
            return _strings([None if v is None else str(v) for v in col.tolist()])
        raise TypeError(f"unsupported column dtype {col.dtype}")
    vals = list(col)
    present = [v for v in vals if v is not None]
    if present and all(isinstance(v, str) for v in present):
        return _strings(vals)
    if present and not all(isinstance(v, (int, float, np.integer, np.floating, bool)) for v in present):
        raise TypeError("mixed column types")
    is_float = any(isinstance(v, (float, np.floating)) for v in present)
    nulls = np.array([v is None for v in vals], dtype=bool)
    if is_float or not present:
        arr = np.array([0.0 if v is None else float(v) for v in vals], dtype=np.float64)
        kind = N.OB_COL_F64
    else:
        arr = np.array([0 if v is None else int(v) for v in vals], dtype=np.int64)
        kind = N.OB_COL_I64
    return kind, arr, ((~nulls).astype(np.uint8) if nulls.any() else None)


def _strings(vals):
    return N.OB_COL_STR, [None if v is None else v.encode("utf-8") for v in vals], None


def read_csv(path) -> dict:
    """The reference CLI's CSV front end (main.rs:161-165, polars ``LazyCsvReader`` with a header)
    through the native reader: dtypes from the first 100 rows (i64, else f64, else str), empty
    fields are nulls (masked numeric entries / ``None`` strings). Returns a dict frame."""
    lib = N.lib()
    h = C.c_void_p()
    N.check(lib.ob_csv_read(str(path).encode(), C.byref(h)))
    try:
        nrows, ncols = C.c_int64(), C.c_int32()
        N.check(lib.ob_csv_dims(h, C.byref(nrows), C.byref(ncols)))
        n = nrows.value
        out = {}
        for j in range(ncols.value):
            col = N.ob_column()
            N.check(lib.ob_csv_column(h, j, C.byref(col)))
            valid = np.ctypeslib.as_array(col.valid, shape=(n,)).astype(bool) if n else np.zeros(0, bool)
            if col.kind == N.OB_COL_STR:
                vals = [col.str[i].decode() if valid[i] else None for i in range(n)]
            else:
                ptr = col.f64 if col.kind == N.OB_COL_F64 else col.i64
                arr = np.ctypeslib.as_array(ptr, shape=(n,)).copy() if n else np.zeros(0)
                vals = arr if valid.all() else np.ma.MaskedArray(arr, mask=~valid)
            out[col.name.decode()] = vals
        return out
    finally:
        lib.ob_csv_free(h)
