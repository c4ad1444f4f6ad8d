"""ctypes front-end of the native multi-threaded CSV reader (``csrc_host/csv_panel.cpp``)."""
from __future__ import annotations

import ctypes as C
import os

import numpy as np
import pandas as pd

from .._build import HOST_LIB_PATH, build_host

_lib = None


_warned = False


def _load_or_none():
    """The host library, or None with ONE logged warning (callers then use pandas / numpy)."""
    global _warned
    try:
        return _load()
    except Exception as e:  # missing toolchain / unbuildable: the pure-Python path still works
        if not _warned:
            import logging
            logging.getLogger("mfa").warning("native host IO unavailable (%s); using pandas", e)
            _warned = True
        return None


def _load():
    global _lib
    if _lib is None:
        if not HOST_LIB_PATH.exists():
            build_host()
        lib = C.CDLL(str(HOST_LIB_PATH))
        lib.mfa_csv_shape.argtypes = [C.c_char_p, C.POINTER(C.c_int)]
        lib.mfa_csv_shape.restype = C.c_int64
        lib.mfa_csv_parse.argtypes = [C.c_char_p, C.c_int, C.POINTER(C.c_int), C.POINTER(C.c_void_p), C.c_int]
        lib.mfa_csv_parse.restype = C.c_int64
        lib.mfa_write_matrix_csv.argtypes = [C.c_char_p, C.c_char_p, C.POINTER(C.c_char_p),
                                             C.c_longlong, C.c_longlong, C.c_void_p, C.c_int]
        lib.mfa_write_matrix_csv.restype = C.c_int
        lib.mfa_date_span.argtypes = []
        lib.mfa_date_span.restype = C.c_int64
        lib.mfa_date_mask.argtypes = [C.c_void_p, C.c_int64, C.c_void_p, C.c_int]
        lib.mfa_date_mask.restype = C.c_int
        lib.mfa_csv_parse_ix.argtypes = [C.c_char_p, C.c_int, C.POINTER(C.c_int), C.POINTER(C.c_void_p),
                                         C.c_int, C.c_int, C.c_int, C.c_void_p, C.POINTER(C.c_void_p)]
        lib.mfa_csv_parse_ix.restype = C.c_int64
        lib.mfa_mask_dates.argtypes = [C.c_void_p, C.c_void_p, C.c_int64]
        lib.mfa_mask_dates.restype = C.c_int64
        lib.mfa_row_index.argtypes = [C.c_void_p, C.c_void_p, C.c_int64, C.c_void_p, C.c_int]
        lib.mfa_row_index.restype = C.c_void_p
        lib.mfa_row_index_count.argtypes = [C.c_void_p]
        lib.mfa_row_index_count.restype = C.c_int64
        lib.mfa_row_index_get.argtypes = [C.c_void_p, C.c_void_p]
        lib.mfa_row_index_get.restype = None
        lib.mfa_row_index_free.argtypes = [C.c_void_p]
        lib.mfa_row_index_free.restype = None
        lib.mfa_shard_rows_ix.argtypes = [C.c_void_p, C.c_int64, C.c_int64, C.c_void_p, C.c_void_p,
                                          C.c_int32, C.c_int32, C.c_int64, C.c_int, C.c_void_p,
                                          C.c_void_p, C.c_int]
        lib.mfa_shard_rows_ix.restype = C.c_int64
        lib.mfa_gather_ranges.argtypes = [C.c_void_p, C.c_int64, C.c_void_p, C.c_void_p, C.c_int64,
                                          C.c_void_p, C.c_int]
        lib.mfa_gather_ranges.restype = C.c_int
        _lib = lib
    return _lib


STRING_COLS = {"stocknames", "ts_code", "industry", "l1_code", "code", "industry_names", "date",
               "trade_date"}


def read_csv(path: str, string_cols=STRING_COLS, date_cols=(), nthreads: int = 0) -> pd.DataFrame | None:
    """Columns in ``string_cols`` stay strings (dates keep their file format, as pandas does),
    ``date_cols`` become int32 YYYYMMDD, everything else float64."""
    """Parse a simple (unquoted-comma) CSV with a header into a DataFrame; None if unsupported."""
    lib = _load_or_none()
    if lib is None:
        return None
    with open(path, "rb") as fh:
        header = fh.readline().decode("utf-8-sig").strip().split(",")
    ncol = C.c_int(0)
    rows = lib.mfa_csv_shape(path.encode(), C.byref(ncol))
    if rows < 0 or ncol.value != len(header):
        return None
    types, bufs = [], []
    for name in header:
        if name in date_cols:
            types.append(2); bufs.append(np.empty(rows, dtype=np.int32))
        elif name in string_cols:
            types.append(1); bufs.append(np.zeros(rows, dtype="S16"))
        else:
            types.append(0); bufs.append(np.empty(rows, dtype=np.float64))
    t_arr = (C.c_int * len(types))(*types)
    p_arr = (C.c_void_p * len(bufs))(*[b.ctypes.data for b in bufs])
    got = lib.mfa_csv_parse(path.encode(), len(header), t_arr, p_arr, nthreads)
    if got != rows:
        bufs = [b[:got] for b in bufs]
    cols = {}
    for name, t, b in zip(header, types, bufs):
        if t == 2:
            cols[name] = b
        elif t == 1:
            u = b.astype("U16").astype(object)
            u[b == b""] = np.nan
            cols[name] = u
        else:
            cols[name] = b
    return pd.DataFrame(cols)


def read_barra_csv(path: str) -> pd.DataFrame | None:
    if os.environ.get("MFA_NO_NATIVE_IO"):
        return None
    return read_csv(path)


def _host_buffer(rows: int, dtype, pinned: bool) -> np.ndarray:
    """A numpy array of ``rows`` elements, in page-locked (pinned) host memory when ``pinned``:
    the parser writes straight into DMA-able staging buffers (no extra host copy before the
    device upload)."""
    if pinned:
        import torch
        tdt = {np.float32: torch.float32, np.float64: torch.float64, np.int32: torch.int32}.get(dtype)
        if tdt is not None:
            return torch.empty(rows, dtype=tdt, pin_memory=True).numpy()
        if dtype == "S16":
            return torch.zeros(rows * 16, dtype=torch.uint8, pin_memory=True).numpy().view("S16")
    return np.zeros(rows, dtype=dtype) if dtype == "S16" else np.empty(rows, dtype=dtype)


def read_columns(path: str, types: dict, nthreads: int = 0, pinned: bool = False,
                 index: tuple | None = None):
    """Raw columnar parse: ``types`` maps column name -> 0 float64 / 1 bytes16 / 2 int YYYYMMDD /
    3 float32 (float64 parse rounded to float32, the reference's load downcast).

    Returns ``{name: ndarray}`` (bytes columns stay ``S16``), or None if unavailable.  With
    ``pinned`` (a GPU is present) the buffers are page-locked host memory.  ``index`` = (code
    column, date column): the parser also builds the row-group index of the rows while it parses
    them (:class:`RowIndex`, under ``ROW_INDEX``; absent when the rows are not (code, date)
    sorted).
    """
    lib = _load_or_none()
    if lib is None:
        return None
    with open(path, "rb") as fh:
        header = fh.readline().decode("utf-8-sig").strip().split(",")
    ncol = C.c_int(0)
    rows = lib.mfa_csv_shape(path.encode(), C.byref(ncol))
    if rows < 0 or ncol.value != len(header):
        return None
    tl, bufs = [], []
    for name in header:
        t = types.get(name, 0)
        tl.append(t)
        dt = {1: "S16", 2: np.int32, 3: np.float32}.get(t, np.float64)
        bufs.append(_host_buffer(rows, dt, pinned))
    t_arr = (C.c_int * len(tl))(*tl)
    p_arr = (C.c_void_p * len(bufs))(*[b.ctypes.data for b in bufs])
    if index is not None and index[0] in header and index[1] in header:
        mask = np.zeros(int(lib.mfa_date_span()), np.uint8)
        h = C.c_void_p()
        got = lib.mfa_csv_parse_ix(path.encode(), len(header), t_arr, p_arr, nthreads,
                                   header.index(index[0]), header.index(index[1]),
                                   mask.ctypes.data, C.byref(h))
        out = {n: b[:got] for n, b in zip(header, bufs)}
        ix = _take_index(lib, h, mask, got)
        if ix is not None:
            out[ROW_INDEX] = ix
        return out
    got = lib.mfa_csv_parse(path.encode(), len(header), t_arr, p_arr, nthreads)
    return {n: b[:got] for n, b in zip(header, bufs)}


_NEEDS_QUOTING = set(',"\n\r')


def write_matrix_csv(path: str, values: np.ndarray, row_labels, col_labels, index_label: str = "",
                     nthreads: int = 0) -> bool:
    """Write a float32 [rows, cols] matrix with row / column labels as pandas ``to_csv`` would
    (``csrc_host/csv_write.cpp``, multi-threaded).  Returns False (nothing written) when the
    native library is unavailable or a label would need CSV quoting: the caller then uses
    pandas."""
    if os.environ.get("MFA_NO_NATIVE_IO"):
        return False
    labels = [str(x) for x in row_labels]
    cols = [str(x) for x in col_labels]
    if any(_NEEDS_QUOTING & set(x) for x in labels + cols + [index_label]):
        return False
    lib = _load_or_none()
    if lib is None:
        return False
    v = np.ascontiguousarray(values, dtype=np.float32)
    if v.shape != (len(labels), len(cols)):
        raise ValueError(f"matrix {v.shape} vs {len(labels)} x {len(cols)} labels")
    header = ",".join([index_label] + cols).encode()
    arr = (C.c_char_p * len(labels))(*[x.encode() for x in labels])
    rc = lib.mfa_write_matrix_csv(path.encode(), header, arr, v.shape[0], v.shape[1],
                                  v.ctypes.data, nthreads)
    if rc != 0:
        raise OSError(f"mfa_write_matrix_csv failed for {path}")
    return True


DATE_BASE = 19000101  # csrc_host/row_index.h: mask span [19000101, 21000101)
ROW_INDEX = "__row_index__"   # key of the RowIndex in a loader's column dict


class RowIndex:
    """Row-group index of (code, date)-sorted loader rows (csrc_host/row_index.h):
    ``seg_first`` [N] int64 first row of every stock (segment k = global stock id k, codes
    ascending), ``dates`` [D] int32 the sorted distinct trade dates, ``rows`` the row count it
    was built on (a column dict whose rows changed since no longer matches it)."""
    __slots__ = ("seg_first", "dates", "rows")

    def __init__(self, seg_first: np.ndarray, dates: np.ndarray, rows: int):
        self.seg_first, self.dates, self.rows = seg_first, dates, int(rows)


def _mask_dates(lib, mask: np.ndarray) -> np.ndarray:
    n = int(lib.mfa_mask_dates(mask.ctypes.data, None, 0))
    out = np.empty(n, np.int32)
    lib.mfa_mask_dates(mask.ctypes.data, out.ctypes.data, n)
    return out


def _take_index(lib, h, mask, rows) -> RowIndex | None:
    """RowIndex from a native index handle (freed here); None if the order check failed."""
    if not h or not h.value:
        return None
    try:
        n = int(lib.mfa_row_index_count(h))
        if n < 0:
            return None
        seg_first = np.empty(n, np.int64)
        lib.mfa_row_index_get(h, seg_first.ctypes.data)
    finally:
        lib.mfa_row_index_free(h)
    return RowIndex(seg_first, _mask_dates(lib, mask), rows)


def row_index(codes: np.ndarray, dates: np.ndarray, nthreads: int = 0) -> RowIndex | None:
    """The row-group index of loader columns from a source other than the CSV reader (one
    threaded pass over codes and dates); None when the rows are not grouped by code in ascending
    order with strictly ascending dates per stock, a date is outside 1900-2100, or the native
    library is missing."""
    lib = _load_or_none()
    if lib is None:
        return None
    c = np.ascontiguousarray(codes, dtype="S16")
    d = np.ascontiguousarray(dates, dtype=np.int32)
    if d.size == 0 or c.size != d.size:
        return None
    mask = np.zeros(int(lib.mfa_date_span()), np.uint8)
    h = C.c_void_p(lib.mfa_row_index(c.ctypes.data, d.ctypes.data, d.size, mask.ctypes.data, nthreads))
    return _take_index(lib, h, mask, d.size)


def trade_dates(dates: np.ndarray, nthreads: int = 0) -> np.ndarray | None:
    """Sorted unique YYYYMMDD trade dates of a loader column (one threaded pass, a bitmap)."""
    lib = _load_or_none()
    if lib is None:
        return None
    d = np.ascontiguousarray(dates, dtype=np.int32)
    mask = np.zeros(int(lib.mfa_date_span()), np.uint8)
    if lib.mfa_date_mask(d.ctypes.data, d.size, mask.ctypes.data, nthreads) != 0:
        return None
    return _mask_dates(lib, mask)


def shard_rows_ix(ix: RowIndex, dates: np.ndarray, end_dates: np.ndarray | None, date_lo: int,
                  date_hi: int, halo: int, nstmt: int = 4, nthreads: int = 0):
    """One rank's rows of indexed loader rows: per stock, its rows with trade date in
    [date_lo, date_hi), the ``halo`` rows before them and the statement rows of the ``nstmt``
    most recent distinct end dates before them (csrc_host/shard_rows.cpp, binary searches per
    stock).  Returns ``(ranges [n, 2] int64, seg_id [n] int32)``: the kept row ranges and the
    global stock id of each."""
    lib = _load()
    d = np.ascontiguousarray(dates, dtype=np.int32)
    e = None if end_dates is None else np.ascontiguousarray(end_dates, dtype=np.int32)
    sf = np.ascontiguousarray(ix.seg_first, dtype=np.int64)
    ns = sf.size
    ranges = np.empty(2 * max(ns, 1), np.int64)
    seg_id = np.empty(max(ns, 1), np.int32)
    nr = int(lib.mfa_shard_rows_ix(sf.ctypes.data, ns, d.size, d.ctypes.data,
                                   None if e is None else e.ctypes.data, int(date_lo), int(date_hi),
                                   int(halo), int(nstmt), ranges.ctypes.data, seg_id.ctypes.data,
                                   nthreads))
    return ranges[:2 * nr].reshape(-1, 2), seg_id[:nr]


def shard_rows(codes: np.ndarray, dates: np.ndarray, end_dates: np.ndarray | None,
               date_lo: int, date_hi: int, halo: int, nstmt: int = 4, nthreads: int = 0):
    """:func:`shard_rows_ix` on a fresh :func:`row_index` of the columns.  Returns ``(ranges,
    seg_id, seg_first)``, or None when the native library is missing or the rows are not
    sorted by (code, date)."""
    ix = row_index(codes, dates, nthreads)
    if ix is None:
        return None
    ranges, seg_id = shard_rows_ix(ix, dates, end_dates, date_lo, date_hi, halo, nstmt, nthreads)
    return ranges, seg_id, ix.seg_first


def gather_ranges(x: np.ndarray, ranges: np.ndarray, offs: np.ndarray, out: np.ndarray,
                  nthreads: int = 0) -> np.ndarray:
    """out = concatenation of x[a:b] over ``ranges`` (threaded memcpy); ``offs`` = [0, cumsum of
    the range lengths]."""
    lib = _load()
    xs = np.ascontiguousarray(x)
    r = np.ascontiguousarray(ranges, dtype=np.int64)
    o = np.ascontiguousarray(offs, dtype=np.int64)
    rc = lib.mfa_gather_ranges(xs.ctypes.data, xs.itemsize, r.ctypes.data, o.ctypes.data,
                               r.shape[0], out.ctypes.data, nthreads)
    if rc != 0:
        raise RuntimeError("mfa_gather_ranges failed")
    return out
