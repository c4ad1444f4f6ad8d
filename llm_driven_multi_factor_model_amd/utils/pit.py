"""Point-in-time panel assembly (L3): statement dedupe, as-of joins, fills.

Reference: ``Barra_factor_cal/load_data.py`` — ``optimize_dtypes`` (:13-25),
``robust_merge_asof`` (:41-62, a per-stock ``pd.merge_asof`` loop), the statement dedupe rules
(:264-310) and the ffill / fill step (:393-418).

``robust_merge_asof`` here runs the native multi-threaded two-pointer join
(``csrc_host/asof.cpp``) on (stock code, int64 key) arrays; pandas is only used to sort and to
gather the matched columns.  Results are identical to the reference's per-stock loop.
"""
from __future__ import annotations

import ctypes as C
import itertools

import numpy as np
import pandas as pd

from .._build import HOST_LIB_PATH, build_host

_lib = None


def _load():
    global _lib
    if _lib is None:
        if not HOST_LIB_PATH.exists():
            build_host()
        lib = C.CDLL(str(HOST_LIB_PATH))
        lib.mfa_asof_join.argtypes = [C.c_void_p, C.c_void_p, C.c_int64, C.c_void_p, C.c_void_p,
                                      C.c_int64, C.c_void_p, C.c_int]
        lib.mfa_asof_join.restype = C.c_int
        _lib = lib
    return _lib


def optimize_dtypes(df: pd.DataFrame) -> pd.DataFrame:
    """float64 -> float32, int64 -> int32, ts_code -> category (load_data.py:13-25, quirk Q27)."""
    for col in df.select_dtypes(include=["float64"]).columns:
        df[col] = df[col].astype("float32")
    for col in df.select_dtypes(include=["int64"]).columns:
        df[col] = df[col].astype("int32")
    if "ts_code" in df.columns:
        df["ts_code"] = df["ts_code"].astype("category")
    return df


def stream_collection(db, collection_name: str, query: dict | None = None,
                      projection: dict | None = None, chunk_size: int = 500_000):
    """Yield dtype-optimised DataFrames of at most ``chunk_size`` documents from one cursor.

    Memory-bounded load pattern of ``Barra_database/database/datause.ipynb#c6`` (500k-document
    chunks over the 6.6 M-row ``daily_prices``): only one chunk of Python dicts is alive at a
    time; each chunk is downcast (float32/int32) before the next is read.
    """
    if chunk_size < 1:
        raise ValueError("chunk_size must be >= 1")
    cursor = db[collection_name].find(query or {}, projection)
    if hasattr(cursor, "batch_size"):
        cursor = cursor.batch_size(min(chunk_size, 100_000))
    it = iter(cursor)
    while True:
        docs = list(itertools.islice(it, chunk_size))
        if not docs:
            return
        df = pd.DataFrame(docs)
        del docs
        if "_id" in df.columns:
            df = df.drop(columns="_id")
        yield optimize_dtypes(df)


def load_collection_chunked(db, collection_name: str, query: dict | None = None,
                            projection: dict | None = None, chunk_size: int = 500_000) -> pd.DataFrame:
    """Concatenate :func:`stream_collection` chunks; ``ts_code`` ends as one categorical."""
    parts = list(stream_collection(db, collection_name, query, projection, chunk_size))
    if not parts:
        return pd.DataFrame()
    for p in parts:
        if "ts_code" in p.columns:
            p["ts_code"] = p["ts_code"].astype(str)
    df = pd.concat(parts, ignore_index=True)
    del parts
    if "ts_code" in df.columns:
        df["ts_code"] = df["ts_code"].astype("category")
    return df


def _keys(s: pd.Series) -> np.ndarray:
    if np.issubdtype(s.dtype, np.datetime64):
        return s.values.astype("datetime64[ns]").astype(np.int64)
    return pd.to_datetime(s.astype(str), format="mixed").values.astype("datetime64[ns]").astype(np.int64)


def asof_indices(left_groups, left_keys, right_groups, right_keys) -> np.ndarray:
    """For (group, key)-sorted inputs: index of the last right row with the same group and
    key <= left key, else -1."""
    lg = np.ascontiguousarray(left_groups, dtype=np.int32)
    lk = np.ascontiguousarray(left_keys, dtype=np.int64)
    rg = np.ascontiguousarray(right_groups, dtype=np.int32)
    rk = np.ascontiguousarray(right_keys, dtype=np.int64)
    out = np.empty(len(lg), dtype=np.int64)
    try:
        lib = _load()
    except Exception as e:  # no host toolchain: the numpy loop below is the same join
        import logging
        logging.getLogger("mfa").warning("native as-of join unavailable (%s); using numpy", e)
        lib = None
    if lib is None:
        for i in range(len(lg)):
            lo = np.searchsorted(rg, lg[i], "left")
            hi = np.searchsorted(rg, lg[i], "right")
            k = np.searchsorted(rk[lo:hi], lk[i], "right") - 1
            out[i] = lo + k if k >= 0 else -1
        return out
    lib.mfa_asof_join(lg.ctypes.data, lk.ctypes.data, len(lg), rg.ctypes.data, rk.ctypes.data, len(rg),
                      out.ctypes.data, 0)
    return out


def robust_merge_asof(left_df: pd.DataFrame, right_df: pd.DataFrame, left_on: str, right_on: str,
                      by: str, device: str | None = None) -> pd.DataFrame:
    """Per-``by`` backward as-of merge (semantics of load_data.py:41-62).

    Output rows are ordered like the reference (sorted by [by, left_on]); right-side columns
    that collide with left ones get pandas' ``_x`` / ``_y`` suffixes.  ``device="cuda"`` runs
    the index search on the GPU (``ops.asof``, HIP kernel ``csrc/asof.hip``); the default is the
    multi-threaded host join.
    """
    left = left_df.reset_index(drop=True).sort_values(by=[by, left_on], kind="stable").reset_index(drop=True)
    right = right_df.reset_index(drop=True).sort_values(by=[by, right_on], kind="stable").reset_index(drop=True)
    cats = pd.Index(pd.unique(pd.concat([left[by].astype(str), right[by].astype(str)]))).sort_values()
    lg = cats.get_indexer(left[by].astype(str))
    rg = cats.get_indexer(right[by].astype(str))
    # keys must be non-decreasing within each group on both sides (they are: sorted above)
    if device is not None and str(device).startswith("cuda"):
        import torch
        from ..ops.asof import asof_search
        t = lambda a, dt: torch.as_tensor(np.ascontiguousarray(a, dtype=dt), device=device)  # noqa: E731
        idx = asof_search(t(lg, np.int32), t(_keys(left[left_on]), np.int64), t(rg, np.int32),
                          t(_keys(right[right_on]), np.int64), check_sorted=False).cpu().numpy()
    else:
        idx = asof_indices(lg, _keys(left[left_on]), rg, _keys(right[right_on]))
    rcols = [c for c in right.columns if c != by]
    taken = right.iloc[np.where(idx >= 0, idx, 0)][rcols].reset_index(drop=True)
    taken.loc[idx < 0, :] = np.nan
    overlap = [c for c in rcols if c in left.columns]
    taken = taken.rename(columns={c: c + "_y" for c in overlap})
    left = left.rename(columns={c: c + "_x" for c in overlap})
    out = pd.concat([left, taken], axis=1)
    return out


def dedupe_statements(df: pd.DataFrame, ann_col: str = "f_ann_date") -> pd.DataFrame:
    """load_data.py:264-310: keep the latest announcement per (ts_code, end_date), then the
    latest report period per (ts_code, announcement date)."""
    d = df.copy()
    d[ann_col] = pd.to_datetime(d[ann_col].astype(str), format="%Y%m%d", errors="coerce")
    d["end_date"] = pd.to_datetime(d["end_date"].astype(str), format="%Y%m%d", errors="coerce")
    if ann_col == "f_ann_date":
        d = d.sort_values(["ts_code", "end_date", ann_col], ascending=[True, True, False]) \
            .drop_duplicates(subset=["ts_code", "end_date"], keep="first")
    d = d.sort_values(["ts_code", ann_col, "end_date"], ascending=[True, True, False]) \
        .drop_duplicates(subset=["ts_code", ann_col], keep="first")
    return d


FILL_COLS = ["pe_ttm", "pb", "total_ncl", "total_hldr_eqy_inc_min_int", "debt_to_assets", "q_sales_yoy",
             "q_profit_yoy", "n_cashflow_act", "balance_sheet_f_ann_date",
             "financial_indicators_ann_date", "cashflow_f_ann_date", "end_date"]


def fill_missing(df: pd.DataFrame, cols=FILL_COLS, fix_order: bool = False) -> pd.DataFrame:
    """load_data.py:393-418: per-stock ffill, then fillna(0), then per-date median (a no-op
    after fillna(0), quirk Q19).  ``fix_order=True`` applies the median before the zero fill,
    as the prototype in try_1023.ipynb#c3 intended."""
    out = df.sort_values(by=["ts_code", "trade_date"]).reset_index(drop=True)
    cols = [c for c in cols if c in out.columns]
    out[cols] = out.groupby("ts_code", observed=True)[cols].ffill()
    num = [c for c in cols if pd.api.types.is_numeric_dtype(out[c])]
    if fix_order:
        med = out.groupby("trade_date")[num].transform("median")
        out[num] = out[num].fillna(med)
    out[cols] = out[cols].fillna(0)
    return out
