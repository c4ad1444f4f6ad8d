"""Data contracts: ``barra_data_csi.csv`` / ``industry_info.csv`` in, ``results/*.csv`` out.

* ``barra_data_csi.csv`` (``Barra_factor_cal/config.py:68-71``): 15 columns ``date,
  stocknames, capital, ret (t+1), industry, size, beta, momentum, residual_volatility,
  non_linear_size, book_to_price_ratio, liquidity, earnings_yield, growth, leverage``;
* ``industry_info.csv``: ``code, industry_names, start_date``;
* the MFM input frame (``Barra-master/demo.py:25-35``): NaN rows dropped, industries one-hot
  against ``industry_info.code`` -> ``[date, stocknames, capital, ret, <P one-hots>, <Q styles>]``;
* risk outputs (``demo.py:65-94``): ``factor_returns.csv``, ``r_squared.csv``,
  ``specific_returns.csv``, ``final_vol_regime_adj_covariance.csv``,
  ``volatility_multiplier_lambda.csv``.

Long frames become dense (date x stock) device panels in one vectorised scatter (no per-date
boolean masking as in ``MFM.py:58``).  The native CSV parser (``csrc_host/csv_panel.cpp``) is
used for the 15-column Barra file when built; pandas is the fallback.
"""
from __future__ import annotations

import os
import warnings

import numpy as np
import pandas as pd
import torch

from ..models.panel import RiskPanel

BARRA_COLUMNS = [
    "date", "stocknames", "capital", "ret", "industry",
    "size", "beta", "momentum", "residual_volatility", "non_linear_size",
    "book_to_price_ratio", "liquidity", "earnings_yield", "growth", "leverage",
]


def read_barra_csv(path: str) -> pd.DataFrame:
    from . import native_io
    df = native_io.read_barra_csv(path)
    if df is None:
        df = pd.read_csv(path)
    return df


def mfm_frame(barra: pd.DataFrame, industry_info: pd.DataFrame) -> pd.DataFrame:
    """demo.py:25-35 — drop NaN rows, one-hot industries against industry_info.code."""
    data = barra[~barra.isna().any(axis=1)].reset_index(drop=True)
    codes = industry_info["code"].values
    ind = (data["industry"].values[:, None] == codes[None, :]).astype(np.int64)
    ind = pd.DataFrame(ind, columns=list(industry_info["industry_names"].values))
    return pd.concat([data.iloc[:, :4], ind, data.iloc[:, 5:]], axis=1)


def panel_from_frame(data: pd.DataFrame, P: int, Q: int, device="cpu",
                     industry_from_onehot: bool = True, dtype=torch.float64) -> RiskPanel:
    """Dense panel from the MFM positional frame ([date, stocknames, capital, ret, P inds, Q styles]).

    ``dtype`` = panel storage: float64 (default) keeps the frame's values exactly as the
    reference regresses them (``demo.py:21`` -> ``CrossSection.reg``); float32 halves HBM.

    Positional contract of ``MFM.py:36,61`` (quirk Q13).  Rows whose industry one-hot is all
    zero cannot be expressed as an industry id and are dropped with a warning (the reference
    would regress them with zero industry exposure); duplicate (date, stock) rows keep the last.
    """
    dates = pd.to_datetime(data.iloc[:, 0].values)
    d_codes, d_uni = pd.factorize(dates, sort=True)
    names = data.iloc[:, 1].astype(str).values
    s_codes, s_uni = pd.factorize(names, sort=True)
    D, N = len(d_uni), len(s_uni)
    npdt = np.float64 if dtype == torch.float64 else np.float32
    cap = np.full((D, N), np.nan, dtype=npdt)
    ret = np.full((D, N), np.nan, dtype=npdt)
    sty = np.full((D, Q, N), np.nan, dtype=npdt)
    ind = np.full((D, N), -1, dtype=np.int16)
    if pd.Index(d_codes * N + s_codes).has_duplicates:
        warnings.warn("duplicate (date, stock) rows: keeping the last occurrence")
    cap[d_codes, s_codes] = data.iloc[:, 2].values.astype(npdt)
    ret[d_codes, s_codes] = data.iloc[:, 3].values.astype(npdt)
    styles = data.iloc[:, data.shape[1] - Q:].values.astype(npdt)
    for q in range(Q):
        sty[d_codes, q, s_codes] = styles[:, q]
    if P > 0:
        oh = data.iloc[:, 4:4 + P].values
        has = oh.sum(1) > 0
        if not has.all():
            warnings.warn(f"{int((~has).sum())} rows without an industry dummy are excluded")
        ids = np.where(has, oh.argmax(1), -1).astype(np.int16)
        ind[d_codes, s_codes] = ids
    ind_names = list(data.columns[4:4 + P]) if P > 0 else []
    sty_names = list(data.columns[data.shape[1] - Q:])
    dev = torch.device(device)
    return RiskPanel(
        styles=torch.from_numpy(sty).to(dev), cap=torch.from_numpy(cap).to(dev),
        ret=torch.from_numpy(ret).to(dev),
        ind=torch.from_numpy(ind).to(dev) if P > 0 else None, P=P,
        dates=np.asarray(d_uni.values, dtype="datetime64[ns]"), stocks=np.asarray(s_uni, dtype=object),
        style_names=sty_names, industry_names=ind_names)


def _unique_s16(a: np.ndarray):
    """``np.unique(a, return_inverse=True)`` for an ``S16`` array via hash factorisation of its
    two 8-byte words (O(n); the string sort took ~0.4 s per million rows), then a sort of the
    few uniques only."""
    if a.dtype != np.dtype("S16") or not a.flags.c_contiguous:
        return np.unique(a, return_inverse=True)
    w = a.view(np.uint64).reshape(-1, 2)
    c0, u0 = pd.factorize(w[:, 0])
    c1, u1 = pd.factorize(w[:, 1])
    codes, pairs = pd.factorize(c0.astype(np.int64) * len(u1) + c1)
    uw = np.stack([u0[pairs // len(u1)], u1[pairs % len(u1)]], 1).astype(np.uint64)
    uniq = np.ascontiguousarray(uw).view("S16").reshape(-1)
    order = np.argsort(uniq, kind="stable")
    rank = np.empty_like(order)
    rank[order] = np.arange(len(order))
    return uniq[order], rank[codes]


def panel_from_barra_csv(path: str, industry_info_path: str, device="cpu",
                         dtype=torch.float64) -> RiskPanel:
    """barra_data_csi.csv + industry_info.csv -> dense panel (demo.py:22-35 semantics).

    ``dtype`` = panel storage; float64 (default) is the reference's precision (pd.read_csv).

    Fast path: the native reader's columnar buffers are factorised directly (no per-row Python
    objects); falls back to pandas + :func:`mfm_frame`.
    """
    info = pd.read_csv(industry_info_path)
    from . import native_io
    cols = None if os.environ.get("MFA_NO_NATIVE_IO") else native_io.read_columns(
        path, {"date": 1, "stocknames": 1, "industry": 1})
    if cols is None:
        barra = read_barra_csv(path)
        frame = mfm_frame(barra, info)
        return panel_from_frame(frame, len(info), barra.shape[1] - 5, device=device, dtype=dtype)
    names = list(cols)
    styles = names[5:]
    Q = len(styles)
    P = len(info)
    ok = (cols["date"] != b"") & (cols["stocknames"] != b"") & (cols["industry"] != b"")
    for c in ["capital", "ret", *styles]:  # demo.py:25-27 drops rows with any NaN
        ok &= np.isfinite(cols[c])
    codes = np.asarray(info["code"].astype(str).values).astype("S16")
    order = np.argsort(codes)
    pos = np.searchsorted(codes[order], cols["industry"])
    pos = np.clip(pos, 0, len(codes) - 1)
    hit = codes[order][pos] == cols["industry"]
    ind_id = np.where(hit, order[pos], -1)
    if ok.any() and (~hit[ok]).any():
        warnings.warn(f"{int((~hit[ok]).sum())} rows have an industry code missing from "
                      "industry_info and are excluded")
    sel = ok & hit
    d_uni, d_codes = _unique_s16(cols["date"][sel])
    s_uni, s_codes = _unique_s16(cols["stocknames"][sel])
    D, N = len(d_uni), len(s_uni)
    npdt = np.float64 if dtype == torch.float64 else np.float32
    cap = np.full((D, N), np.nan, dtype=npdt)
    ret = np.full((D, N), np.nan, dtype=npdt)
    sty = np.full((D, Q, N), np.nan, dtype=npdt)
    ind = np.full((D, N), -1, dtype=np.int16)
    flat = d_codes * N + s_codes
    cap.reshape(-1)[flat] = cols["capital"][sel]
    ret.reshape(-1)[flat] = cols["ret"][sel]
    sflat = d_codes * (Q * N) + s_codes
    for q, c in enumerate(styles):
        sty.reshape(-1)[sflat + q * N] = cols[c][sel]
    ind.reshape(-1)[flat] = ind_id[sel].astype(np.int16)
    dates = pd.to_datetime(pd.Index(d_uni.astype("U16")), format="mixed").values
    dev = torch.device(device)
    return RiskPanel(
        styles=torch.from_numpy(sty).to(dev), cap=torch.from_numpy(cap).to(dev),
        ret=torch.from_numpy(ret).to(dev), ind=torch.from_numpy(ind).to(dev) if P > 0 else None,
        P=P, dates=np.asarray(dates, dtype="datetime64[ns]"),
        stocks=s_uni.astype("U16").astype(object), style_names=styles,
        industry_names=list(info["industry_names"].astype(str).values))


def panel_from_mongo(db, factors_collection: str = "barra_factors",
                     industry_collection: str = "sw_industry_info_for_factors",
                     device="cpu", dtype=torch.float64) -> RiskPanel:
    """Mongo-driven risk run (``Barra-master/demo.ipynb#c1``): the ``barra_factors`` collection
    written by ``Barra_factor_cal/main.py:150`` and its industry table
    (``sw_industry_info_for_factors``, ``main.py:153``) -> dense panel, with demo.py's NaN-row
    drop and one-hot semantics.  ``db`` is anything with pymongo's ``db[name].find`` surface."""
    barra = pd.DataFrame(list(db[factors_collection].find({}, {"_id": 0})))
    info = pd.DataFrame(list(db[industry_collection].find({}, {"_id": 0})))
    if barra.empty or info.empty:
        raise ValueError(f"empty collection: {factors_collection} ({len(barra)} docs), "
                         f"{industry_collection} ({len(info)} docs)")
    cols = [c for c in BARRA_COLUMNS if c in barra.columns]
    missing = [c for c in BARRA_COLUMNS[:5] if c not in barra.columns]
    if missing:
        raise ValueError(f"{factors_collection} lacks columns {missing}")
    barra = barra[cols]
    frame = mfm_frame(barra, info)
    return panel_from_frame(frame, len(info), barra.shape[1] - 5, device=device, dtype=dtype)


def write_barra_csv(df: pd.DataFrame, path: str) -> None:
    cols = [c for c in BARRA_COLUMNS if c in df.columns]
    df[cols].to_csv(path, index=False)


def write_risk_results(model, out_dir: str, long_specific: bool = False) -> dict:
    """Write the five demo.py result files (rank 0 only in distributed runs)."""
    from ..parallel import dist as pdist
    ctx = model.ctx
    F = pdist.gather_to_root(model.factor_ret, ctx)
    R2 = pdist.gather_to_root(model.r2, ctx)
    E = pdist.gather_to_root(model.specific_ret, ctx)
    lam = pdist.gather_to_root(model.vra_lambda, ctx) if model.vra_lambda is not None else None
    last = None
    if model.vra_cov is not None:  # collective: every rank participates, rank 0 keeps the result
        last = pdist.all_gather_rows(model.vra_cov[-1:], ctx)[-1]
    dates = model._global_dates()
    if ctx.enabled and ctx.rank != 0:
        return {}
    os.makedirs(out_dir, exist_ok=True)
    idx = pd.DatetimeIndex(dates)
    names = model.panel.factor_names
    paths = {}
    fr = pd.DataFrame(F.cpu().numpy(), index=idx, columns=names)
    paths["factor_returns"] = os.path.join(out_dir, "factor_returns.csv")
    fr.to_csv(paths["factor_returns"])
    paths["r_squared"] = os.path.join(out_dir, "r_squared.csv")
    pd.DataFrame(R2.cpu().numpy(), index=idx, columns=["R2"]).to_csv(paths["r_squared"])
    paths["specific_returns"] = os.path.join(out_dir, "specific_returns.csv")
    En = E.cpu().numpy()
    if long_specific:  # demo.ipynb#c5 variant: date, ts_code, specific_ret
        e = pd.DataFrame(En, index=idx, columns=model.panel.stocks)
        e.stack().rename("specific_ret").rename_axis(["date", "ts_code"]).reset_index().to_csv(
            paths["specific_returns"], index=False)
    else:  # dates x stocks: the native multi-threaded writer (pandas format), pandas fallback
        from .native_io import write_matrix_csv
        if En.dtype != np.float32 or not write_matrix_csv(
                paths["specific_returns"], En, idx.strftime("%Y-%m-%d"), model.panel.stocks):
            pd.DataFrame(En, index=idx, columns=model.panel.stocks).to_csv(paths["specific_returns"])
    if last is not None:
        paths["final_cov"] = os.path.join(out_dir, "final_vol_regime_adj_covariance.csv")
        pd.DataFrame(last.cpu().numpy(), index=names, columns=names).to_csv(paths["final_cov"])
    if lam is not None:
        paths["lambda"] = os.path.join(out_dir, "volatility_multiplier_lambda.csv")
        pd.Series(lam.cpu().numpy(), index=idx, name="lambda").to_csv(paths["lambda"])
    return paths
