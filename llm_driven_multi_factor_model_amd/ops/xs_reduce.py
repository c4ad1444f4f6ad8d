"""Per-date cross-sectional reductions (winsorize, composite, OLS residualisation, z-score, shrink).

GPU path: ``csrc/xs_reduce.hip``; CPU path: float64 torch transcriptions of the pandas /
statsmodels semantics of the reference:

* :func:`winsorize` — ``post_processing.winsorize_factors`` (post_processing.py:7-24): per date,
  clip to mean +- n*std with pandas' NaN-skipping ddof-1 std; < 2 valid values -> no clipping;
* :func:`composite` — ``calculate_composite_factors`` (:26-45);
* :func:`ols_resid` — ``orthogonalize_factors`` (:47-69; min rows p+2) and NLSIZE
  (factor_calculator.py:237-293; min rows 2, sign -1);
* :func:`style_norm` — ``CrossSection.style_factor_norm`` (CrossSection.py:12-20);
* :func:`bayes_shrink` — ``mfm.utils.bayes_shrink`` (utils.py:133-168).

Panels are [D, N] float32 tensors (one field) or [D, Q, N] for ``style_norm``.
"""
from __future__ import annotations

import ctypes as C

import torch

from .. import _native

_native.register("mfa_winsorize", [C.c_void_p, C.c_int, C.c_int, C.c_double, C.c_void_p])
_native.register("mfa_composite", [C.c_void_p, C.c_void_p, C.c_int, C.c_size_t, C.c_void_p, C.c_void_p])
_native.register("mfa_ols_resid", [C.c_void_p, C.c_void_p, C.c_int, C.c_int, C.c_int, C.c_int,
                                    C.c_double, C.c_int, C.c_int, C.c_void_p, C.c_void_p])
_native.register("mfa_style_norm", [C.c_void_p, C.c_void_p, C.c_int, C.c_int, C.c_int, C.c_void_p,
                                     C.c_void_p, C.c_void_p])
_native.register("mfa_bayes_shrink", [C.c_void_p, C.c_void_p, C.c_int, C.c_int, C.c_int, C.c_double,
                                       C.c_void_p, C.c_void_p, C.c_void_p])
_native.register("mfa_rows_grid", [C.c_int, C.c_int, C.c_void_p, C.c_int64, C.c_void_p, C.c_void_p,
                                   C.c_int, C.c_int, C.c_int, C.c_void_p, C.c_int64, C.c_int64,
                                   C.c_double, C.c_void_p])
_native.register("mfa_bayes_shrink_presorted", [C.c_void_p, C.c_void_p, C.c_void_p, C.c_int, C.c_int,
                                                 C.c_int, C.c_double, C.c_void_p, C.c_void_p,
                                                 C.c_void_p])


def _f32(t: torch.Tensor) -> torch.Tensor:
    return t.to(torch.float32).contiguous()


# ------------------------------------------------------------------ winsorize
def winsorize(x: torch.Tensor, n_std: float = 2.5) -> torch.Tensor:
    """Per-row (date) clip to mean +- n_std * std (ddof 1, NaN-skipping).  Returns a new tensor."""
    shp = x.shape
    y = _f32(x).clone().reshape(-1, shp[-1])
    if not y.is_cuda:
        return _winsorize_ref(y, n_std).reshape(shp)
    _native.call("mfa_winsorize", _native.ptr(y), y.shape[0], y.shape[1], float(n_std),
                 _native.stream(y.device))
    return y.reshape(shp)


def winsorize_(x: torch.Tensor, n_std: float = 2.5) -> torch.Tensor:
    """:func:`winsorize` in place on a contiguous float32 tensor (rows = dates); returns it."""
    if x.dtype != torch.float32 or not x.is_contiguous():
        raise ValueError("winsorize_: contiguous float32 tensor")
    y = x.view(-1, x.shape[-1])
    if not y.is_cuda:
        y.copy_(_winsorize_ref(y, n_std))
        return x
    _native.call("mfa_winsorize", _native.ptr(y), y.shape[0], y.shape[1], float(n_std),
                 _native.stream(y.device))
    return x


# ------------------------------------------------------------------ rows <-> (date, stock) grid
class GridMap:
    """Rows sorted by (stock, date) <-> a date-major [Dg, Ng] grid, as an LDS-tiled transpose
    (``csrc/gather.hip``, ``mfa_rows_grid``: 64-date x 64-stock tiles, coalesced on both
    sides).  ``sid`` / ``did`` [R]: each row's stock (< Ng) and date (< Dg), (sid, did) strictly
    increasing (else the index fallback).  ``toff`` [Ng, ceil(Dg / 64) + 1]: the first row of every (stock, 64-date
    block), from the sorted key."""

    def __init__(self, sid: torch.Tensor, did: torch.Tensor, Dg: int, Ng: int):
        dev = sid.device
        key = sid.to(torch.int64) * Dg + did.to(torch.int64)
        ntb = (Dg + 63) // 64
        edges = torch.clamp(torch.arange(ntb + 1, device=dev, dtype=torch.int64) * 64, max=Dg)
        q = torch.arange(Ng, device=dev, dtype=torch.int64)[:, None] * Dg + edges[None, :]
        self.toff = torch.searchsorted(key, q.reshape(-1)).contiguous()
        self.did = did.to(torch.int32).contiguous()
        self.idx = did.to(torch.int64) * Ng + sid.to(torch.int64)   # flat cell (CPU path)
        self.Dg, self.Ng, self.R = int(Dg), int(Ng), int(sid.numel())
        # the tile kernel covers one row per (stock, date) cell; duplicate cells (the pandas
        # engine's fall-back input) take the index path (last row of a cell wins on scatter)
        self.strict = self.R < 2 or bool((key[1:] > key[:-1]).all())

    def _cells(self, ds: int) -> torch.Tensor:
        return torch.div(self.idx, self.Ng, rounding_mode="floor") * ds + self.idx % self.Ng

    def scatter(self, X: torch.Tensor, fill: float = float("nan"), out: torch.Tensor | None = None,
                gs: int | None = None, ds: int | None = None) -> torch.Tensor:
        """``X`` [C, R] (float32 or float64) -> grids: cell (c, d, s) at ``c * gs + d * ds + s``
        of ``out`` (contiguous, written in place), default a new [C, Dg * Ng] tensor with
        ``fill`` in the cells without a row."""
        if X.dtype not in (torch.float32, torch.float64):
            X = X.to(torch.float32)
        X = X.contiguous()
        Cn = X.shape[0]
        gs = self.Dg * self.Ng if gs is None else gs
        ds = self.Ng if ds is None else ds
        G = out if out is not None else torch.full((Cn, self.Dg * self.Ng), fill, dtype=X.dtype,
                                                   device=X.device)
        if G.dtype != X.dtype or not G.is_contiguous():
            raise ValueError("GridMap.scatter: contiguous grids of the rows' dtype")
        if not X.is_cuda or self.R == 0 or not self.strict:
            cell = self._cells(ds)
            flat = G.view(-1)
            for c in range(Cn):
                flat[c * gs + cell] = X[c]
            return G
        _native.call("mfa_rows_grid", 1, X.element_size(), _native.ptr(X), X.stride(0),
                     _native.ptr(self.did), _native.ptr(self.toff), self.Dg, self.Ng, Cn,
                     _native.ptr(G), gs, ds, float(fill), _native.stream(X.device))
        return G

    def gather(self, G: torch.Tensor, C: int, gs: int | None = None,
               ds: int | None = None) -> torch.Tensor:
        """The inverse: C grids of ``G`` (same layout, contiguous) -> [C, R] of G's dtype."""
        gs = self.Dg * self.Ng if gs is None else gs
        ds = self.Ng if ds is None else ds
        if not G.is_contiguous():
            raise ValueError("GridMap.gather: contiguous grids")
        X = torch.empty(C, self.R, dtype=G.dtype, device=G.device)
        if not G.is_cuda or self.R == 0 or not self.strict:
            cell = self._cells(ds)
            flat = G.reshape(-1)
            for c in range(C):
                X[c] = flat[c * gs + cell]
            return X
        _native.call("mfa_rows_grid", 0, G.element_size(), _native.ptr(X), X.stride(0),
                     _native.ptr(self.did), _native.ptr(self.toff), self.Dg, self.Ng, C,
                     _native.ptr(G), gs, ds, 0.0, _native.stream(G.device))
        return X


def _winsorize_ref(y: torch.Tensor, n_std: float) -> torch.Tensor:
    v = y.double()
    ok = ~torch.isnan(v)
    c = ok.sum(1, keepdim=True).double()
    z = torch.where(ok, v, torch.zeros((), dtype=torch.float64))
    mean = z.sum(1, keepdim=True) / c
    dev = torch.where(ok, v - mean, torch.zeros((), dtype=torch.float64))
    sd = torch.sqrt((dev * dev).sum(1, keepdim=True) / (c - 1))
    lo, hi = mean - n_std * sd, mean + n_std * sd
    clipped = torch.minimum(torch.maximum(v, lo), hi)
    keep = (c >= 2).expand_as(v)
    return torch.where(ok & keep, clipped, v).float()


# ------------------------------------------------------------------ composite
def composite(xs: list[torch.Tensor], weights: list[float]) -> torch.Tensor:
    """``sum_i w_i x_i.fillna(0) / sum_i w_i notna(x_i)`` (all-missing -> NaN)."""
    if not 1 <= len(xs) <= 8:
        raise ValueError("1..8 components")
    xs = [_f32(x) for x in xs]
    shp = xs[0].shape
    if not xs[0].is_cuda:
        num = torch.zeros(shp, dtype=torch.float64)
        den = torch.zeros(shp, dtype=torch.float64)
        for x, w in zip(xs, weights):
            ok = ~torch.isnan(x)
            num += torch.where(ok, x.double(), torch.zeros((), dtype=torch.float64)) * w
            den += ok.double() * w
        return (num / den).float()
    out = torch.empty(shp, dtype=torch.float32, device=xs[0].device)
    ptrs = (C.c_void_p * len(xs))(*[x.data_ptr() for x in xs])
    ws = (C.c_double * len(xs))(*[float(w) for w in weights])
    _native.call("mfa_composite", ptrs, ws, len(xs), out.numel(), _native.ptr(out),
                 _native.stream(out.device))
    return out


# ------------------------------------------------------------------ OLS residual
def ols_resid(y: torch.Tensor | None, xs: list[torch.Tensor], min_rows: int | None = None,
              sign: float = 1.0, log_x0: bool = False, ypow: int = 0) -> torch.Tensor:
    """Per-date residual of ``y`` [D, N] on ``[1, x_1..x_p]`` over rows where all are finite.

    ``min_rows`` defaults to p + 2 (``orthogonalize_factors``); NLSIZE uses 2 and sign -1 with
    ``log_x0=True, ypow=3`` so SIZE = ln(total_mv) and SIZE^3 are formed in float64 in-kernel
    (as the reference does in numpy) instead of being rounded to float32 first.
    Dates with fewer valid rows are all-NaN (the reference returns a NaN series).
    """
    p = len(xs)
    if p > 4:
        raise ValueError("at most 4 regressors")
    min_rows = p + 2 if min_rows is None else min_rows
    xs = [_f32(x) for x in xs]
    D, N = xs[0].shape if xs else y.shape
    y = _f32(y) if y is not None else None
    if not xs[0].is_cuda if xs else not y.is_cuda:
        return _ols_resid_ref(y, xs, min_rows, sign, log_x0, ypow)
    out = torch.empty(D, N, dtype=torch.float32, device=(xs[0] if xs else y).device)
    ptrs = (C.c_void_p * max(1, p))(*[x.data_ptr() for x in xs]) if p else (C.c_void_p * 1)(0)
    _native.call("mfa_ols_resid", _native.ptr(y), ptrs, p, D, N, int(min_rows), float(sign),
                 int(log_x0), int(ypow), _native.ptr(out), _native.stream(out.device))
    return out


def _ols_resid_ref(y, xs, min_rows, sign, log_x0=False, ypow=0):
    D, N = xs[0].shape if xs else y.shape
    out = torch.full((D, N), float("nan"), dtype=torch.float32)
    for d in range(D):
        xd = [x[d].double() for x in xs]
        if log_x0:
            xd[0] = torch.log(xd[0])
        cols = [torch.ones(N, dtype=torch.float64)] + xd
        Xd = torch.stack(cols, 1)
        yd = xd[0] ** ypow if ypow > 0 else y[d].double()
        ok = torch.isfinite(yd) & torch.isfinite(Xd).all(1)
        if int(ok.sum()) < min_rows:
            continue
        b = torch.linalg.pinv(Xd[ok]) @ yd[ok]
        e = yd - Xd @ b
        out[d][ok] = (sign * e[ok]).float()
    return out


# ------------------------------------------------------------------ z-score
def style_norm(X: torch.Tensor, cap: torch.Tensor):
    """``(x - cap-weighted mean_q) / pooled std`` for X [D, Q, N]; returns (Z, mu [D,Q], sigma [D])."""
    Z = _f32(X).clone()
    cap = _f32(cap)
    D, Q, N = Z.shape
    if not Z.is_cuda:
        Xd = Z.double()
        c = cap.double()
        ok = torch.isfinite(c) & torch.isfinite(Xd).all(1)
        w = torch.where(ok, c, torch.zeros((), dtype=torch.float64))
        Xz = torch.where(ok[:, None, :], Xd, torch.zeros((), dtype=torch.float64))
        mu = (Xz * w[:, None, :]).sum(2) / w.sum(1, keepdim=True)
        n = ok.sum(1).double() * Q
        m = Xz.sum((1, 2)) / n
        sig = torch.sqrt(torch.clamp((Xz * Xz).sum((1, 2)) / n - m * m, min=0))
        return ((Xd - mu[..., None]) / sig[:, None, None]).float(), mu, sig
    mu = torch.empty(D, Q, dtype=torch.float64, device=Z.device)
    sig = torch.empty(D, dtype=torch.float64, device=Z.device)
    _native.call("mfa_style_norm", _native.ptr(Z), _native.ptr(cap), D, Q, N, _native.ptr(mu),
                 _native.ptr(sig), _native.stream(Z.device))
    return Z, mu, sig


# ------------------------------------------------------------------ Bayesian shrinkage
BAYES_LDS_N = 16384  # universes up to this size sort their caps in LDS


def bayes_shrink(volatility: torch.Tensor, capital: torch.Tensor, ngroup: int = 10, q: float = 1.0,
                 return_groups: bool = False):
    """Cap-decile Bayesian shrinkage of specific volatility (``utils.bayes_shrink``).

    Accepts [N] (one date) or [D, N].  Groups follow ``pd.qcut(capital, ngroup).codes``.
    """
    squeeze = volatility.dim() == 1
    v = _f32(volatility).reshape(-1, volatility.shape[-1])
    c = _f32(capital).reshape(-1, capital.shape[-1])
    D, N = v.shape
    if not v.is_cuda:
        out, g = _bayes_ref(v, c, ngroup, q)
    else:
        out = torch.empty_like(v)
        g = torch.empty(D, N, dtype=torch.int32, device=v.device)
        if N <= BAYES_LDS_N:  # bitonic sort of the caps in LDS
            _native.call("mfa_bayes_shrink", _native.ptr(v), _native.ptr(c), D, N, ngroup,
                         float(q), _native.ptr(out), _native.ptr(g), _native.stream(v.device))
        else:  # wide universe: device segmented sort (rocPRIM) feeds the same kernel
            keys = torch.where(torch.isfinite(v) & torch.isfinite(c), c,
                               torch.full_like(c, float("inf")))
            srt = torch.sort(keys, dim=1).values.contiguous()
            _native.call("mfa_bayes_shrink_presorted", _native.ptr(v), _native.ptr(c),
                         _native.ptr(srt), D, N, ngroup, float(q), _native.ptr(out),
                         _native.ptr(g), _native.stream(v.device))
    if squeeze:
        out, g = out[0], g[0]
    return (out, g) if return_groups else out


def _bayes_ref(v, c, G, q):
    import numpy as np
    D, N = v.shape
    out = torch.full((D, N), float("nan"), dtype=torch.float32)
    grp = torch.full((D, N), -1, dtype=torch.int32)
    for d in range(D):
        vd, cd = v[d].double().numpy(), c[d].double().numpy()
        ok = np.isfinite(vd) & np.isfinite(cd)
        if not ok.any():  # no (vol, cap) pair on this date (e.g. an all-NaN halo date): NaN row
            continue
        cs = cd[ok]
        edges = np.quantile(cs, np.linspace(0, 1, G + 1))
        g = np.zeros(len(cs), dtype=np.int64)
        for k in range(1, G):
            g[cs > edges[k]] = k
        vv = vd[ok]
        res = np.empty(len(cs))
        for k in range(G):
            sel = g == k
            if not sel.any():
                continue
            m = (vv[sel] * cs[sel]).sum() / cs[sel].sum()
            s = np.sqrt(np.mean((vv[sel] - m) ** 2))
            a = q * np.abs(vv[sel] - m)
            w = a / (a + s)
            res[sel] = w * m + (1 - w) * np.abs(vv[sel])
        o = np.full(N, np.nan)
        o[ok] = res
        gg = np.full(N, -1)
        gg[ok] = g
        out[d] = torch.from_numpy(o).float()
        grp[d] = torch.from_numpy(gg).int()
    return out, grp
