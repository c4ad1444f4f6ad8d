"""Rolling-window descriptor ops on flat (stock-sorted) rows (K4/K5, ``csrc/rolling.hip``).

Rows follow the reference's master frame order — sorted by (ts_code, trade_date) — and
``seg_lo[r]`` is the first row of row r's stock, so every window counts the stock's own trading
rows exactly as ``groupby('ts_code').rolling(...)`` does (factor_calculator.py:79-367).
CPU paths are direct float64 transcriptions of the pandas callbacks (used as test oracles).
"""
from __future__ import annotations

import contextlib
import ctypes as C
import math

import numpy as np
import torch

from .. import _native

_vp, _i, _d = C.c_void_p, C.c_int, C.c_double
_native.register("mfa_beta_hsigma", [_vp, _vp, _vp, _i, _i, _d, _i, _vp, _vp, _vp])
_native.register("mfa_rstr", [_vp, _vp, _i, _i, _i, _d, _i, _vp, _vp])
_native.register("mfa_dastd", [_vp, _vp, _vp, _i, _i, _d, _i, _vp, _vp])
_native.register("mfa_cmra", [_vp, _vp, _i, _i, _i, _vp, _vp])
_native.register("mfa_rolling_sum", [_vp, _vp, _i, _i, _i, _d, _i, _vp, _vp])
_native.register("mfa_returns", [_vp, _vp, _i, _vp, _vp, _vp])
_native.register("mfa_ttm_flags", [_vp, _vp, _vp, _i, _vp, _vp, _vp])
_native.register("mfa_ttm_finish", [_vp, _vp, _vp, _vp, _i, _vp, _vp, _vp, _vp])
_native.register("mfa_leverage", [_vp, _vp, _vp, _i, _vp, _vp, _vp])
_native.register("mfa_rolling_set_mode", [_i])
_native.register("mfa_beta_hsigma_aligned", [_vp, _vp, _vp, _i, _i, _d, _i, _vp, _vp, _vp])
_native.register("mfa_dastd_aligned", [_vp, _vp, _vp, _i, _i, _d, _i, _vp, _vp])

ALIGN = 256      # rank-invariant EW kernels: tiles on global multiples of 256 rows
ALIGN_MAX_W = 255


def aligned_layout(seg_lo: torch.Tensor, row_ord: torch.Tensor):
    """Virtual row layout of the rank-invariant EW kernels (csrc/rolling.hip,
    mfa_beta_hsigma_aligned): the rows of each stock at B_s + t - T0_s, t = ``row_ord`` (the
    row's ordinal in the stock's FULL history), T0_s = t_first rounded down to a multiple of
    ALIGN, B_s = multiples of ALIGN.  Returns (v [R] int64 virtual position of every row,
    seg_v [Rv] int32 virtual seg_lo, Rv)."""
    dev = seg_lo.device
    R = seg_lo.numel()
    sl = seg_lo.long()
    ro = row_ord.long()
    # per row: T0 of its stock (first row's ordinal rounded down to ALIGN); a stock's padded
    # block count sits at its LAST row, so an exclusive prefix over rows gives, on every row of
    # stock s, the blocks of the stocks before it (B_s / ALIGN) -- no per-stock compaction
    T0 = torch.div(ro[sl], ALIGN, rounding_mode="floor") * ALIGN
    last = torch.ones(R, dtype=torch.bool, device=dev)
    if R > 1:
        last[:-1] = sl[1:] != sl[:-1]
    nb = torch.where(last, torch.div(ro - T0 + ALIGN, ALIGN, rounding_mode="floor"),
                     torch.zeros((), dtype=torch.int64, device=dev))
    cb = torch.cumsum(nb, 0) - nb
    base = cb * ALIGN - T0
    v = base + ro
    Rv = int(cb[-1] + nb[-1]) * ALIGN   # the one host read
    seg_v = torch.arange(Rv, device=dev, dtype=torch.int32)   # padding rows: their own starts
    seg_v[v] = (base + ro[sl]).to(torch.int32)
    return v, seg_v, Rv


def _layout(seg_lo, row_ord):
    """``row_ord`` is either the ordinals or an :func:`aligned_layout` built from them (an
    engine builds it once for BETA and DASTD)."""
    return tuple(row_ord) if isinstance(row_ord, tuple) else aligned_layout(seg_lo, row_ord)


def _to_virtual(x: torch.Tensor, v: torch.Tensor, Rv: int) -> torch.Tensor:
    out = torch.full((Rv,), float("nan"), dtype=torch.float32, device=x.device)
    out[v] = x
    return out


def _f(t):
    return t.to(torch.float32).contiguous()


@contextlib.contextmanager
def direct_kernels(on: bool = True):
    """GPU rolling descriptors from the direct per-row window kernels (``mfa_rolling_set_mode(1)``)
    inside the block: every output row is a fixed-order sum over its own window, so a row's
    value does not depend on which other rows share its launch (date shards reproduce the full
    panel bitwise).  No-op without a GPU or with ``on=False``."""
    if not (on and torch.cuda.is_available()):
        yield
        return
    lib = _native.lib()
    if lib.mfa_rolling_set_mode(1) != 0:
        raise _native.NativeError("mfa_rolling_set_mode(1) failed")
    try:
        yield
    finally:
        lib.mfa_rolling_set_mode(0)


def _i32(t):
    return t.to(torch.int32).contiguous()


def seg_lo_from_codes(codes: torch.Tensor) -> torch.Tensor:
    """First row index of each row's group for a group-sorted code vector."""
    codes = codes.to(torch.int64)
    R = codes.numel()
    start = torch.ones(R, dtype=torch.bool, device=codes.device)
    if R > 1:
        start[1:] = codes[1:] != codes[:-1]
    # segment id by an int32 prefix sum (rocPRIM scan) + gather of the segment starts; the
    # cummax-with-indices formulation took 57 ms at 18.9M rows on the MI355X
    sid = torch.cumsum(start.to(torch.int32), 0, dtype=torch.int32) - 1
    starts = torch.nonzero(start).flatten().to(torch.int32)
    return starts[sid.long()].contiguous()


# ---------------------------------------------------------------- returns
def returns(close, seg_lo):
    close, seg_lo = _f(close), _i32(seg_lo)
    R = close.numel()
    if close.is_cuda:
        ret, lr = torch.empty_like(close), torch.empty_like(close)
        _native.call("mfa_returns", _native.ptr(close), _native.ptr(seg_lo), R, _native.ptr(ret),
                     _native.ptr(lr), _native.stream(close.device))
        return ret, lr
    c = close.double().numpy()
    s = seg_lo.numpy()
    ret = np.full(R, np.nan)
    lr = np.full(R, np.nan)
    for r in range(R):
        if r == s[r]:
            continue
        if np.isfinite(c[r]) and np.isfinite(c[r - 1]) and c[r] > 0 and c[r - 1] > 0:
            lr[r] = math.log(c[r]) - math.log(c[r - 1])
        i = r
        while i >= s[r] and not np.isfinite(c[i]):
            i -= 1
        k = r - 1
        while k >= s[r] and not np.isfinite(c[k]):
            k -= 1
        if i >= s[r] and k >= s[r]:
            ret[r] = c[i] / c[k] - 1
    return torch.from_numpy(ret).float(), torch.from_numpy(lr).float()


# ---------------------------------------------------------------- BETA / HSIGMA
def beta_hsigma(ret, mret, seg_lo, window=252, half_life=63.0, min_periods=42, row_ord=None):
    """``row_ord`` (GPU, window <= 255): the rows' ordinals in their stocks' full histories (or
    their :func:`aligned_layout`) -- the rank-invariant aligned-tile kernel on the virtual
    layout (a date shard reproduces the full panel bit for bit)."""
    ret, mret, seg_lo = _f(ret), _f(mret), _i32(seg_lo)
    R = ret.numel()
    lam = 0.5 ** (1.0 / half_life)
    if ret.is_cuda and row_ord is not None and window <= ALIGN_MAX_W and R:
        v, seg_v, Rv = _layout(seg_lo, row_ord)
        bv = torch.empty(Rv, dtype=torch.float32, device=ret.device)
        hv = torch.empty_like(bv)
        # bound to names: a temporary passed as ptr(...) is freed before the launch, and the
        # caching allocator then hands its block to the next temporary (the inputs alias)
        yv, xv = _to_virtual(ret, v, Rv), _to_virtual(mret, v, Rv)
        _native.call("mfa_beta_hsigma_aligned", _native.ptr(yv), _native.ptr(xv), _native.ptr(seg_v), Rv, window, lam,
                     min_periods, _native.ptr(bv), _native.ptr(hv), _native.stream(ret.device))
        return bv[v].contiguous(), hv[v].contiguous()
    if ret.is_cuda:
        b, h = torch.empty_like(ret), torch.empty_like(ret)
        _native.call("mfa_beta_hsigma", _native.ptr(ret), _native.ptr(mret), _native.ptr(seg_lo), R,
                     window, lam, min_periods, _native.ptr(b), _native.ptr(h), _native.stream(ret.device))
        return b, h
    y, x, s = ret.double().numpy(), mret.double().numpy(), seg_lo.numpy()
    wfull = lam ** np.arange(window - 1, -1, -1)
    b = np.full(R, np.nan)
    h = np.full(R, np.nan)
    for r in range(R):
        lo = max(s[r], r - window + 1)
        yy, xx = y[lo:r + 1], x[lo:r + 1]
        ok = np.isfinite(yy) & np.isfinite(xx)
        n = int(ok.sum())
        if n < min_periods or n <= 2:
            continue
        w = wfull[-n:]
        X = np.column_stack([np.ones(n), xx[ok]])
        sw = np.sqrt(w)
        coef, *_ = np.linalg.lstsq(X * sw[:, None], yy[ok] * sw, rcond=None)
        e = yy[ok] - X @ coef
        b[r] = coef[1]
        h[r] = math.sqrt((w * e * e).sum() / (n - 2))
    return torch.from_numpy(b).float(), torch.from_numpy(h).float()


# ---------------------------------------------------------------- RSTR
def rstr(log_ret, seg_lo, T=504, L=21, half_life=126.0, min_periods=42):
    lr, seg_lo = _f(log_ret), _i32(seg_lo)
    R = lr.numel()
    W = T - L
    lam = 0.5 ** (1.0 / half_life)
    if lr.is_cuda:
        out = torch.empty_like(lr)
        _native.call("mfa_rstr", _native.ptr(lr), _native.ptr(seg_lo), R, L, W, lam, min_periods,
                     _native.ptr(out), _native.stream(lr.device))
        return out
    v, s = lr.double().numpy(), seg_lo.numpy()
    out = np.full(R, np.nan)
    for r in range(R):
        lo = max(s[r], r - W + 1)
        js = np.arange(lo, r + 1)
        src = js - L
        xv = np.where(src >= s[r], v[np.clip(src, 0, None)], np.nan)
        w = lam ** np.arange(len(js))
        ok = np.isfinite(xv)
        if ok.sum() >= min_periods:
            out[r] = (xv[ok] * w[ok]).sum() / w[ok].sum()
    return torch.from_numpy(out).float()


# ---------------------------------------------------------------- DASTD
def dastd(ret, mret, seg_lo, window=252, half_life=42.0, min_periods=42, row_ord=None):
    """``row_ord``: the rank-invariant aligned-tile kernel (see :func:`beta_hsigma`)."""
    ret, mret, seg_lo = _f(ret), _f(mret), _i32(seg_lo)
    R = ret.numel()
    lam = 0.5 ** (1.0 / half_life)
    if ret.is_cuda and row_ord is not None and window <= ALIGN_MAX_W and R:
        v, seg_v, Rv = _layout(seg_lo, row_ord)
        ov = torch.empty(Rv, dtype=torch.float32, device=ret.device)
        yv, xv = _to_virtual(ret, v, Rv), _to_virtual(mret, v, Rv)   # named: see beta_hsigma
        _native.call("mfa_dastd_aligned", _native.ptr(yv), _native.ptr(xv), _native.ptr(seg_v), Rv, window, lam,
                     min_periods, _native.ptr(ov), _native.stream(ret.device))
        return ov[v].contiguous()
    if ret.is_cuda:
        out = torch.empty_like(ret)
        _native.call("mfa_dastd", _native.ptr(ret), _native.ptr(mret), _native.ptr(seg_lo), R, window,
                     lam, min_periods, _native.ptr(out), _native.stream(ret.device))
        return out
    e, s = (ret.double() - mret.double()).numpy(), seg_lo.numpy()
    wfull = lam ** np.arange(window - 1, -1, -1)
    out = np.full(R, np.nan)
    for r in range(R):
        lo = max(s[r], r - window + 1)
        xv = e[lo:r + 1]
        xv = xv[np.isfinite(xv)]
        n = len(xv)
        if n < min_periods:
            continue
        w = wfull[-n:] / wfull[-n:].sum()
        m = (xv * w).sum()
        out[r] = math.sqrt((w * (xv - m) ** 2).sum())
    return torch.from_numpy(out).float()


# ---------------------------------------------------------------- CMRA
def cmra(log_ret, seg_lo, window=252, partial=False):
    lr, seg_lo = _f(log_ret), _i32(seg_lo)
    R = lr.numel()
    if lr.is_cuda:
        out = torch.empty_like(lr)
        _native.call("mfa_cmra", _native.ptr(lr), _native.ptr(seg_lo), R, window, int(partial),
                     _native.ptr(out), _native.stream(lr.device))
        return out
    v, s = lr.double().numpy(), seg_lo.numpy()
    out = np.full(R, np.nan)
    for r in range(R):
        if not partial:
            if r - window + 1 < s[r]:
                continue
            w = v[r - window + 1:r + 1]
            if not np.isfinite(w).all():
                continue
        else:
            w = v[max(s[r], r - window + 1):r + 1]
            w = w[np.isfinite(w)]
            if len(w) == 0:
                continue
        z = np.exp(np.cumsum(w)) - 1
        out[r] = np.log(1 + z.max()) - np.log(1 + z.min())
    return torch.from_numpy(out).float()


# ---------------------------------------------------------------- rolling sums (liquidity)
def rolling_sum(x, seg_lo, window, min_periods, scale=1.0, log=False):
    x, seg_lo = _f(x), _i32(seg_lo)
    R = x.numel()
    if x.is_cuda:
        out = torch.empty_like(x)
        _native.call("mfa_rolling_sum", _native.ptr(x), _native.ptr(seg_lo), R, window, min_periods,
                     float(scale), int(log), _native.ptr(out), _native.stream(x.device))
        return out
    v, s = x.double().numpy() * scale, seg_lo.numpy()
    out = np.full(R, np.nan)
    for r in range(R):
        w = v[max(s[r], r - window + 1):r + 1]
        w = w[np.isfinite(w)]
        if len(w) >= min_periods:
            t = w.sum()
            out[r] = (np.nan if t == 0 else math.log(t)) if log else t
    return torch.from_numpy(out).float()


# ---------------------------------------------------------------- statement-row TTM, leverage
TTM_RESTATED, TTM_MULTIVALUE = 1, 2


def ttm_runs(stock_id, end_date, v):
    """Statement-row TTM on the device (``csrc/rolling.hip`` ttm_* kernels): rows sorted by
    (stock, date); a run = consecutive rows of one (stock, end_date); each row gets the
    NaN-skipping sum of its run's and the 3 previous runs' values (min 4), fp32-rounded like the
    rolling-sum path, as float64.  Returns ``(ttm [R] float64, flags int32 [1] device tensor)``:
    flag ``TTM_RESTATED`` = end_date moved backwards within a stock (the result is then not
    valid: use the sort-based path), ``TTM_MULTIVALUE`` = one statement carries two values."""
    sid = _i32(stock_id)
    e = end_date.to(torch.int64).contiguous()
    x = _f(v)
    R = x.numel()
    dev = x.device
    start = torch.empty(R, dtype=torch.int32, device=dev)
    flags = torch.zeros(1, dtype=torch.int32, device=dev)
    out = torch.empty(R, dtype=torch.float64, device=dev)
    if R == 0:
        return out, flags
    st = _native.stream(dev)
    _native.call("mfa_ttm_flags", _native.ptr(sid), _native.ptr(e), _native.ptr(x), R,
                 _native.ptr(start), _native.ptr(flags), st)
    run_incl = torch.cumsum(start, 0, dtype=torch.int32)
    vf = torch.empty(R, dtype=torch.float32, device=dev)
    rsid = torch.empty(R, dtype=torch.int32, device=dev)
    _native.call("mfa_ttm_finish", _native.ptr(sid), _native.ptr(x), _native.ptr(start),
                 _native.ptr(run_incl), R, _native.ptr(vf), _native.ptr(rsid), _native.ptr(out), st)
    return out, flags


def leverage(mv, ncl, be):
    """(MLEV, BLEV) float32 (factor_calculator.py:464-509) in one device pass."""
    mv, ncl, be = _f(mv), _f(ncl), _f(be)
    mlev, blev = torch.empty_like(mv), torch.empty_like(mv)
    _native.call("mfa_leverage", _native.ptr(mv), _native.ptr(ncl), _native.ptr(be), mv.numel(),
                 _native.ptr(mlev), _native.ptr(blev), _native.stream(mv.device))
    return mlev, blev
