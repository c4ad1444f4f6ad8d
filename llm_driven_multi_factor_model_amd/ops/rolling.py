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
# direct per-row kernels (reference kernels, fallback beyond the segment kernels' limits)
_native.register("mfa_beta_hsigma", [_vp, _vp, _vp, _i, _i, _d, _i, _vp, _vp, _vp])
_native.register("mfa_rstr", [_vp, _vp, _i, _i, _i, _d, _i, _vp, _vp])
_native.register("mfa_dastd", [_vp, _vp, _vp, _i, _i, _d, _i, _vp, _vp])
_native.register("mfa_cmra", [_vp, _vp, _i, _i, _i, _vp, _vp])
_native.register("mfa_rolling_sum", [_vp, _vp, _i, _i, _i, _d, _i, _vp, _vp])
# segment-anchored kernels on the segment layout (the production path)
_native.register("mfa_beta_hsigma_seg", [_vp, _vp, _vp, _vp, _i, _i, _d, _i, _vp, _vp, _vp])
_native.register("mfa_dastd_seg", [_vp, _vp, _vp, _vp, _i, _i, _d, _i, _vp, _vp])
_native.register("mfa_rstr_seg", [_vp, _vp, _vp, _i, _i, _i, _d, _i, _vp, _vp])
_native.register("mfa_window_sums_seg", [_vp, _vp, _vp, _i, _i, _vp, _vp, _d, _i, _vp, _vp, _vp, _vp])
_native.register("mfa_cmra_seg", [_vp, _vp, _vp, _i, _i, _vp, _vp])
_native.register("mfa_seg_count", [_vp, _vp, _i, _vp, _vp])
_native.register("mfa_seg_place", [_vp, _vp, _vp, _i, _i, _vp, _vp, _i, _vp, _vp, _vp])
_native.register("mfa_returns", [_vp, _vp, _i, _vp, _vp, _vp])
_native.register("mfa_ttm_flags", [_vp, _vp, _vp, _i, _vp, _vp, _vp])
_native.register("mfa_ttm_finish", [_vp, _vp, _vp, _vp, _i, _vp, _vp, _vp, _vp])
_native.register("mfa_leverage", [_vp, _vp, _vp, _i, _vp, _vp, _vp])

# Segment layout (csrc/rolling.hip, "segment-anchored window kernels"): every stock's rows sit
# at virtual positions B_s + t - T0_s, t = the row's ordinal in the stock's FULL history, B_s and
# T0_s multiples of ALIGN, so the kernels' anchor segments fall on fixed ordinals whatever slice
# of the history a launch holds.
ALIGN = 256        # virtual block size (stock histories padded to multiples of it)
EW_SEG = 256       # BETA / DASTD anchor segments (prefixes anchored one segment back)
POS_SEG = 64       # RSTR / window sums / CMRA anchor segments (the window's first row's segment)
EW_MAX_W = 256     # segment kernels' window limits; larger windows take the direct kernels
POS_MAX_REACH = 512
CMRA_MIN_W, CMRA_MAX_W = 65, 257


def ew_reach(window: int) -> int:
    """Rows of a stock's history before an output row that BETA / DASTD of that row depend on
    (the anchor: the start of the 256-row segment before the row's own)."""
    return 2 * EW_SEG - 1 if window <= EW_MAX_W else window - 1


def pos_reach(window: int, lag: int = 0) -> int:
    """The same for a positional window over sources [r - window + 1 - lag, r - lag] (RSTR,
    the turnover sums): its first source's 64-row segment."""
    r = window + lag - 1
    return r + POS_SEG - 1 if r <= POS_MAX_REACH else r


def cmra_reach(window: int, partial: bool = False) -> int:
    seg = not partial and CMRA_MIN_W <= window <= CMRA_MAX_W
    return window - 1 + (POS_SEG - 1 if seg else 0)


def aligned_layout(seg_lo: torch.Tensor, row_ord: torch.Tensor):
    """The segment layout's index vectors: (v [R] int64 virtual position of every row,
    seg_v [Rv] int32 virtual stock start of every virtual position -- a padding position is its
    own start --, Rv)."""
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


class SegLayout:
    """The segment layout of a set of flat stock-sorted rows (built once per engine and shared
    by every descriptor): ``seg_v`` [Rv] virtual stock starts, ``omap`` [Rv] the real row of
    every virtual position (-1 on padding), and :meth:`virt` -- a series in virtual positions
    (NaN padding), cached per source tensor.  ``row_ord``: each row's ordinal in its stock's
    full history (default: the rows ARE the full histories).  ``series``: float32 [R] tensors
    placed in the same pass as the layout (GPU: csrc/rolling.hip seg_count / seg_place, three
    row-parallel kernels around one int32 prefix sum)."""

    def __init__(self, seg_lo: torch.Tensor, row_ord: torch.Tensor | None = None, series=()):
        seg_lo = _i32(seg_lo)
        R = seg_lo.numel()
        dev = seg_lo.device
        self.R = R
        self._virt = {}
        if dev.type != "cuda":
            if row_ord is None:
                row_ord = torch.arange(R, device=dev, dtype=torch.int32) - seg_lo
            self.v, self.seg_v, self.Rv = aligned_layout(seg_lo, row_ord)
            self.omap = torch.full((self.Rv,), -1, dtype=torch.int32, device=dev)
            self.omap[self.v] = torch.arange(R, device=dev, dtype=torch.int32)
            for x in series:
                self.virt(x)
            return
        ro = None if row_ord is None else _i32(row_ord)
        st = _native.stream(dev)
        nb = torch.empty(R, dtype=torch.int32, device=dev)
        _native.call("mfa_seg_count", _native.ptr(seg_lo), _native.ptr(ro), R, _native.ptr(nb), st)
        incl = torch.cumsum(nb, 0, dtype=torch.int32)
        self.Rv = int(incl[-1]) * ALIGN if R else 0   # the one host read
        self.seg_v = torch.empty(self.Rv, dtype=torch.int32, device=dev)
        self.omap = torch.empty(self.Rv, dtype=torch.int32, device=dev)
        self._ro, self._incl, self._seg_lo = ro, incl, seg_lo   # for virt() of later series
        series = [x for x in series if x is not None]
        for k in range(0, max(len(series), 1), 4):
            self._place(series[k:k + 4], first=k == 0)

    def _place(self, xs, first: bool) -> None:
        """GPU: place up to 4 series (and, on the first call, the layout vectors themselves)."""
        dev = self.seg_v.device
        srcs = [_f(x) for x in xs]
        dsts = [torch.empty(self.Rv, dtype=torch.float32, device=dev) for _ in xs]
        sv, om = (self.seg_v, self.omap) if first else (None, None)   # None: series only
        S = (C.c_void_p * 4)(*[x.data_ptr() for x in srcs], *[0] * (4 - len(srcs)))
        D = (C.c_void_p * 4)(*[x.data_ptr() for x in dsts], *[0] * (4 - len(dsts)))
        _native.call("mfa_seg_place", _native.ptr(self._seg_lo), _native.ptr(self._ro),
                     _native.ptr(self._incl), self.R, self.Rv, _native.ptr(sv), _native.ptr(om),
                     len(xs), C.cast(S, _vp), C.cast(D, _vp), _native.stream(dev))
        for x, d in zip(xs, dsts):
            self._virt[id(x)] = (x, d)   # the source stays referenced: its id cannot be reused

    def virt(self, x: torch.Tensor) -> torch.Tensor:
        hit = self._virt.get(id(x))
        if hit is not None and hit[0] is x:
            return hit[1]
        if x.is_cuda:
            self._place([x], first=False)
            return self._virt[id(x)][1]
        out = torch.full((self.Rv,), float("nan"), dtype=torch.float32, device=x.device)
        out[self.v] = x.to(torch.float32)
        self._virt[id(x)] = (x, out)
        return out


def _layout(seg_lo, row_ord, series=()) -> SegLayout:
    """``row_ord``: None (the rows are full histories), ordinals, or a ready :class:`SegLayout`.
    A layout built here places ``series`` in its first pass (one launch for layout + inputs)."""
    return row_ord if isinstance(row_ord, SegLayout) else SegLayout(seg_lo, row_ord, series)


def _f(t):
    return t.to(torch.float32).contiguous()


_DIRECT = [False]


@contextlib.contextmanager
def direct_kernels(on: bool = True):
    """Run the GPU descriptors on the direct per-row kernels inside the block (every row sums
    its own window in one fixed order: the tests' reference kernels).  Nests: the previous
    setting comes back on exit."""
    prev = _DIRECT[0]
    _DIRECT[0] = bool(on)
    try:
        yield
    finally:
        _DIRECT[0] = prev


def _seg_path(x: torch.Tensor) -> bool:
    return x.is_cuda and x.numel() > 0 and not _DIRECT[0]


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
    """GPU: the segment-anchored kernel (window <= 256) on the segment layout of ``row_ord``
    (None = the rows are full histories; ordinals; or a :class:`SegLayout`), else the direct
    per-row kernel.  Either way a row's value depends only on its stock's rows from its anchor
    on: a date shard holding :func:`ew_reach` rows before its first owned row reproduces the
    full-panel outputs bit for bit."""
    R = ret.numel()
    lam = 0.5 ** (1.0 / half_life)
    if _seg_path(ret) and window <= EW_MAX_W:
        lay = _layout(seg_lo, row_ord, (ret, mret))
        b = torch.empty(R, dtype=torch.float32, device=ret.device)
        h = torch.empty_like(b)
        # bound to names: a temporary passed as ptr(...) is freed before the launch, and the
        # caching allocator then hands its block to the next temporary (the inputs alias)
        yv, xv = lay.virt(ret), lay.virt(mret)
        _native.call("mfa_beta_hsigma_seg", _native.ptr(yv), _native.ptr(xv), _native.ptr(lay.seg_v),
                     _native.ptr(lay.omap), lay.Rv, window, lam, min_periods, _native.ptr(b),
                     _native.ptr(h), _native.stream(ret.device))
        return b, h
    ret, mret, seg_lo = _f(ret), _f(mret), _i32(seg_lo)
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
def rstr(log_ret, seg_lo, T=504, L=21, half_life=126.0, min_periods=42, row_ord=None):
    """GPU: the segment-anchored positional-window kernel (reach T - 1 <= 512) on the segment
    layout of ``row_ord`` (see :func:`beta_hsigma`), else the direct kernel."""
    R = log_ret.numel()
    W = T - L
    lam = 0.5 ** (1.0 / half_life)
    if _seg_path(log_ret) and W >= 1 and L >= 0 and W + L - 1 <= POS_MAX_REACH:
        lay = _layout(seg_lo, row_ord, (log_ret,))
        out = torch.empty(R, dtype=torch.float32, device=log_ret.device)
        xv = lay.virt(log_ret)
        _native.call("mfa_rstr_seg", _native.ptr(xv), _native.ptr(lay.seg_v), _native.ptr(lay.omap),
                     lay.Rv, L, W, lam, min_periods, _native.ptr(out), _native.stream(out.device))
        return out
    lr, seg_lo = _f(log_ret), _i32(seg_lo)
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
    """GPU: the segment-anchored kernel (see :func:`beta_hsigma`)."""
    R = ret.numel()
    lam = 0.5 ** (1.0 / half_life)
    if _seg_path(ret) and window <= EW_MAX_W:
        lay = _layout(seg_lo, row_ord, (ret, mret))
        out = torch.empty(R, dtype=torch.float32, device=ret.device)
        yv, xv = lay.virt(ret), lay.virt(mret)   # named: see beta_hsigma
        _native.call("mfa_dastd_seg", _native.ptr(yv), _native.ptr(xv), _native.ptr(lay.seg_v),
                     _native.ptr(lay.omap), lay.Rv, window, lam, min_periods, _native.ptr(out),
                     _native.stream(ret.device))
        return out
    ret, mret, seg_lo = _f(ret), _f(mret), _i32(seg_lo)
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
def cmra(log_ret, seg_lo, window=252, partial=False, row_ord=None):
    """GPU: full windows with 64 < window <= 257 take the segment-anchored kernel on the
    segment layout of ``row_ord`` (see :func:`beta_hsigma`); the partial-window variant (quirk
    Q15) and other windows the direct kernel (rank-invariant too)."""
    R = log_ret.numel()
    if _seg_path(log_ret) and not partial and CMRA_MIN_W <= window <= CMRA_MAX_W:
        lay = _layout(seg_lo, row_ord, (log_ret,))
        out = torch.empty(R, dtype=torch.float32, device=log_ret.device)
        xv = lay.virt(log_ret)
        _native.call("mfa_cmra_seg", _native.ptr(xv), _native.ptr(lay.seg_v), _native.ptr(lay.omap),
                     lay.Rv, window, _native.ptr(out), _native.stream(out.device))
        return out
    lr, seg_lo = _f(log_ret), _i32(seg_lo)
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
def window_sums(x, seg_lo, windows, scale=1.0, log=False, row_ord=None):
    """Several NaN-skipping window sums of ``x * scale`` (``windows``: [(window, min_periods)],
    at most 3 per pass; ``log``: ln(sum), a zero sum -> NaN) -- STOM / STOQ / STOA in one pass
    of the segment-anchored kernel.  Returns a list of tensors."""
    R = x.numel()
    windows = [(int(w), int(m)) for w, m in windows]
    if not _seg_path(x) or any(w < 1 or w - 1 > POS_MAX_REACH for w, _ in windows):
        return [rolling_sum(x, seg_lo, w, m, scale, log) for w, m in windows]
    lay = _layout(seg_lo, row_ord, (x,))
    xv = lay.virt(x)
    outs = []
    for k in range(0, len(windows), 3):
        grp = windows[k:k + 3]
        o = [torch.empty(R, dtype=torch.float32, device=x.device) for _ in grp]
        W = (C.c_int * 3)(*[w for w, _ in grp], *[0] * (3 - len(grp)))
        M = (C.c_int * 3)(*[m for _, m in grp], *[0] * (3 - len(grp)))
        op = [_native.ptr(t) for t in o] + [None] * (3 - len(o))
        _native.call("mfa_window_sums_seg", _native.ptr(xv), _native.ptr(lay.seg_v), _native.ptr(lay.omap),
                     lay.Rv, len(grp), C.cast(W, _vp), C.cast(M, _vp), float(scale), int(log), *op,
                     _native.stream(x.device))
        outs += o
    return outs


def rolling_sum(x, seg_lo, window, min_periods, scale=1.0, log=False, row_ord=None):
    if _seg_path(x) and 1 <= window and window - 1 <= POS_MAX_REACH:
        return window_sums(x, seg_lo, [(window, min_periods)], scale, log, row_ord)[0]
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
