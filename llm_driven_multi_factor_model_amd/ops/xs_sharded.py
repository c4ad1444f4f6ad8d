"""Stock-sharded (tensor-parallel) cross-sectional WLS, SURVEY.md §2.5 "TP".

The date-sharded path (``cross_section.xs_wls`` on a rank's dates) is the default: at N = 5000 a
date's slice is ~250 KB and every date is independent.  For universes with N >> 10^4 stocks
(or panels too large for one GPU's dates), the STOCK axis is sharded instead.  Every rank holds
its stocks for all dates and

1. streams them into the raw weighted moments of ``CrossSection.reg`` (the same K1 layout as the
   fused kernel).  Moments are sums over stocks, so one ``all_reduce(SUM)`` of D x msize fp64
   gives every rank the full-universe moments (~9.7 MB at D = 2520, P = 31, Q = 10);
2. solves every date redundantly from the summed moments (K2, identical on every rank);
3. forms its own stocks' specific returns and the five R^2 sums (sum e, sum e^2, sum r, sum r^2,
   n) per date.  A second ``all_reduce`` of D x 5 fp64 completes R^2.

Two collectives per call, both sized by D, never by N.  The CPU path (gloo tests, CPU runs)
implements the same decomposition with torch ops on the raw K x K moment matrix
``G = Xf^T W Xf`` of ``[1 | one-hot | raw styles]``.  The z-scoring is the affine map T applied
after the reduction (``G_std = T^T G T``), so it reproduces ``xs_wls_reference`` (pinv semantics).

Reference: ``Barra-master/mfm/CrossSection.py:57-108`` (one date, all stocks in one process).
"""
from __future__ import annotations

import ctypes as C

import torch

from .. import _native
from .cross_section import (XS_BAD_SIGMA, XS_NO_ROWS, XS_PIVOT_EMPTY, XsResult, _validate,
                            valid_mask)

_vp, _i, _d = C.c_void_p, C.c_int, C.c_double
_native.register("mfa_xs_moments", [_vp, _vp, _vp, _vp, _i, _i, _i, _i, _vp, _vp])
_native.register("mfa_xs_solve", [_vp, _i, _i, _i, _i, _d, _vp, _vp, _vp, _vp, _vp])
_native.register("mfa_xs_resid_sums", [_vp, _vp, _vp, _vp, _i, _i, _i, _i, _vp, _vp, _vp, _vp, _vp])
_native.register("mfa_xs_moments_bytes", [_i, _i])
_native.register("mfa_xs_refine_coef", [_vp, _i, _i, _i, _i, _vp, _vp, _vp, _vp])
_native.register("mfa_xs_moments_f64", [_vp, _vp, _vp, _vp, _i, _i, _i, _i, _vp, _vp])
_native.register("mfa_xs_resid_sums_f64", [_vp, _vp, _vp, _vp, _i, _i, _i, _i, _vp, _vp, _vp, _vp,
                                           _vp])

_BAD = XS_NO_ROWS | XS_BAD_SIGMA | XS_PIVOT_EMPTY


def _all_reduce(t: torch.Tensor, ctx) -> torch.Tensor:
    """SUM over ranks; CPU tensors travel through the backend's device (RCCL needs HBM)."""
    if ctx is None or not ctx.enabled:
        return t
    import torch.distributed as dist
    x = t if t.device == ctx.device else t.to(ctx.device)
    dist.all_reduce(x, op=dist.ReduceOp.SUM)
    return x if x is t else x.to(t.device)


def _r2_from_sums(sums: torch.Tensor, status: torch.Tensor) -> torch.Tensor:
    a, b, c, e2, n = sums.unbind(-1)
    ve = b / n - (a / n) ** 2
    vr = e2 / n - (c / n) ** 2
    r2 = 1.0 - ve / vr
    return torch.where((status & _BAD) != 0, torch.full_like(r2, float("nan")), r2)


# ------------------------------------------------------------------------------- CPU path
def _moments_cpu(X, cap, ret, ind, P):
    """Per-date additive moments [D, K*K + K + Q + 4 + P] of the local stocks (fp64)."""
    D, Q, N = X.shape
    K = 1 + P + Q
    m = valid_mask(X, cap, ret, ind, P)
    mf = m.double()
    z = torch.zeros((), dtype=torch.float64)
    x = torch.where(m[:, None, :], X.double(), z).transpose(1, 2)  # [D, N, Q]
    c = torch.where(m, cap.double(), z)
    r = torch.where(m, ret.double(), z)
    cols = [mf[..., None]]
    if P > 0:
        oh = torch.nn.functional.one_hot(ind.long().clamp(0, P - 1), P).double() * mf[..., None]
        cols.append(oh)
    cols.append(x)
    Xf = torch.cat(cols, 2)  # [D, N, K] raw columns
    w = torch.sqrt(c)
    G = (Xf * w[..., None]).transpose(1, 2) @ Xf
    h = (Xf * (w * r)[..., None]).sum(1)
    parts = [G.reshape(D, K * K), h, c.sum(1, keepdim=True), (c[..., None] * x).sum(1),
             x.sum((1, 2))[:, None], (x * x).sum((1, 2))[:, None], mf.sum(1, keepdim=True)]
    if P > 0:
        parts.append((oh * c[..., None]).sum(1))
    return torch.cat(parts, 1)


def _solve_cpu(mom, P, Q, pivot_mode):
    """``xs_wls_reference`` algebra from the summed moments: returns f, f_raw, stats, status."""
    D = mom.shape[0]
    K = 1 + P + Q
    o = 0
    G = mom[:, :K * K].view(D, K, K); o += K * K
    h = mom[:, o:o + K]; o += K
    Sc = mom[:, o]; o += 1
    Scx = mom[:, o:o + Q]; o += Q
    Sx, Sxx, n = mom[:, o], mom[:, o + 1], mom[:, o + 2]; o += 3
    s = mom[:, o:o + P] if P > 0 else None
    mu = Scx / Sc[:, None]
    nq = n * Q
    sigma = torch.sqrt(torch.clamp(Sxx / nq - (Sx / nq) ** 2, min=0.0))
    # z = (x - mu) / sigma as a column map: Xf_std = Xf_raw @ T
    T = torch.eye(K, dtype=torch.float64).repeat(D, 1, 1)
    T[:, 0, 1 + P:] = -mu / sigma[:, None]
    T[:, 1 + P:, 1 + P:] = torch.diag_embed((1.0 / sigma)[:, None].expand(D, Q))
    Gs = T.transpose(1, 2) @ G @ T
    hs = (T.transpose(1, 2) @ h[..., None]).squeeze(-1)
    status = torch.zeros(D, dtype=torch.int32)
    if P > 0:
        if pivot_mode == 1:
            piv = torch.full((D,), P - 1, dtype=torch.long)
        else:
            last = torch.where(s > 0, torch.arange(P).expand_as(s), torch.full_like(s, -1, dtype=torch.long))
            piv = last.max(1).values
            piv = torch.where(piv < 0, torch.full_like(piv, P - 1), piv)
        sp = s.gather(1, piv[:, None]).squeeze(1)
        status |= torch.where(sp > 0, 0, XS_PIVOT_EMPTY).int()
        Rm = torch.eye(K, dtype=torch.float64).repeat(D, 1, 1)
        Rm[torch.arange(D), 1 + piv, 1:1 + P] = -s / sp[:, None]
        keep = torch.ones(D, K, dtype=torch.bool)
        keep[torch.arange(D), 1 + piv] = False
        Rm = Rm[keep[:, None, :].expand(-1, K, -1)].view(D, K, K - 1)
        A = Rm.transpose(1, 2) @ Gs @ Rm
        rhs = (Rm.transpose(1, 2) @ hs[..., None]).squeeze(-1)
    else:
        Rm, A, rhs = None, Gs, hs
    good = torch.isfinite(A).all(-1).all(-1)
    Ai = torch.full_like(A, float("nan"))
    if good.any():
        Ai[good] = torch.linalg.pinv(A[good], rtol=1e-15, hermitian=False)
    g = (Ai @ rhs[..., None]).squeeze(-1)
    f = (Rm @ g[..., None]).squeeze(-1) if Rm is not None else g
    status |= torch.where(n > 0, 0, XS_NO_ROWS).int()
    status |= torch.where((sigma > 0) & torch.isfinite(sigma), 0, XS_BAD_SIGMA).int()
    f[(status & _BAD) != 0] = float("nan")
    f_raw = (T @ f[..., None]).squeeze(-1)
    stats = torch.cat([mu, sigma[:, None], n[:, None]], 1)
    return f, f_raw, stats, status


def _resid_cpu(X, cap, ret, ind, P, f_raw):
    D, Q, N = X.shape
    m = valid_mask(X, cap, ret, ind, P)
    fr = f_raw
    fit = fr[:, :1] + (X.double() * fr[:, 1 + P:, None]).sum(1)
    if P > 0:
        fit = fit + fr[:, 1:1 + P].gather(1, ind.long().clamp(0, P - 1))
    e = ret.double() - fit
    e = torch.where(m, e, torch.full_like(e, float("nan")))
    em = torch.where(m, e, torch.zeros_like(e))
    r = torch.where(m, ret.double(), torch.zeros_like(e))
    sums = torch.stack([em.sum(1), (em * em).sum(1), r.sum(1), (r * r).sum(1), m.double().sum(1)], 1)
    return e.to(X.dtype) if X.dtype in (torch.float32, torch.float64) else e.float(), sums


def _xs_sharded_cpu(X, cap, ret, ind, P, ctx, pivot_mode, want_resid):
    mom = _all_reduce(_moments_cpu(X, cap, ret, ind, P), ctx)
    f, f_raw, stats, status = _solve_cpu(mom, P, X.shape[1], pivot_mode)
    e, sums = _resid_cpu(X, cap, ret, ind, P, f_raw)
    sums = _all_reduce(sums, ctx)
    return XsResult(f=f, resid=e if want_resid else None, r2=_r2_from_sums(sums, status),
                    stats=stats, status=status)


# ------------------------------------------------------------------------------- GPU path
def xs_wls_stock_sharded(X: torch.Tensor, cap: torch.Tensor, ret: torch.Tensor,
                         ind: torch.Tensor | None, P: int, ctx=None, *, pivot_mode: int = 0,
                         tol: float = 1e-14, want_resid: bool = True,
                         refine: bool = True) -> XsResult:
    """Regress every date with this rank's STOCKS ``[D, Q, N_local]`` (all ranks hold the same
    dates).  Returns full-universe ``f``, ``r2``, ``stats`` and ``status`` (identical on every
    rank) and this rank's ``resid`` columns.  ``ctx`` = ``parallel.dist`` context (None or world
    1: plain single-process run).  ``refine`` re-solves the dates the solve flags near-singular
    with the device pseudo-inverse (pinv semantics, quirk Q4) from the all-reduced moments,
    before the residual pass: no host synchronisation and no extra collective (the flags and
    the moments are identical on every rank).
    """
    D, Q, N = _validate(X, cap, ret, ind, P)
    if not X.is_cuda:
        return _xs_sharded_cpu(X, cap, ret, ind, P, ctx, pivot_mode, want_resid)
    dev = X.device
    K = 1 + P + Q
    dt = X.dtype if X.dtype == torch.float64 else torch.float32
    sfx = "_f64" if dt == torch.float64 else ""
    X = _native.check_device_tensor(X, dt, "X")
    cap = _native.check_device_tensor(cap, dt, "cap")
    ret = _native.check_device_tensor(ret, dt, "ret")
    if P > 0:
        ind = _native.check_device_tensor(ind, torch.int16, "ind")
    Np = (N + 7) // 8 * 8  # 16-byte rows for the residual pass; padding = absent stocks
    Xp, cp, rp, ip = X, cap, ret, ind
    if Np != N:
        pad = Np - N
        Xp = torch.nn.functional.pad(X, (0, pad), value=float("nan"))
        cp = torch.nn.functional.pad(cap, (0, pad), value=float("nan"))
        rp = torch.nn.functional.pad(ret, (0, pad), value=float("nan"))
        if P > 0:
            ip = torch.nn.functional.pad(ind, (0, pad), value=-1)
    MS = _native.query("mfa_xs_moments_bytes", P, Q) // 8
    mom = torch.empty(D, MS, dtype=torch.float64, device=dev)
    st = _native.stream(dev)
    iptr = _native.ptr(ip if P > 0 else None)
    _native.call("mfa_xs_moments" + sfx, _native.ptr(Xp), _native.ptr(cp), _native.ptr(rp), iptr, D, Np,
                 P, Q, _native.ptr(mom), st)
    _all_reduce(mom, ctx)                                      # collective 1: D x msize fp64
    f = torch.empty(D, K, dtype=torch.float64, device=dev)
    coef = torch.empty(D, Q + 1 + P, dtype=torch.float64, device=dev)
    stats = torch.empty(D, Q + 2, dtype=torch.float64, device=dev)
    status = torch.empty(D, dtype=torch.int32, device=dev)
    _native.call("mfa_xs_solve", _native.ptr(mom), D, P, Q, pivot_mode, tol, _native.ptr(f),
                 _native.ptr(coef), _native.ptr(stats), _native.ptr(status), st)
    if refine:  # device pinv of flagged dates: rewrites f / coef / status in place, any K
        _native.call("mfa_xs_refine_coef", _native.ptr(mom), D, P, Q, pivot_mode, _native.ptr(f),
                     _native.ptr(coef), _native.ptr(status), st)
    e = torch.empty(D, Np, dtype=dt, device=dev) if want_resid else None
    sums = torch.empty(D, 5, dtype=torch.float64, device=dev)
    _native.call("mfa_xs_resid_sums" + sfx, _native.ptr(Xp), _native.ptr(cp), _native.ptr(rp), iptr, D,
                 Np, P, Q, _native.ptr(coef), _native.ptr(status), _native.ptr(e),
                 _native.ptr(sums), st)
    _all_reduce(sums, ctx)                                     # collective 2: D x 5 fp64
    return XsResult(f=f, resid=(e[:, :N] if Np != N else e) if want_resid else None,
                    r2=_r2_from_sums(sums, status), stats=stats, status=status)
