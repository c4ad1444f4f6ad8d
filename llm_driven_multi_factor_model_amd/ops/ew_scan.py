"""Expanding-window Newey-West / EWMA factor covariance series and decayed prefix means.

Reference: ``Barra-master/mfm/utils.py:16-50`` (``Newey_West``) evaluated on every prefix by
``MFM.Newey_West_by_time`` (``MFM.py:80-101``), and the VRA multiplier of
``MFM.vol_regime_adj_by_time`` (``MFM.py:149-164``).

The GPU path (``csrc/ew_scan.hip``) is a blocked decayed-moment scan: O(T K^2 q) work for the
whole series instead of the reference's O(T^2 K^2 q), one launch per pass and lag group, and an
output window ``[t_lo, t_hi)`` so a data-parallel rank writes only its own dates.  Any lag
count is accepted (the reference's ``Newey_West`` takes any ``q < T``; USE4-S uses 5): lags run
in register groups of 8, so only the chunk's LDS rows bound q (``mfa_nw_max_lags``, ~450 at
K = 42).  The CPU path is the same
recurrence in float64 torch.
"""
from __future__ import annotations

import ctypes as C
import math

import torch

from .. import _native

_native.register("mfa_nw_series", [C.c_void_p, C.c_int, C.c_int, C.c_int, C.c_double, C.c_int,
                                    C.c_int, C.c_void_p, C.c_void_p, C.c_void_p])
_native.register("mfa_ew_prefix_mean", [C.c_void_p, C.c_int, C.c_double, C.c_void_p, C.c_void_p])
_native.register("mfa_nw_workspace_bytes", [C.c_int, C.c_int, C.c_int])
_native.register("mfa_nw_max_lags", [C.c_int])


def _ws_bytes(T: int, K: int, q: int) -> int:
    return _native.query("mfa_nw_workspace_bytes", T, K, q)


def newey_west_series(F: torch.Tensor, q: int = 2, tau: float = 252.0, t_lo: int = 0,
                      t_hi: int | None = None) -> torch.Tensor:
    """Newey-West covariance of every expanding prefix.

    ``F`` [T, K] float64 factor returns.  Returns ``V`` [t_hi - t_lo, K, K] float64 with
    ``V[t - t_lo] = Newey_West(F[:t+1], q, tau)``; entries whose prefix length n satisfies
    ``n <= q or n <= K`` are NaN (the reference raises and stores an empty frame there).
    """
    T, K = F.shape
    t_hi = T if t_hi is None else t_hi
    if not (0 <= t_lo <= t_hi <= T):
        raise ValueError("invalid output window")
    if q < 0:
        raise ValueError("q must be >= 0")
    F = F.to(torch.float64).contiguous()
    if not F.is_cuda:
        return newey_west_series_reference(F, q, tau, t_lo, t_hi)
    qmax = _native.query("mfa_nw_max_lags", K)
    if q > qmax:
        raise ValueError(f"q={q} exceeds the GPU scan's LDS limit of {qmax} lags at K={K}")
    V = torch.empty(t_hi - t_lo, K, K, dtype=torch.float64, device=F.device)
    if t_hi == t_lo:
        return V
    ws = torch.empty(max(8, _ws_bytes(t_hi, K, q)), dtype=torch.uint8, device=F.device)
    _native.call("mfa_nw_series", _native.ptr(F), t_hi, K, q, float(tau), t_lo, t_hi,
                 _native.ptr(V), _native.ptr(ws), _native.stream(F.device))
    return V


def newey_west_series_reference(F: torch.Tensor, q: int = 2, tau: float = 252.0, t_lo: int = 0,
                                t_hi: int | None = None) -> torch.Tensor:
    """float64 recurrence (CPU) — identical algebra to the HIP scan, vectorised over K x K."""
    T, K = F.shape
    t_hi = T if t_hi is None else t_hi
    lam = 0.5 ** (1.0 / tau)
    F = F.double()
    dt, dev = torch.float64, F.device
    Z = torch.zeros((), dtype=dt, device=dev)
    m = torch.zeros(K, dtype=dt, device=dev)
    S0 = torch.zeros(K, K, dtype=dt, device=dev)
    A = torch.zeros(q, K, K, dtype=dt, device=dev)
    a = torch.zeros(q, K, dtype=dt, device=dev)
    b = torch.zeros(q, K, dtype=dt, device=dev)
    z = torch.zeros(q, dtype=dt, device=dev)
    out = torch.full((t_hi - t_lo, K, K), float("nan"), dtype=dt, device=dev)
    for u in range(t_hi):
        fu = F[u]
        Z = lam * Z + 1.0
        m = lam * m + fu
        S0 = lam * S0 + torch.outer(fu, fu)
        for ii in range(q):
            i = ii + 1
            A[ii] *= lam
            a[ii] *= lam
            b[ii] *= lam
            z[ii] *= lam
            if u >= i:
                g = F[u - i]
                A[ii] += torch.outer(g, fu)
                a[ii] += g
                b[ii] += fu
                z[ii] += 1.0
        n = u + 1
        if u >= t_lo and n > q and n > K:
            mu = m / Z
            V = S0 / Z - torch.outer(mu, mu)
            for ii in range(q):
                i = ii + 1
                G = (A[ii] - torch.outer(a[ii], mu) - torch.outer(mu, b[ii]) + z[ii] * torch.outer(mu, mu)) / Z
                V = V + (1.0 - i / (q + 1)) * (G + G.T)
            out[u - t_lo] = V
    return out


def newey_west_single(F: torch.Tensor, q: int = 2, tau: float = 252.0) -> torch.Tensor:
    """One Newey-West matrix of the full sample (``utils.Newey_West`` semantics), float64."""
    T, K = F.shape
    if T <= q or T <= K:
        raise ValueError("T <= q or T <= K")
    F = F.double()
    w = 0.5 ** (torch.arange(T - 1, -1, -1, dtype=torch.float64, device=F.device) / tau)
    w = w / w.sum()
    r = F - (w[:, None] * F).sum(0)
    V = (r * w[:, None]).T @ r
    for i in range(1, q + 1):
        G = (r[:-i] * w[i:, None]).T @ r[i:]
        V = V + (1 - i / (1 + q)) * (G + G.T)
    return V


def ew_prefix_mean(x: torch.Tensor, tau: float) -> torch.Tensor:
    """``out[t] = sum_{s<=t, finite} l^(t-s) x_s / sum_{s<=t, finite} l^(t-s)``, l = 0.5^(1/tau)."""
    x = x.to(torch.float64).contiguous()
    T = x.shape[0]
    if not x.is_cuda:
        return ew_prefix_mean_reference(x, tau)
    out = torch.empty_like(x)
    _native.call("mfa_ew_prefix_mean", _native.ptr(x), T, float(tau), _native.ptr(out),
                 _native.stream(x.device))
    return out


def ew_prefix_mean_reference(x: torch.Tensor, tau: float) -> torch.Tensor:
    lam = 0.5 ** (1.0 / tau)
    out = torch.empty_like(x, dtype=torch.float64)
    num = den = 0.0
    xs = x.double().cpu().tolist()
    for t, v in enumerate(xs):
        ok = math.isfinite(v)
        num = lam * num + (v if ok else 0.0)
        den = lam * den + (1.0 if ok else 0.0)
        out[t] = num / den if den > 0 else float("nan")
    return out.to(x.device)
