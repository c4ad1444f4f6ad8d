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
    # the scan runs over all T dates whatever the window, so every window is bitwise the slice
    # of the full series (rank-invariant gather mode)
    ws = torch.empty(max(8, _ws_bytes(T, K, q)), dtype=torch.uint8, device=F.device)
    _native.call("mfa_nw_series", _native.ptr(F), T, K, q, float(tau), t_lo, t_hi,
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


# ------------------------------------------------------------------------------------------
# Time-axis scan across date shards (SURVEY 2.5 "SP": block carries + exclusive scan across
# ranks + q-row halo).  Every state the expanding-window statistics carry is a decayed sum, so
# the state at date T0 - 1 of shard r is  sum_{r' < r} l^(T0_r - T1_r') own_r'  where own_r' is
# shard r''s contribution at its last date (its own dates only; the lag products f_{s-i} f_s are
# attributed to the shard owning s, which reads f_{s-i} from a q-row halo).  Two small
# collectives per call: the heads / tails of every shard (halo rows and the global first q rows)
# and the own-contribution states (O(q K^2) per rank), then each rank scans only its own dates:
# O(T K^2 q / world) work instead of every rank rescanning the whole gathered series.
# ------------------------------------------------------------------------------------------
_native.register("mfa_nw_state_doubles", [C.c_int, C.c_int])
_native.register("mfa_nw_shard_workspace_bytes", [C.c_int, C.c_int, C.c_int, C.c_int])
_native.register("mfa_nw_series_shard", [C.c_void_p, C.c_void_p, C.c_void_p, C.c_int, C.c_int,
                                          C.c_int, C.c_int, C.c_double, C.c_void_p, C.c_void_p,
                                          C.c_void_p, C.c_void_p, C.c_void_p, C.c_void_p])
_native.register("mfa_ew_prefix_mean_shard", [C.c_void_p, C.c_int, C.c_double, C.c_void_p,
                                               C.c_void_p, C.c_void_p, C.c_void_p])


def _nw_state_cpu(K: int, q: int, dev) -> dict:
    z = lambda *s: torch.zeros(*s, dtype=torch.float64, device=dev)  # noqa: E731
    return {"Z": z(1), "m": z(K), "S0": z(K, K), "A": z(q, K, K), "a": z(q, K), "b": z(q, K),
            "z": z(q)}


def _flat(st: dict) -> torch.Tensor:
    return torch.cat([st[k].reshape(-1) for k in ("Z", "m", "S0", "A", "a", "b", "z")])


def _unflat(v: torch.Tensor, K: int, q: int) -> dict:
    st, o = {}, 0
    for k, shape in (("Z", (1,)), ("m", (K,)), ("S0", (K, K)), ("A", (q, K, K)), ("a", (q, K)),
                     ("b", (q, K)), ("z", (q,))):
        n = math.prod(shape)
        st[k] = v[o:o + n].reshape(shape).clone()
        o += n
    return st


def _nw_shard_cpu(Fx: torch.Tensor, h: int, T0: int, q: int, lam: float, st: dict | None,
                  emit: bool):
    """float64 recurrence over the shard's dates [T0, T0 + D) of ``Fx`` = [halo h rows | shard].
    st None: the shard's own contribution (zero state in, returns the state at its last date);
    otherwise the carried state at T0 - 1 (returns V [D, K, K])."""
    D, K = Fx.shape[0] - h, Fx.shape[1]
    own = st is None
    st = _nw_state_cpu(K, q, Fx.device) if own else {k: v.clone() for k, v in st.items()}
    Z, m, S0, A, a, b, z = (st[k] for k in ("Z", "m", "S0", "A", "a", "b", "z"))
    V = torch.full((D, K, K), float("nan"), dtype=torch.float64, device=Fx.device) if emit else None
    for du in range(D):
        u = T0 + du
        fu = Fx[h + du]
        Z.mul_(lam).add_(1.0)
        m.mul_(lam).add_(fu)
        S0.mul_(lam).add_(torch.outer(fu, fu))
        for ii in range(q):
            i = ii + 1
            A[ii] *= lam
            a[ii] *= lam
            b[ii] *= lam
            z[ii] *= lam
            if u >= i:
                g = Fx[h + du - i]
                A[ii] += torch.outer(g, fu)
                a[ii] += g
                b[ii] += fu
                z[ii] += 1.0
        n = u + 1
        if emit and n > q and n > K:
            Zs = Z[0]
            mu = m / Zs
            Vu = S0 / Zs - torch.outer(mu, mu)
            for ii in range(q):
                i = ii + 1
                G = (A[ii] - torch.outer(a[ii], mu) - torch.outer(mu, b[ii])
                     + z[ii] * torch.outer(mu, mu)) / Zs
                Vu = Vu + (1.0 - i / (q + 1)) * (G + G.T)
            V[du] = Vu
    return V if emit else _flat(st)


def _rows_from_ends(t_lo: int, t_hi: int, seg_bounds: list, heads: list, tails: list, q: int,
                    K: int, dev) -> torch.Tensor:
    """Global rows [t_lo, t_hi) assembled from the segments' first / last q rows."""
    out = torch.zeros(max(0, t_hi - t_lo), K, dtype=torch.float64, device=dev)
    for t in range(max(0, t_lo), t_hi):
        for (a, b), hd, tl in zip(seg_bounds, heads, tails):
            if a <= t < b:
                if t - a < q and hd is not None:
                    out[t - t_lo] = hd[t - a]
                else:  # within the last q rows of the segment (tail stored end-aligned)
                    out[t - t_lo] = tl[q - (b - t)]
                break
    return out


def newey_west_series_sharded(F_own: torch.Tensor, q: int, tau: float, ctx=None,
                              sizes: list | None = None,
                              history: torch.Tensor | None = None) -> torch.Tensor:
    """This rank's block of the expanding-window Newey-West series from ITS factor returns only.

    ``F_own`` [D, K]: the rank's contiguous date block (rank order = date order); ``sizes``:
    every rank's D (``parallel.dist.shard_sizes``); ``history`` [T_h, K]: factor returns of
    dates before every rank's block (checkpoint resume), identical on all ranks.  Returns
    V [D, K, K] equal to ``newey_west_series(all_F)[T0:T0 + D]`` (to rounding: the scan order
    differs from the single-GPU chunking; the default risk-model path gathers F instead and is
    bitwise identical to one GPU)."""
    from ..parallel import dist as pdist
    ctx = ctx or pdist.context()
    F_own = F_own.to(torch.float64).contiguous()
    D, K = F_own.shape
    dev = F_own.device
    sizes = sizes if sizes is not None else pdist.shard_sizes(D, ctx)
    rank = ctx.rank if ctx.enabled else 0
    Th = 0 if history is None else int(history.shape[0])
    starts = [Th + sum(sizes[:r]) for r in range(len(sizes))]
    T0, T1 = starts[rank], starts[rank] + D
    lam = 0.5 ** (1.0 / tau)
    hq = max(q, 1)
    gpu = F_own.is_cuda
    # 1. heads / tails of every shard (halo rows, and the global first q rows)
    pad = torch.zeros(hq, K, dtype=torch.float64, device=dev)
    head = torch.cat([F_own[:hq], pad])[:hq]
    tail = torch.cat([pad, F_own[-hq:] if D else pad])[-hq:]
    ends = pdist.all_gather_rows(torch.cat([head, tail]).contiguous(), ctx,
                                 [2 * hq] * len(sizes)).reshape(len(sizes), 2, hq, K)
    bounds = [(s, s + n) for s, n in zip(starts, sizes)]
    heads, tails = [e[0] for e in ends], [e[1] for e in ends]
    if history is not None and Th:
        hist = history.to(dev, torch.float64)
        bounds = [(0, Th)] + bounds
        hh = torch.cat([hist[:hq], pad])[:hq]
        ht = torch.cat([pad, hist[-hq:]])[-hq:]
        heads, tails = [hh] + heads, [ht] + tails
    lo = max(0, T0 - hq)
    Fx = torch.cat([_rows_from_ends(lo, T0, bounds, heads, tails, hq, K, dev), F_own])
    h = T0 - lo
    # 2. own contributions (the history's too, computed identically on every rank)
    def own_state(Fx_, h_, T0_, n_):
        if not gpu:
            return _nw_shard_cpu(Fx_, h_, T0_, q, lam, None, emit=False)
        ns = _native.query("mfa_nw_state_doubles", K, q)
        ctot = torch.empty(ns + K, dtype=torch.float64, device=dev)
        ws = torch.empty(max(8, _native.query("mfa_nw_shard_workspace_bytes", T0_, T0_ + n_, K, q)),
                         dtype=torch.uint8, device=dev)
        _native.call("mfa_nw_series_shard", _native.ptr(Fx_), None, None, T0_, T0_ + n_, K, q,
                     float(tau), None, None, _native.ptr(ctot), _native.ptr(ctot[ns:]),
                     _native.ptr(ws), _native.stream(dev))
        return ctot
    mine = own_state(Fx, h, T0, D) if D else None
    nst = (_native.query("mfa_nw_state_doubles", K, q) + K) if gpu else \
        _flat(_nw_state_cpu(K, q, dev)).numel()
    if mine is None:
        mine = torch.zeros(nst, dtype=torch.float64, device=dev)
    own_all = pdist.all_gather_rows(mine[None].contiguous(), ctx, [1] * len(sizes))
    segs = list(zip([(s, s + n) for s, n in zip(starts, sizes)], own_all))
    if history is not None and Th:
        segs = [((0, Th), own_state(hist, 0, 0, Th))] + segs
    # 3. exclusive combine: state at T0 - 1
    cin = torch.zeros(nst, dtype=torch.float64, device=dev)
    for (a, b), o in segs:
        if b <= T0:
            cin += (lam ** (T0 - b)) * o
    if D == 0:
        return torch.empty(0, K, K, dtype=torch.float64, device=dev)
    # 4. scan of the own dates from the carried state
    if not gpu:
        return _nw_shard_cpu(Fx, h, T0, q, lam, _unflat(cin, K, q), emit=True)
    ns = nst - K
    M_in = cin[ns:]
    Mh = torch.empty(h, K, dtype=torch.float64, device=dev)  # global M rows [lo, T0)
    if h:
        Mh[h - 1] = M_in
        for j in range(h - 1, 0, -1):  # M[t - 1] = (M[t] - f_t) / l
            Mh[j - 1] = (Mh[j] - Fx[j]) / lam
    first = _rows_from_ends(0, min(q, T1), bounds, heads, tails, hq, K, dev)
    Mg = torch.empty(max(1, first.shape[0]), K, dtype=torch.float64, device=dev)
    acc = torch.zeros(K, dtype=torch.float64, device=dev)
    for t in range(first.shape[0]):
        acc = lam * acc + first[t]
        Mg[t] = acc
    V = torch.empty(D, K, K, dtype=torch.float64, device=dev)
    ws = torch.empty(max(8, _native.query("mfa_nw_shard_workspace_bytes", T0, T1, K, q)),
                     dtype=torch.uint8, device=dev)
    _native.call("mfa_nw_series_shard", _native.ptr(Fx), _native.ptr(Mh) if h else None,
                 _native.ptr(Mg), T0, T1, K, q, float(tau), _native.ptr(cin[:ns]) if T0 else None,
                 _native.ptr(V), None, None, _native.ptr(ws), _native.stream(dev))
    return V


def ew_prefix_mean_sharded(x_own: torch.Tensor, tau: float, ctx=None, sizes: list | None = None,
                           history: torch.Tensor | None = None) -> torch.Tensor:
    """This rank's block of :func:`ew_prefix_mean` over the concatenated series (history, then
    every rank's block in rank order): one all_gather of the (num, den) own totals."""
    from ..parallel import dist as pdist
    ctx = ctx or pdist.context()
    x_own = x_own.to(torch.float64).contiguous()
    D = x_own.shape[0]
    dev = x_own.device
    sizes = sizes if sizes is not None else pdist.shard_sizes(D, ctx)
    rank = ctx.rank if ctx.enabled else 0
    lam = 0.5 ** (1.0 / tau)

    def totals(x):
        if x.is_cuda:
            tot = torch.zeros(2, dtype=torch.float64, device=dev)
            if x.shape[0]:
                _native.call("mfa_ew_prefix_mean_shard", _native.ptr(x), x.shape[0], float(tau),
                             None, None, _native.ptr(tot), _native.stream(dev))
            return tot
        num = den = 0.0
        for v in x.tolist():
            ok = math.isfinite(v)
            num = lam * num + (v if ok else 0.0)
            den = lam * den + (1.0 if ok else 0.0)
        return torch.tensor([num, den], dtype=torch.float64, device=dev)
    own_all = pdist.all_gather_rows(totals(x_own)[None].contiguous(), ctx, [1] * len(sizes))
    Th = 0 if history is None else int(history.shape[0])
    starts = [Th + sum(sizes[:r]) for r in range(len(sizes))]
    T0 = starts[rank]
    cin = torch.zeros(2, dtype=torch.float64, device=dev)
    for s, n, o in zip(starts, sizes, own_all):
        if s + n <= T0:
            cin += (lam ** (T0 - s - n)) * o
    if Th:
        cin += (lam ** (T0 - Th)) * totals(history.to(dev, torch.float64).contiguous())
    if D == 0:
        return torch.empty(0, dtype=torch.float64, device=dev)
    if x_own.is_cuda:
        out = torch.empty_like(x_own)
        _native.call("mfa_ew_prefix_mean_shard", _native.ptr(x_own), D, float(tau),
                     _native.ptr(cin), _native.ptr(out), None, _native.stream(dev))
        return out
    num, den = float(cin[0]), float(cin[1])
    out = torch.empty(D, dtype=torch.float64)
    for t, v in enumerate(x_own.tolist()):
        ok = math.isfinite(v)
        num = lam * num + (v if ok else 0.0)
        den = lam * den + (1.0 if ok else 0.0)
        out[t] = num / den if den > 0 else float("nan")
    return out.to(dev)
