"""Batched cross-sectional WLS factor-return regression (kernel K1+K2+K3).

Semantics follow ``Barra-master/mfm/CrossSection.py``:

* style z-score ``(x - mu_c) / sigma`` with the cap-weighted mean ``mu_c`` and ONE pooled
  ddof-0 std over all N*Q style entries (``CrossSection.py:12-20``);
* WLS weights ``sqrt(cap)`` (the reference normalises them, ``:50``; the solution is scale
  invariant);
* industry-neutral constraint ``sum_j s_j f_j = 0`` with raw industry caps ``s_j``
  (``:66-71``), pseudo-inverse solve (``:76``);
* ``f = Omega r``, ``e = r - X f``, unweighted ``R^2 = 1 - var(e)/var(r)`` (``:101-106``).

Ragged universes are expressed with ``ind < 0`` (absent stock) or any non-finite input.

Panels may be stored in float64 (the reference's own input precision: ``demo.py:21-35`` reads
float64 CSV columns) or float32 (the factor pipeline's downcast, ``load_data.py:18-21``); the
moments, the solve and every reduction are float64 either way, and specific returns come back
in the storage dtype.

GPU tensors run the fused HIP kernel (``csrc/xs_wls_impl.h``; ``mfa_xs_wls`` / ``mfa_xs_wls_f64``,
one launch for all dates) followed, with ``refine=True``, by the device pseudo-inverse pass
for near-singular dates (no host synchronisation).  CPU tensors run :func:`xs_wls_reference`,
a dense float64 transcription of the reference formula (batched ``pinv``) that also serves as
the numerics oracle for the kernel.
"""
from __future__ import annotations

from dataclasses import dataclass

import torch

from .. import _native

# status bits (csrc/xs_wls.hip XsStatus)
XS_NO_ROWS = 1
XS_PIVOT_EMPTY = 2
XS_NEAR_SINGULAR = 4
XS_ZERO_PIVOT = 8
XS_BAD_SIGMA = 16
XS_REFINED = 32          # re-solved by the device pseudo-inverse pass
# Industry count bounds: the fused kernel's in-kernel solve is sized for FUSED_MAX_P industries;
# up to XS_MAX_P the GPU runs the split kernels instead (moments -> solve -> device pinv ->
# residuals, the stock-sharded path at world size 1: csrc/xs_wls_impl.h kXsSplitMaxP).
FUSED_MAX_P = 128
XS_MAX_P = 256
XS_PINV_CUT = 128        # that pinv cut a direction below 1e-15 lambda_max (rank-deficient)
XS_DETERMINISTIC = 0x100  # pivot_mode flag of mfa_xs_wls: bitwise-deterministic kernel
XS_REFINE = 0x200         # pivot_mode flag: device pinv pass for near-singular dates
REFINE_MAX_K = 64         # full-matrix Jacobi pinv up to this K; structured device pinv above


@dataclass
class XsResult:
    """Per-date regression outputs (all dates of the shard).

    f:      [D, K] float64 factor returns, K = 1 + P + Q (country, industries, styles)
    resid:  [D, N] specific returns in the panel's dtype (NaN where the stock is absent) or None
    r2:     [D]    float64 unweighted R^2
    stats:  [D, Q+2] float64 = (cap-weighted style means, pooled sigma, n_valid)
    status: [D]    int32 XS_* bit flags
    """

    f: torch.Tensor
    resid: torch.Tensor | None
    r2: torch.Tensor
    stats: torch.Tensor
    status: torch.Tensor


def _validate(X, cap, ret, ind, P):
    if X.dim() != 3:
        raise ValueError("X must be [D, Q, N]")
    D, Q, N = X.shape
    if cap.shape != (D, N) or ret.shape != (D, N):
        raise ValueError(f"cap/ret must be [D, N] = {(D, N)}; got {tuple(cap.shape)}, {tuple(ret.shape)}")
    if P > 0 and (ind is None or ind.shape != (D, N)):
        raise ValueError("ind must be [D, N] when P > 0")
    if Q < 1:
        raise ValueError(f"Q={Q}: at least one style factor is needed (the pooled style sigma)")
    if X.is_cuda and Q > 16:  # the kernels' register / LDS layouts; the CPU path takes any Q, P
        raise ValueError(f"Q={Q} outside the GPU kernels' 1..16 range")
    if X.is_cuda and P > XS_MAX_P:
        raise ValueError(f"P={P} > {XS_MAX_P} industries is not supported on the GPU")
    return D, Q, N


def xs_wls(X: torch.Tensor, cap: torch.Tensor, ret: torch.Tensor, ind: torch.Tensor | None,
           P: int, *, pivot_mode: int = 0, tol: float = 1e-14, want_resid: bool = True,
           refine: bool = True, out: XsResult | None = None,
           workspace: torch.Tensor | None = None, deterministic: bool | None = None) -> XsResult:
    """Regress every date of the panel in one batched call.

    X [D,Q,N] styles, cap/ret [D,N] (all float64 or all float32), ind [D,N] int16 industry ids
    (or None if P == 0).
    ``pivot_mode`` 0 eliminates the last NON-EMPTY industry (identical solution whenever the
    reference's choice is valid); 1 reproduces the reference exactly (always the last column,
    NaN when it is empty, quirk Q3).  ``refine`` re-solves dates the kernel flags as
    near-singular with the pseudo-inverse (pinv semantics, quirk Q4): on the GPU a device pass
    in the same stream, no host sync, for any K (eigen-pinv of the constrained normal matrix for
    K <= 64; above, the structured pinv that eigen-decomposes only the dense block's Schur
    complement and projects out the null directions of the full matrix).
    ``out`` / ``workspace`` let a caller (e.g. a timed loop) reuse preallocated buffers.
    The GPU kernels need N % 8 == 0 (16-byte rows for the LDS-DMA ring); other N are padded
    here with absent stocks (``ind = -1``), which costs a copy — keep panels padded.
    ``deterministic`` (default: on whenever the kernel supports it, i.e. the 8-replica segment
    table fits, ``mfa_xs_det_supported``: P <= 57 industries at Q = 10) selects the
    bitwise-reproducible kernel: each LDS segment replica is owned by one wave and the wave
    partials are summed in a fixed order.  It costs 0-3 % (profiles/r02_xs_deterministic.md);
    ``False`` shares the replicas across waves (reproducible to rounding only).
    More than FUSED_MAX_P = 128 industries (up to XS_MAX_P = 256) run on the split kernels
    (moments -> solve -> device pinv -> residuals, :func:`.xs_sharded.xs_wls_stock_sharded` at
    world size 1): fresh outputs every call (``out`` / ``workspace`` are not used there) and a
    shared-replica industry table (reproducible to rounding only).
    """
    D, Q, N = _validate(X, cap, ret, ind, P)
    K = 1 + P + Q
    if not X.is_cuda:
        return xs_wls_reference(X, cap, ret, ind, P, pivot_mode=pivot_mode, want_resid=want_resid)
    if P > FUSED_MAX_P:
        from .xs_sharded import xs_wls_stock_sharded
        return xs_wls_stock_sharded(X, cap, ret, ind, P, None, pivot_mode=pivot_mode, tol=tol,
                                    want_resid=want_resid, refine=refine)
    dev = X.device
    dt = X.dtype
    if dt not in (torch.float32, torch.float64):
        raise TypeError(f"X: expected float32 or float64, got {dt}")
    X = _native.check_device_tensor(X, dt, "X")
    cap = _native.check_device_tensor(cap, dt, "cap")
    ret = _native.check_device_tensor(ret, dt, "ret")
    if P > 0:
        ind = _native.check_device_tensor(ind, torch.int16, "ind")
    Np = (N + 7) // 8 * 8
    if Np != N:
        pad = Np - N
        X = torch.nn.functional.pad(X, (0, pad), value=float("nan"))
        cap = torch.nn.functional.pad(cap, (0, pad), value=float("nan"))
        ret = torch.nn.functional.pad(ret, (0, pad), value=float("nan"))
        if P > 0:
            ind = torch.nn.functional.pad(ind, (0, pad), value=-1)
    if out is None:
        out = XsResult(
            f=torch.empty(D, K, dtype=torch.float64, device=dev),
            resid=torch.empty(D, N, dtype=dt, device=dev) if want_resid else None,
            r2=torch.empty(D, dtype=torch.float64, device=dev),
            stats=torch.empty(D, Q + 2, dtype=torch.float64, device=dev),
            status=torch.empty(D, dtype=torch.int32, device=dev),
        )
    resid_buf = out.resid
    if resid_buf is not None and Np != N:
        resid_buf = torch.empty(D, Np, dtype=dt, device=dev)
    need = _native.query("mfa_xs_wls_workspace", D, Np, P, Q)
    if workspace is None:
        workspace = torch.empty(need, dtype=torch.uint8, device=dev)
    elif workspace.numel() < need:
        # a silently reallocated buffer would defeat reuse and allocate inside captured graphs
        raise ValueError(f"xs_wls: workspace of {workspace.numel()} B is too small for D={D}, "
                         f"N={N}, P={P}, Q={Q} ({need} B): size it with xs_wls_workspace(D, P, "
                         "Q, device, N)")
    if deterministic is None:
        deterministic = bool(_native.lib().mfa_xs_det_supported(P, Q))
    flags = (XS_DETERMINISTIC if deterministic else 0) | (XS_REFINE if refine else 0)
    _native.call("mfa_xs_wls_f64" if dt == torch.float64 else "mfa_xs_wls", _native.ptr(X),
                 _native.ptr(cap), _native.ptr(ret),
                 _native.ptr(ind if P > 0 else None), D, Np, P, Q, pivot_mode | flags, tol,
                 _native.ptr(out.f), _native.ptr(resid_buf), _native.ptr(out.r2),
                 _native.ptr(out.stats), _native.ptr(out.status), _native.ptr(workspace),
                 _native.stream(dev))
    if resid_buf is not None and Np != N:
        out.resid.copy_(resid_buf[:, :N])
    return out


def xs_wls_workspace(D: int, P: int, Q: int, device, N: int) -> torch.Tensor:
    """Preallocated kernel workspace for repeated :func:`xs_wls` calls on the same shapes
    (its size depends on N -- per-tile validity bits -- and on the path, i.e. on the stock
    chunks per date chosen for (D, N)).  :func:`xs_wls` refuses a workspace that is too small."""
    Np = (N + 7) // 8 * 8
    return torch.empty(_native.query("mfa_xs_wls_workspace", D, Np, P, Q), dtype=torch.uint8,
                       device=device)


def valid_mask(X, cap, ret, ind, P) -> torch.Tensor:
    """Rows entering the regression: industry assigned, finite inputs, non-negative capital."""
    m = torch.isfinite(cap) & (cap >= 0) & torch.isfinite(ret) & torch.isfinite(X).all(dim=1)
    if P > 0:
        m &= (ind >= 0) & (ind < P)
    return m


def xs_wls_reference(X, cap, ret, ind, P, *, pivot_mode: int = 0, want_resid: bool = True,
                     chunk: int = 256) -> XsResult:
    """Dense float64 oracle, a direct batched transcription of ``CrossSection.reg``.

    Builds ``[1 | one-hot | z-scored styles]``, the constraint matrix ``R`` and solves with a
    batched ``pinv`` (numpy's rcond=1e-15 semantics), exactly the algebra of
    ``CrossSection.py:57-106`` minus the dense N x N weight matrix.
    """
    D, Q, N = X.shape
    K = 1 + P + Q
    fs, es, r2s, stats_l, sts = [], [], [], [], []
    for a in range(0, D, chunk):
        b = min(D, a + chunk)
        Xs = X[a:b].double().transpose(1, 2)  # [d,N,Q]
        c = cap[a:b].double()
        r = ret[a:b].double()
        m = valid_mask(X[a:b], cap[a:b], ret[a:b], ind[a:b] if P > 0 else None, P)
        mf = m.double()
        Xs = torch.where(m[..., None], Xs, torch.zeros((), dtype=torch.float64))
        c = torch.where(m, c, torch.zeros((), dtype=torch.float64))
        r = torch.where(m, r, torch.zeros((), dtype=torch.float64))
        n = mf.sum(1)
        Sc = c.sum(1)
        mu = (c[..., None] * Xs).sum(1) / Sc[:, None]
        nq = n * Q
        mean_all = Xs.sum((1, 2)) / nq
        sigma = torch.sqrt(torch.clamp((Xs * Xs).sum((1, 2)) / nq - mean_all ** 2, min=0.0))
        Xz = (Xs - mu[:, None, :]) / sigma[:, None, None] * mf[..., None]
        cols = [mf[..., None]]
        status = torch.zeros(b - a, dtype=torch.int32)
        if P > 0:
            oh = torch.nn.functional.one_hot(ind[a:b].long().clamp(0, P - 1), P).double() * mf[..., None]
            cols.append(oh)
        cols.append(Xz)
        Xf = torch.cat(cols, dim=2)  # [d,N,K]
        w = torch.sqrt(c)
        if P > 0:
            s = (oh * c[..., None]).sum(1)  # [d,P]
            if pivot_mode == 1:
                piv = torch.full((b - a,), P - 1, dtype=torch.long)
            else:
                nz = s > 0
                last = torch.where(nz, torch.arange(P).expand_as(s), torch.full_like(s, -1, dtype=torch.long))
                piv = last.max(1).values
                piv = torch.where(piv < 0, torch.full_like(piv, P - 1), piv)
            sp = s.gather(1, piv[:, None]).squeeze(1)
            status |= torch.where(sp > 0, 0, XS_PIVOT_EMPTY).int()
            Rm = torch.eye(K, dtype=torch.float64).repeat(b - a, 1, 1)
            rows = 1 + piv
            ratio = -s / sp[:, None]
            Rm[torch.arange(b - a), rows, 1:1 + P] = ratio
            keep = torch.ones(b - a, K, dtype=torch.bool)
            keep[torch.arange(b - a), rows] = False
            Rm = Rm[keep[:, None, :].expand(-1, K, -1)].view(b - a, K, K - 1)
            Xt = Xf @ Rm
        else:
            Rm = None
            Xt = Xf
        A = (Xt * w[..., None]).transpose(1, 2) @ Xt
        rhs = (Xt * (w * r)[..., None]).sum(1)
        good = torch.isfinite(A).all(-1).all(-1)
        Ai = torch.full_like(A, float("nan"))
        if good.any():
            Ai[good] = torch.linalg.pinv(A[good], rtol=1e-15, hermitian=False)
        g = (Ai @ rhs[..., None]).squeeze(-1)
        f = (Rm @ g[..., None]).squeeze(-1) if Rm is not None else g
        status |= torch.where(n > 0, 0, XS_NO_ROWS).int()
        status |= torch.where((sigma > 0) & torch.isfinite(sigma), 0, XS_BAD_SIGMA).int()
        bad = (status & (XS_NO_ROWS | XS_BAD_SIGMA | XS_PIVOT_EMPTY)) != 0
        f[bad] = float("nan")
        fit = (Xf @ f[..., None]).squeeze(-1)
        e = r - fit
        e = torch.where(m, e, torch.full_like(e, float("nan")))
        em = torch.where(m, e, torch.zeros_like(e))
        ve = (em * em).sum(1) / n - (em.sum(1) / n) ** 2
        vr = (r * r).sum(1) / n - (r.sum(1) / n) ** 2
        r2 = 1.0 - ve / vr
        r2[bad] = float("nan")
        fs.append(f)
        es.append(e.to(X.dtype) if X.dtype in (torch.float32, torch.float64) else e.float())
        r2s.append(r2)
        stats_l.append(torch.cat([mu, sigma[:, None], n[:, None]], 1))
        sts.append(status)
    return XsResult(f=torch.cat(fs), resid=torch.cat(es) if want_resid else None,
                    r2=torch.cat(r2s), stats=torch.cat(stats_l), status=torch.cat(sts))


def pure_factor_portfolio(X_d: torch.Tensor, cap_d: torch.Tensor, ind_d: torch.Tensor | None,
                          P: int, mu: torch.Tensor, sigma: float, pivot: int | None = None):
    """Pure-factor-portfolio weights ``Omega`` (K x N) and exposures ``Omega X`` for ONE date.

    Only the ``mfm.CrossSection.reg`` compatibility API needs the explicit K x N matrix
    (``CrossSection.py:76,104``); the batched path never forms it.  Runs with torch ops on
    whatever device the inputs live on.  ``X_d`` is [Q, N] raw styles of valid rows.
    """
    dt = torch.float64
    Xs = ((X_d.to(dt).T - mu.to(dt)) / sigma)
    N = Xs.shape[0]
    c = cap_d.to(dt)
    cols = [torch.ones(N, 1, dtype=dt, device=Xs.device)]
    if P > 0:
        cols.append(torch.nn.functional.one_hot(ind_d.long(), P).to(dt))
    cols.append(Xs)
    Xf = torch.cat(cols, 1)
    K = Xf.shape[1]
    w = torch.sqrt(c)
    if P > 0:
        s = (cols[1] * c[:, None]).sum(0)
        p = P - 1 if pivot is None else pivot
        R = torch.eye(K, dtype=dt, device=Xs.device)
        R[1 + p, 1:1 + P] = -s / s[p]
        R = torch.cat([R[:, :1 + p], R[:, 2 + p:]], 1)
        Xt = Xf @ R
        omega = R @ torch.linalg.pinv((Xt * w[:, None]).T @ Xt, rtol=1e-15) @ (Xt * w[:, None]).T
    else:
        omega = torch.linalg.pinv((Xf * w[:, None]).T @ Xf, rtol=1e-15) @ (Xf * w[:, None]).T
    return omega, omega @ Xf
