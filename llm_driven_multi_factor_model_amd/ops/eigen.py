"""Batched symmetric eigensolver and Monte-Carlo eigenfactor risk adjustment.

Reference: ``Barra-master/mfm/utils.py:55-92`` (``eigen_risk_adj``) applied per date by
``MFM.eigen_risk_adj_by_time`` (``MFM.py:105-126``).  GPU path: ``csrc/eigen.hip``.

Semantics kept from the reference:

* the simulation length defaults to the TOTAL number of dates for every date (quirk Q9);
* the same M draws are used for every date (``np.random.seed(m+1)``, quirk Q8) — here the
  draw covariances ``cov(z_m)`` come from a counter-based Philox stream keyed by ``(seed, m)``;
* a date whose covariance has a negative eigenvalue (or is NaN) yields NaN (the reference
  raises inside a bare ``except`` and stores an empty frame, quirk Q7/Q12).

Deliberate difference (documented, statistical parity only): eigenpairs are paired by
descending eigenvalue rank (the reference pairs by ``np.linalg.eig``'s unspecified order), and
the normals come from Philox rather than MT19937 (bitwise parity with numpy is impossible).
"""
from __future__ import annotations

import contextlib
import os
import ctypes as C

import torch

from .. import _native

_native.register("mfa_eigh_batched", [C.c_void_p, C.c_int, C.c_int, C.c_int, C.c_double,
                                       C.c_void_p, C.c_void_p, C.c_void_p, C.c_void_p])
_native.register("mfa_mc_cov", [C.c_int, C.c_int, C.c_int, C.c_uint64, C.c_void_p, C.c_void_p])
_native.register("mfa_eigen_adjust", [C.c_void_p, C.c_void_p, C.c_void_p, C.c_int, C.c_int,
                                       C.c_int, C.c_void_p, C.c_double, C.c_int, C.c_double,
                                       C.c_void_p, C.c_void_p, C.c_void_p, C.c_void_p])
_native.register("mfa_mc_cov_range", [C.c_int, C.c_int, C.c_int, C.c_int, C.c_uint64, C.c_void_p,
                                       C.c_void_p])
_native.register("mfa_mc_cov_ws_doubles", [C.c_int, C.c_int])
_native.register("mfa_mc_cov_range_ws", [C.c_int, C.c_int, C.c_int, C.c_int, C.c_uint64,
                                          C.c_void_p, C.c_void_p, C.c_void_p])
_native.register("mfa_eigen_bias_accumulate", [C.c_void_p, C.c_void_p, C.c_int, C.c_int, C.c_int,
                                                C.c_void_p, C.c_int, C.c_double, C.c_void_p,
                                                C.c_void_p, C.c_void_p])
_native.register("mfa_philox_normals", [C.c_int, C.c_int, C.c_int, C.c_int, C.c_uint64, C.c_void_p,
                                         C.c_void_p])
_native.register("mfa_eigen_bias_accumulate_wide", [C.c_void_p, C.c_void_p, C.c_int, C.c_int, C.c_int,
                                                     C.c_void_p, C.c_void_p, C.c_void_p, C.c_void_p])
_native.register("mfa_eigen_wide_set_variant", [C.c_int])
_native.register("mfa_eigh_wide", [C.c_void_p, C.c_int, C.c_int, C.c_void_p, C.c_void_p,
                                   C.c_void_p])
_native.register("mfa_eigh_wide_fix_psd", [C.c_void_p, C.c_int, C.c_int, C.c_double, C.c_double,
                                           C.c_void_p, C.c_void_p, C.c_void_p, C.c_void_p,
                                           C.c_void_p])
_native.register("mfa_eigh_wide_fix", [C.c_void_p, C.c_int, C.c_int, C.c_double, C.c_void_p,
                                       C.c_void_p, C.c_void_p, C.c_void_p, C.c_void_p])
_native.register("mfa_mc_cov_wide", [C.c_int, C.c_int, C.c_int, C.c_int, C.c_uint64, C.c_void_p,
                                     C.c_void_p, C.c_void_p])
_native.register("mfa_mc_cov_wide_ws_doubles", [C.c_int, C.c_int, C.c_int])
_native.register("mfa_eigen_set_date_origin", [C.c_int])
_native.register("mfa_eigen_xl_ws_doubles", [C.c_int, C.c_int])
_native.register("mfa_eigh_xl", [C.c_void_p, C.c_int, C.c_int, C.c_double, C.c_double, C.c_void_p,
                                 C.c_void_p, C.c_void_p, C.c_void_p, C.c_void_p])
_native.register("mfa_eigen_bias_accumulate_xl", [C.c_void_p, C.c_void_p, C.c_int, C.c_int, C.c_int,
                                                  C.c_void_p, C.c_void_p, C.c_void_p, C.c_void_p,
                                                  C.c_void_p])
_native.register("mfa_eigen_xl_set_wpe", [C.c_int])
_native.register("mfa_mc_cov_xl_ws_doubles", [C.c_int, C.c_int, C.c_int])
_native.register("mfa_mc_cov_xl", [C.c_int, C.c_int, C.c_int, C.c_int, C.c_uint64, C.c_void_p,
                                   C.c_void_p, C.c_void_p])
_native.register("mfa_eigen_finalize_sum", [C.c_void_p, C.c_int, C.c_void_p, C.c_void_p,
                                             C.c_void_p, C.c_int, C.c_int, C.c_double, C.c_void_p,
                                             C.c_void_p, C.c_void_p])

MAX_SWEEPS = 30
TOL = 1e-15
# Factor sets wider than one wave (K > 64, e.g. SW-L2 industries: K = 140) leave the
# register-resident one-wave kernels.  Up to WIDE_HIP_MAX_K everything stays on hand-written
# kernels: the draw covariances on the fp64 matrix cores (mc_cov_wide_kernel, the same Philox
# stream: factor k < 64 of a sim is the same number at any K), the F0 eigh and the bias statistic
# on the multi-wave tridiagonal solver (csrc/eigen_wide.hip, with a device orthogonality check
# and Jacobi re-solve; KP = 96 / 144 / 160 instantiations), the finalize on eigen_finalize_kernel.
# From WIDE_HIP_MAX_K to XL_MAX_K the
# XL kernels take over (csrc/eigen_xl.hip: one persistent 8-wave workgroup per problem with its
# working matrix in a global slot; output-tiled MFMA draw covariances in csrc/eigen.hip), still
# with no vendor library and no host synchronisation.  Only K > XL_MAX_K (or the "rocsolver"
# A/B setting) uses rocSOLVER's batched symmetric solver and a rocBLAS GEMM in bounded chunks.
WIDE_K = 64
ORTHO_TOL = 1e-10                # wide eigh: max |U^T U - I| above this -> device Jacobi re-solve
WIDE_CHUNK_DOUBLES = 1 << 27     # ~1 GB of fp64 per batched eigh / draw chunk
# Bias statistic for 64 < K <= WIDE_HIP_MAX_K: "hip" (default: csrc/eigen_wide.hip, mode 5's
# tridiagonal solver on one 2-3-wave workgroup per (date, sim): 4.6 us per 140 x 140 problem at
# the GPU's throughput, within 3e-14 of rocSOLVER, profiles/r04/wide_bias_ab.jsonl) or
# "rocsolver" (batched syevd through torch: 27.7 us).  Wider K always takes rocSOLVER.
# MFA_WIDE_BIAS selects the solver at import.
WIDE_HIP_MAX_K = 160   # KP = 96 / 144 / 160 instantiations of the multi-wave kernels
XL_MAX_K = 1024
WIDE_BIAS_SOLVERS = ("rocsolver", "hip")
_wide_solver = os.environ.get("MFA_WIDE_BIAS", "hip")
if _wide_solver not in WIDE_BIAS_SOLVERS:  # a typo must not silently select rocSOLVER
    raise ValueError(f"MFA_WIDE_BIAS must be one of {WIDE_BIAS_SOLVERS}, got {_wide_solver!r}")


def set_wide_bias_solver(name: str) -> None:
    """Select the bias-statistic solver for factor sets wider than one wave (process-wide)."""
    global _wide_solver
    if name not in WIDE_BIAS_SOLVERS:
        raise ValueError(f"wide bias solver must be one of {WIDE_BIAS_SOLVERS}, got {name!r}")
    _wide_solver = name


# Layout of the "hip" wide solver: "pair" = two lanes per matrix row (default: half the registers
# per lane; 3 waves per problem for K <= 96, 5 for K > 96; K = 80 bias 8.2 vs 10.1 ms with
# "mixed", profiles/r06/wide_householder/layout_ab.log), "mixed" = one lane per row for K <= 96 and
# two for K > 96 (round 5's default), "row" = one lane per row at every K (A/B builds only).
WIDE_LAYOUTS = {"row": 0, "mixed": 1, "pair": 2}


def set_wide_kernel_layout(name: str) -> None:
    if name not in WIDE_LAYOUTS:
        raise ValueError(f"wide kernel layout must be one of {sorted(WIDE_LAYOUTS)}, got {name!r}")
    if _native.lib().mfa_eigen_wide_set_variant(WIDE_LAYOUTS[name]) != 0:
        raise ValueError(f"wide kernel layout {name!r} is an A/B variant (MFA_AB build only)")


@contextlib.contextmanager
def using_wide_bias_solver(name: str):
    global _wide_solver
    old = _wide_solver
    set_wide_bias_solver(name)
    try:
        yield
    finally:
        _wide_solver = old

# Per-(date, sim) solver of the bias statistic (csrc/eigen.hip): "tridiag" (mode 5, the default)
# = Householder tridiagonalisation, count-guided Laguerre eigenvalues (division-free Sturm
# recurrence), twisted-factorisation eigenvectors, back-transform, lean register / LDS layout;
# "tridiag_chain" (mode 21, opt-in; ~3 % faster before round 5's eps ||T|| tolerance, level after
# it, and now ~25 % SLOWER: its date loop keeps the 8-step reflector groups and 64-entry LDS
# tables, which the default's 2-step groups / KP-entry tables outrun, profiles/r05) = the same
# solver with each wave walking 8
# consecutive dates of a sim, the Laguerre iteration of every eigenvalue rank started from the
# previous date's (chains aligned to global multiples of 8 through ``date0``: bitwise
# rank-invariant only for date shards that start on a chain boundary, e.g. sims sharding);
# "jacobi" = pair-block tournament Jacobi carrying M = V^T D0 V.  A/B builds only (``_build
# --ab``, slower in their measurements): "tridiag_v1" / "tridiag_lean" = the round-2 kernel
# (mode 3) / lean layout with the pivot-form Sturm recurrence (mode 4); "tridiag_dense" = mode
# 5's arithmetic with three problems on the 126 lanes of a 2-wave workgroup (mode 11, K <= 42).
BIAS_SOLVERS = {"jacobi": 0, "tridiag": 5, "tridiag_chain": 21, "tridiag_v1": 3, "tridiag_lean": 4,
                "tridiag_dense": 11}
PRODUCTION_BIAS_SOLVERS = ("jacobi", "tridiag", "tridiag_chain")
_bias_solver = "tridiag"


def available_bias_solvers() -> tuple[str, ...]:
    """Solvers the loaded kernel library contains (all of BIAS_SOLVERS in an A/B build)."""
    if torch.cuda.is_available() and _native.ab_build():
        return tuple(sorted(BIAS_SOLVERS))
    return PRODUCTION_BIAS_SOLVERS


def set_bias_solver(name: str) -> None:
    """Select the GPU bias-statistic solver (process-wide)."""
    global _bias_solver
    if name not in BIAS_SOLVERS:
        raise ValueError(f"bias solver must be one of {sorted(BIAS_SOLVERS)}, got {name!r}")
    if torch.cuda.is_available():
        if _native.lib().mfa_eigen_set_bias_mode(BIAS_SOLVERS[name]) != 0:
            raise ValueError(f"bias solver {name!r} is an A/B variant: not in this kernel library "
                             f"(build it with python -m llm_driven_multi_factor_model_amd._build "
                             f"--ab and set MFA_HIP_LIB)")
    _bias_solver = name


def bias_solver() -> str:
    return _bias_solver


@contextlib.contextmanager
def using_bias_solver(name: str):
    old = _bias_solver
    set_bias_solver(name)
    try:
        yield
    finally:
        set_bias_solver(old)


LAST_EIGH_FLAGS: torch.Tensor | None = None


def eigh(A: torch.Tensor, max_sweeps: int = MAX_SWEEPS, tol: float = TOL, *,
         resolve_psd_tol: float | None = None):
    """Batched symmetric eigendecomposition, eigenvalues DESCENDING.

    ``A`` [..., K, K] float64 (any K; K > 64 on the GPU goes through :func:`_eigh_wide`).  Returns ``(w [..., K], U [..., K, K])``
    with ``A = U diag(w) U^T`` and ``U[..., :, k]`` the k-th eigenvector.  Non-finite input
    matrices give NaN outputs.
    """
    A = A.to(torch.float64)
    shp = A.shape
    K = shp[-1]
    Ab = A.reshape(-1, K, K).contiguous()
    if not A.is_cuda:
        return _eigh_reference(Ab, shp)
    if K > WIDE_K:
        return _eigh_wide(Ab, shp, resolve_psd_tol)
    B = Ab.shape[0]
    w = torch.empty(B, K, dtype=torch.float64, device=A.device)
    U = torch.empty(B, K, K, dtype=torch.float64, device=A.device)
    # Householder-tridiagonal eigh; `flags` marks matrices whose eigenvectors came out
    # non-orthogonal (clustered spectra), re-solved by the Jacobi in the same call (no sync)
    flags = torch.empty(B, dtype=torch.int32, device=A.device)
    _native.call("mfa_eigh_batched", _native.ptr(Ab), B, K, max_sweeps, tol, _native.ptr(w),
                 _native.ptr(U), _native.ptr(flags), _native.stream(A.device))
    global LAST_EIGH_FLAGS
    LAST_EIGH_FLAGS = flags   # diagnostics (tools/risk_timing.py): matrices re-solved by Jacobi
    return w.reshape(shp[:-1]), U.reshape(shp)


def _eigh_wide(Ab, shp, resolve_psd_tol=None):
    """K > 64 on the device: for K <= WIDE_HIP_MAX_K the multi-wave HIP solver
    (``mfa_eigh_wide_fix``: matrices whose eigenvectors come out non-orthogonal to ORTHO_TOL,
    i.e. clustered spectra, or NaN for a finite input, are re-solved on the device by a Jacobi),
    otherwise rocSOLVER's batched eigh of the finite (symmetrised) matrices in chunks of
    ~WIDE_CHUNK_DOUBLES; NaN for non-finite inputs.  Eigenvalues descending."""
    B, K = Ab.shape[0], Ab.shape[-1]
    if _wide_solver == "hip" and K <= WIDE_HIP_MAX_K:
        w = torch.empty(B, K, dtype=torch.float64, device=Ab.device)
        U = torch.empty(B, K, K, dtype=torch.float64, device=Ab.device)
        ws = torch.empty(B * K * K, dtype=torch.float64, device=Ab.device)
        # tridiagonal EIG kernel, then per matrix max |U^T U - I| on the matrix cores and a
        # device Jacobi re-solve of the finite matrices that fail it (no host synchronisation)
        flags = torch.empty(B, dtype=torch.int32, device=Ab.device)
        psd = -1.0 if resolve_psd_tol is None else float(resolve_psd_tol)
        _native.call("mfa_eigh_wide_fix_psd", _native.ptr(Ab), B, K, ORTHO_TOL, psd, _native.ptr(w),
                     _native.ptr(U), _native.ptr(ws), _native.ptr(flags), _native.stream(Ab.device))
        global LAST_EIGH_FLAGS
        LAST_EIGH_FLAGS = flags
        return w.reshape(shp[:-1]), U.reshape(shp)
    if _wide_solver == "hip" and K <= XL_MAX_K:
        return _eigh_xl(Ab, shp, resolve_psd_tol)
    w = torch.full((B, K), float("nan"), dtype=torch.float64, device=Ab.device)
    U = torch.full((B, K, K), float("nan"), dtype=torch.float64, device=Ab.device)
    ok = torch.isfinite(Ab).all(-1).all(-1)
    idx = torch.nonzero(ok).flatten()
    step = max(1, WIDE_CHUNK_DOUBLES // (K * K))
    for a in range(0, idx.numel(), step):
        sel = idx[a:a + step]
        S = Ab[sel]
        ww, UU = torch.linalg.eigh(0.5 * (S + S.transpose(-1, -2)))
        w[sel] = ww.flip(-1)
        U[sel] = UU.flip(-1)
    return w.reshape(shp[:-1]), U.reshape(shp)


def _eigh_xl(Ab, shp, resolve_psd_tol=None):
    """WIDE_HIP_MAX_K < K <= XL_MAX_K: ``mfa_eigh_xl`` (csrc/eigen_xl.hip) -- Householder with the
    working matrix in a per-workgroup global slot, bisection eigenvalues, twisted-factorisation
    eigenvectors, an MFMA orthogonality check and an in-slot Jacobi re-solve of the matrices that
    fail it; no host synchronisation."""
    B, K = Ab.shape[0], Ab.shape[-1]
    dev = Ab.device
    w = torch.empty(B, K, dtype=torch.float64, device=dev)
    U = torch.empty(B, K, K, dtype=torch.float64, device=dev)
    flags = torch.empty(B, dtype=torch.int32, device=dev)
    ws = torch.empty(max(1, _native.query("mfa_eigen_xl_ws_doubles", B, K)), dtype=torch.float64,
                     device=dev)
    psd = -1.0 if resolve_psd_tol is None else float(resolve_psd_tol)
    _native.call("mfa_eigh_xl", _native.ptr(Ab), B, K, ORTHO_TOL, psd, _native.ptr(w), _native.ptr(U),
                 _native.ptr(flags), _native.ptr(ws), _native.stream(dev))
    global LAST_EIGH_FLAGS
    LAST_EIGH_FLAGS = flags
    return w.reshape(shp[:-1]), U.reshape(shp)


def set_xl_waves_per_simd(w: int) -> None:
    """XL solver occupancy (process-wide; bitwise the same results): 2 = one 8-wave workgroup per
    CU, 4 = two workgroups per CU in 128 VGPRs, 0 = auto (default: 4 for the bias batches, 2 for
    the eigh)."""
    if _native.lib().mfa_eigen_xl_set_wpe(int(w)) != 0:
        raise ValueError(f"XL waves per SIMD must be 0, 2 or 4, got {w!r}")


def _eigh_reference(Ab, shp):
    K = Ab.shape[-1]
    ok = torch.isfinite(Ab).all(-1).all(-1)
    w = torch.full(Ab.shape[:-1], float("nan"), dtype=torch.float64)
    U = torch.full(Ab.shape, float("nan"), dtype=torch.float64)
    if ok.any():
        S = 0.5 * (Ab[ok] + Ab[ok].transpose(-1, -2))
        ww, UU = torch.linalg.eigh(S)
        w[ok] = ww.flip(-1)
        U[ok] = UU.flip(-1)
    return w.reshape(shp[:-1]), U.reshape(shp)


def mc_cov(M: int, K: int, T: int, seed: int = 1, device="cuda", m0: int = 0) -> torch.Tensor:
    """Draw covariances ``cov(z_m)`` (ddof 1) of simulations ``m0 .. m0+M-1``, each an
    independent [T x K] standard-normal panel.

    Every simulation has its own counter-based stream keyed by ``(seed, m)`` (Philox on the GPU,
    a per-sim ``torch.Generator`` on the CPU), so splitting the sims over chunks or ranks draws
    exactly the covariances of one unsplit call.
    """
    dev = torch.device(device)
    if dev.type != "cuda":
        Cz = torch.empty(M, K, K, dtype=torch.float64)
        for i in range(M):
            g = torch.Generator().manual_seed((int(seed) * 1_000_003 + m0 + i) & 0x7FFFFFFFFFFFFFFF)
            z = torch.randn(T, K, generator=g, dtype=torch.float64)
            Cz[i] = torch.cov(z.T)
        return Cz
    if K > WIDE_K:
        return _mc_cov_wide(M, K, T, seed, dev, m0)
    Cz = torch.empty(M, K, K, dtype=torch.float64, device=dev)
    # the time axis is split into chunks that depend on T only (partials added in chunk order),
    # so a sim's covariance is bitwise the same in any launch that contains it
    nws = _native.query("mfa_mc_cov_ws_doubles", M, T)
    ws = torch.empty(max(1, nws), dtype=torch.float64, device=dev)
    _native.call("mfa_mc_cov_range_ws", M, int(m0), K, T, int(seed) & 0xFFFFFFFFFFFFFFFF,
                 _native.ptr(ws), _native.ptr(Cz), _native.stream(dev))
    return Cz


def _mc_cov_wide(M: int, K: int, T: int, seed: int, dev, m0: int) -> torch.Tensor:
    """K > 64.  K <= WIDE_HIP_MAX_K: ``mc_cov_wide_kernel`` draws each sim's normals block by
    block into LDS and accumulates Z^T Z on the fp64 matrix cores (time chunks a function of T
    only, summed in order).  Wider: Philox normals Z [sims, T, K] (same stream keys) and
    cov = (Z^T Z - s s^T / T) / (T - 1) as one batched rocBLAS GEMM per chunk of sims.  Each
    sim's covariance depends on that sim only, so any partition of the sims gives the same
    matrices."""
    if K <= WIDE_HIP_MAX_K:
        Cz = torch.empty(M, K, K, dtype=torch.float64, device=dev)
        ws = torch.empty(max(1, _native.query("mfa_mc_cov_wide_ws_doubles", M, K, T)),
                         dtype=torch.float64, device=dev)
        _native.call("mfa_mc_cov_wide", M, int(m0), K, T, int(seed) & 0xFFFFFFFFFFFFFFFF,
                     _native.ptr(ws), _native.ptr(Cz), _native.stream(dev))
        return Cz
    if _wide_solver == "hip" and K <= XL_MAX_K:
        # output-tiled MFMA kernel (mc_cov_xl_kernel), sims chunked to bound the partials
        Cz = torch.empty(M, K, K, dtype=torch.float64, device=dev)
        per = max(1, _native.query("mfa_mc_cov_xl_ws_doubles", 1, K, T))
        step = max(1, WIDE_CHUNK_DOUBLES // per)
        ws = torch.empty(per * min(step, M), dtype=torch.float64, device=dev)
        for a in range(0, M, step):
            mc = min(step, M - a)
            Cc = Cz[a:a + mc]
            _native.call("mfa_mc_cov_xl", mc, int(m0 + a), K, T, int(seed) & 0xFFFFFFFFFFFFFFFF,
                         _native.ptr(ws), _native.ptr(Cc), _native.stream(dev))
        return Cz
    Kp = K + (K & 1)
    Cz = torch.empty(M, K, K, dtype=torch.float64, device=dev)
    step = max(1, WIDE_CHUNK_DOUBLES // (T * Kp))
    for a in range(0, M, step):
        mc = min(step, M - a)
        Z = torch.empty(mc, T, Kp, dtype=torch.float64, device=dev)
        _native.call("mfa_philox_normals", mc, int(m0 + a), K, T, int(seed) & 0xFFFFFFFFFFFFFFFF,
                     _native.ptr(Z), _native.stream(dev))
        Zk = Z[:, :, :K]
        cs = Zk.sum(1)
        G = torch.bmm(Zk.transpose(1, 2), Zk)
        Cz[a:a + mc] = (G - cs[:, :, None] * cs[:, None, :] / T) / (T - 1)
    return Cz


def _bias_sum_wide(w, valid, Cz):
    """K > 64 on the device: S[d, k] = sum_m v_m[d, k] with v_m = diag(V^T D0 V) / lambda of
    A = sqrt(D0) C_z sqrt(D0) (the identity of SURVEY.md §2.3.4), eigen-decomposed by rocSOLVER
    in chunks of (dates x sims), or by the multi-wave HIP solver (``set_wide_bias_solver``);
    invalid dates give NaN."""
    D, K = w.shape
    M = Cz.shape[0]
    dev = w.device
    if _wide_solver == "hip" and K <= WIDE_HIP_MAX_K:
        return _bias_sum_wide_hip(w, valid, Cz)
    if _wide_solver == "hip" and K <= XL_MAX_K:
        return _bias_sum_xl(w, valid, Cz)
    S = torch.zeros(D, K, dtype=torch.float64, device=dev)
    dd = torch.nonzero(valid).flatten()
    sq = torch.sqrt(w.clamp_min(0.0))
    nm = max(1, min(M, WIDE_CHUNK_DOUBLES // (K * K)))
    nd = max(1, WIDE_CHUNK_DOUBLES // (nm * K * K))
    for a in range(0, dd.numel(), nd):
        ds = dd[a:a + nd]
        s = sq[ds]                                                     # [nd, K]
        acc = torch.zeros(ds.numel(), K, dtype=torch.float64, device=dev)
        for b in range(0, M, nm):
            cz = Cz[b:b + nm]
            A = s[:, None, :, None] * cz[None] * s[:, None, None, :]   # [nd, nm, K, K]
            lam, V = torch.linalg.eigh(A.reshape(-1, K, K))
            lam, V = lam.flip(-1), V.flip(-1)
            wv = w[ds][:, None, :, None].expand(-1, cz.shape[0], -1, -1).reshape(-1, K, 1)
            v = ((V * V) * wv).sum(1) / lam                            # [nd * nm, K]
            acc += v.view(ds.numel(), cz.shape[0], K).sum(1)
        S[ds] = acc
    S[~valid] = float("nan")
    return S


def _bias_sum_wide_hip(w, valid, Cz):
    """The multi-wave HIP solver over chunks of sims (per-(date, sim) values: D x chunk x K
    doubles at a time), each chunk summed into S in sim order."""
    D, K = w.shape
    M = Cz.shape[0]
    dev = w.device
    S = torch.zeros(D, K, dtype=torch.float64, device=dev)
    wc = w.contiguous()
    dv = valid.to(torch.int32).contiguous()
    mc = max(1, min(M, WIDE_CHUNK_DOUBLES // max(1, D * K)))
    ws = torch.empty(D * mc * K, dtype=torch.float64, device=dev)
    for a in range(0, M, mc):
        n = min(mc, M - a)
        cz = Cz[a:a + n].contiguous()
        _native.call("mfa_eigen_bias_accumulate_wide", _native.ptr(wc), _native.ptr(dv), D, K, n,
                     _native.ptr(cz), _native.ptr(ws), _native.ptr(S), _native.stream(dev))
    return S


def _bias_sum_xl(w, valid, Cz):
    """WIDE_HIP_MAX_K < K <= XL_MAX_K: the XL solver (``mfa_eigen_bias_accumulate_xl``) over
    chunks of sims, each chunk's per-(date, sim) values summed into S in sim order."""
    D, K = w.shape
    M = Cz.shape[0]
    dev = w.device
    S = torch.zeros(D, K, dtype=torch.float64, device=dev)
    wc = w.contiguous()
    dv = valid.to(torch.int32).contiguous()
    mc = max(1, min(M, WIDE_CHUNK_DOUBLES // max(1, D * K)))
    vws = torch.empty(D * mc * K, dtype=torch.float64, device=dev)
    ws = torch.empty(max(1, _native.query("mfa_eigen_xl_ws_doubles", D * mc, K)),
                     dtype=torch.float64, device=dev)
    for a in range(0, M, mc):
        n = min(mc, M - a)
        cz = Cz[a:a + n].contiguous()
        _native.call("mfa_eigen_bias_accumulate_xl", _native.ptr(wc), _native.ptr(dv), D, K, n,
                     _native.ptr(cz), _native.ptr(vws), _native.ptr(ws), _native.ptr(S),
                     _native.stream(dev))
    return S


def _finalize_wide(S, M, w, U, valid, scale_coef):
    """v = a (sqrt(S / M) - 1) + 1, F^ = U diag(v^2 w) U^T: eigen_finalize_kernel (any K)."""
    D, K = w.shape
    dev = w.device
    Fh = torch.empty(D, K, K, dtype=torch.float64, device=dev)
    vb = torch.empty(D, K, dtype=torch.float64, device=dev)
    # operands bound to names: a temporary inside ptr(...) is freed before the launch and its block
    # can be handed to the next temporary of the same call
    Sc, wc, Uc, vi = S.contiguous(), w.contiguous(), U.contiguous(), valid.to(torch.int32).contiguous()
    _native.call("mfa_eigen_finalize_sum", _native.ptr(Sc), int(M), _native.ptr(wc),
                 _native.ptr(Uc), _native.ptr(vi),
                 D, K, float(scale_coef), _native.ptr(Fh), _native.ptr(vb), _native.stream(dev))
    return Fh, vb


def sim_shard(M: int, rank: int, world: int) -> tuple[int, int]:
    """Contiguous block ``[m0, m1)`` of the M simulations owned by ``rank``."""
    base, rem = divmod(M, world)
    m0 = rank * base + min(rank, rem)
    return m0, m0 + base + (1 if rank < rem else 0)


@contextlib.contextmanager
def _date_origin(date0: int, dev):
    """Global index of date 0 of the bias launches inside the block (date-chained solver)."""
    if dev.type != "cuda" or not date0:
        yield
        return
    _native.call("mfa_eigen_set_date_origin", int(date0))
    try:
        yield
    finally:
        _native.call("mfa_eigen_set_date_origin", 0)


def eigen_risk_adjust_sharded(F0: torch.Tensor, *, M: int = 10_000, scale_coef: float = 1.4,
                              T_sim: int | None = None, seed: int = 1, chunk: int = 256,
                              ctx=None, psd_tol: float = 0.0, return_bias: bool = False,
                              date0: int = 0):
    """Monte-Carlo eigen adjustment with the simulations sharded over ranks and chunked in time.

    For large M (the 10k-bootstrap configuration) the per-(date, sim) bias values are never
    materialised: each rank draws only its block of simulations (:func:`sim_shard`), ``chunk``
    at a time, and accumulates ``S[d, k] = sum_m v_m[d, k]`` on the device; one
    ``all_reduce(SUM)`` of the [D, K] float64 sums over RCCL (collective C5 of SURVEY.md §2.5)
    then gives every rank the full-M mean.  ``F0`` must hold the SAME dates on every rank.
    Results equal :func:`eigen_risk_adjust` with the same M and seed up to summation order.
    ``date0``: global index of ``F0[0]`` (the date-chained bias solver aligns its chains to it).
    """
    from ..parallel import dist as pdist
    ctx = ctx or pdist.context()
    F0 = F0.to(torch.float64).contiguous()
    D, K, _ = F0.shape
    T_sim = D if T_sim is None else T_sim
    dev = F0.device
    w, U = eigh(F0, resolve_psd_tol=psd_tol)
    valid = torch.isfinite(w).all(-1) & (w.min(-1).values >= -psd_tol * w.abs().max(-1).values.clamp_min(0))
    w = torch.where(valid[:, None], w.clamp_min(0.0), w).contiguous()
    rank, world = (ctx.rank, ctx.world) if ctx.enabled else (0, 1)
    m0, m1 = sim_shard(M, rank, world)
    S = torch.zeros(D, K, dtype=torch.float64, device=dev)
    wide = dev.type == "cuda" and K > WIDE_K
    if wide:
        for a in range(m0, m1, chunk):
            mc = min(chunk, m1 - a)
            S += _bias_sum_wide(w, valid, mc_cov(mc, K, max(T_sim, 2), seed, dev, m0=a))
    elif dev.type == "cuda":
        dv = valid.to(torch.int32).contiguous()
        ws = torch.empty(D * min(chunk, max(1, m1 - m0)) * K, dtype=torch.float64, device=dev)
        for a in range(m0, m1, chunk):
            mc = min(chunk, m1 - a)
            Cz = mc_cov(mc, K, max(T_sim, 2), seed, dev, m0=a)
            with _date_origin(date0, dev):
                _native.call("mfa_eigen_bias_accumulate", _native.ptr(w), _native.ptr(dv), D, K,
                             mc, _native.ptr(Cz), MAX_SWEEPS, TOL, _native.ptr(ws),
                             _native.ptr(S), _native.stream(dev))
    else:
        for a in range(m0, m1, chunk):
            mc = min(chunk, m1 - a)
            Cz = mc_cov(mc, K, max(T_sim, 2), seed, dev, m0=a)
            S += _bias_sum_reference(w, valid, Cz)
    if ctx.enabled:
        pdist.all_reduce_sum(S, ctx)
    if wide:
        Fh, vb = _finalize_wide(S, M, w, U, valid, scale_coef)
    elif dev.type == "cuda":
        Fh = torch.empty(D, K, K, dtype=torch.float64, device=dev)
        vb = torch.empty(D, K, dtype=torch.float64, device=dev)
        Uc, vi = U.contiguous(), valid.to(torch.int32).contiguous()   # named: see _finalize_wide
        _native.call("mfa_eigen_finalize_sum", _native.ptr(S), int(M), _native.ptr(w),
                     _native.ptr(Uc), _native.ptr(vi),
                     D, K, float(scale_coef), _native.ptr(Fh), _native.ptr(vb), _native.stream(dev))
    else:
        v = scale_coef * (torch.sqrt(S / M) - 1.0) + 1.0
        vb = torch.where(valid[:, None], v, torch.full_like(v, float("nan")))
        Fh = (U * (vb * vb * w)[:, None, :]) @ U.transpose(-1, -2)
        Fh[~valid] = float("nan")
    return (Fh, vb) if return_bias else Fh


def _bias_sum_reference(w, valid, Cz):
    """sum_m v_m[d, k] over the draw covariances ``Cz`` (CPU oracle of the accumulate kernel)."""
    D, K = w.shape
    S = torch.zeros(D, K, dtype=torch.float64)
    for d in torch.nonzero(valid).flatten().tolist():
        s = torch.sqrt(w[d])
        lam, V = torch.linalg.eigh(s[None, :, None] * Cz * s[None, None, :])
        lam, V = lam.flip(-1), V.flip(-1)
        S[d] = (((V * V) * w[d][None, :, None]).sum(1) / lam).sum(0)
    S[~valid] = float("nan")
    return S


def eigen_risk_adjust(F0: torch.Tensor, *, M: int = 100, scale_coef: float = 1.4,
                      T_sim: int | None = None, seed: int = 1, Cz: torch.Tensor | None = None,
                      psd_tol: float = 0.0, return_bias: bool = False, date0: int = 0):
    """Eigenfactor risk adjustment of a batch of covariance matrices.

    ``F0`` [D, K, K] float64 (NaN matrices allowed -> NaN outputs).  ``T_sim`` defaults to D
    (the reference passes the total number of dates for every date, quirk Q9).  ``Cz`` may be
    supplied to share draw covariances between calls (and between CPU and GPU for testing).
    Returns ``F_hat`` [D, K, K] (and the bias multipliers ``v`` [D, K] if ``return_bias``).
    ``date0``: global index of ``F0[0]`` (a date shard's offset: the date-chained bias solver
    aligns its chains to global dates, so shards reproduce one process bit for bit).
    """
    F0 = F0.to(torch.float64).contiguous()
    D, K, _ = F0.shape
    T_sim = D if T_sim is None else T_sim
    dev = F0.device
    w, U = eigh(F0, resolve_psd_tol=psd_tol)
    valid = torch.isfinite(w).all(-1) & (w.min(-1).values >= -psd_tol * w.abs().max(-1).values.clamp_min(0))
    w = torch.where(valid[:, None], w.clamp_min(0.0), w)
    if Cz is None:
        Cz = mc_cov(M, K, max(T_sim, 2), seed, dev)
    Cz = Cz.to(device=dev, dtype=torch.float64).contiguous()
    M = Cz.shape[0]
    if dev.type != "cuda":
        return _eigen_adjust_reference(w, U, valid, Cz, scale_coef, return_bias)
    if K > WIDE_K:
        Fh, vb = _finalize_wide(_bias_sum_wide(w, valid, Cz), M, w, U, valid, scale_coef)
        return (Fh, vb) if return_bias else Fh
    Fh = torch.empty(D, K, K, dtype=torch.float64, device=dev)
    vb = torch.empty(D, K, dtype=torch.float64, device=dev)
    ws = torch.empty(D * M * K, dtype=torch.float64, device=dev)
    dv = valid.to(torch.int32).contiguous()
    with _date_origin(date0, dev):
        wc, Uc = w.contiguous(), U.contiguous()   # named: see _finalize_wide
        _native.call("mfa_eigen_adjust", _native.ptr(wc), _native.ptr(Uc),
                     _native.ptr(dv), D, K, M, _native.ptr(Cz), float(scale_coef), MAX_SWEEPS, TOL,
                     _native.ptr(ws), _native.ptr(Fh), _native.ptr(vb), _native.stream(dev))
    return (Fh, vb) if return_bias else Fh


def _eigen_adjust_reference(w, U, valid, Cz, scale_coef, return_bias):
    D, K = w.shape
    M = Cz.shape[0]
    Fh = torch.full((D, K, K), float("nan"), dtype=torch.float64)
    vb = torch.full((D, K), float("nan"), dtype=torch.float64)
    for d in torch.nonzero(valid).flatten().tolist():
        s = torch.sqrt(w[d])
        Cb = s[None, :, None] * Cz * s[None, None, :]          # [M, K, K]
        lam, V = torch.linalg.eigh(Cb)
        lam, V = lam.flip(-1), V.flip(-1)                       # descending
        vm = ((V * V) * w[d][None, :, None]).sum(1) / lam       # [M, K]
        v = torch.sqrt(vm.mean(0))
        v = scale_coef * (v - 1.0) + 1.0
        vb[d] = v
        Fh[d] = (U[d] * (v * v * w[d])) @ U[d].T
    return (Fh, vb) if return_bias else Fh
