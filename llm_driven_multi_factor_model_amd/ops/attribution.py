"""Portfolio risk attribution on the Barra factor model (BASELINE.json config 5).

The reference stops at the factor covariance series (``Barra-master/mfm/MFM.py:80-167``) and a
never-called specific-vol shrinkage (``mfm/utils.py:153-168``); a user of the risk model then
decomposes a portfolio's risk.  For holdings ``h`` on date d:

* factor exposures ``x = X_d^T h`` with the regression's design matrix ``X_d`` =
  [country | one-hot industries | cap-weighted z-scored styles] (``CrossSection.py:12-20,48,74``)
  — the HIP kernel ``csrc/attribution.hip`` reads the raw panel once per date;
* factor variance ``x^T F x``, specific variance ``sum_i h_i^2 s_i^2``;
* marginal contribution to risk ``MCTR = F x / sigma_p`` and contributions ``x * MCTR`` (they sum
  to the factor part of ``sigma_p``); percentages of total variance.
"""
from __future__ import annotations

import ctypes as C
from dataclasses import dataclass

import torch

from .. import _native
from .cross_section import valid_mask

_native.register("mfa_portfolio_exposure", [C.c_void_p, C.c_void_p, C.c_void_p, C.c_void_p,
                                             C.c_void_p, C.c_void_p, C.c_int, C.c_int, C.c_int,
                                             C.c_int, C.c_void_p, C.c_void_p])
_native.register("mfa_portfolio_exposure_f64", [C.c_void_p] * 6 + [C.c_int] * 4 +
                 [C.c_void_p, C.c_void_p])


_native.register("mfa_trailing_vol", [C.c_void_p, C.c_int, C.c_void_p, C.c_int, C.c_int, C.c_int,
                                       C.c_int, C.c_void_p, C.c_void_p])


def trailing_vol(halo: torch.Tensor, e: torch.Tensor, window: int, min_periods: int = 1) -> torch.Tensor:
    """[D, N] point-in-time trailing ddof-0 std over the ``window`` rows ending at each date of
    ``cat([halo, e])`` (``halo`` = the window - 1 preceding rows, NaN where none), finite values
    only; NaN below ``min_periods`` values.  GPU: one HIP kernel, bitwise equal to the
    newest-first loop of :meth:`RiskModel.specific_vol_series` (its CPU path)."""
    D, N = e.shape
    h = window - 1
    if halo.shape != (h, N):
        raise ValueError(f"halo must be [{h}, {N}], got {tuple(halo.shape)}")
    e = _native.check_device_tensor(e, torch.float64, "e")
    halo = halo.to(torch.float64).contiguous()
    vol = torch.empty(D, N, dtype=torch.float64, device=e.device)
    _native.call("mfa_trailing_vol", _native.ptr(halo) if h > 0 else None, h, _native.ptr(e), D, N,
                 window, min_periods, _native.ptr(vol), _native.stream(e.device))
    return vol


def portfolio_exposure(X: torch.Tensor, cap: torch.Tensor, ret: torch.Tensor,
                       ind: torch.Tensor | None, h: torch.Tensor, stats: torch.Tensor,
                       P: int) -> torch.Tensor:
    """Factor exposures ``[D, 1+P+Q]`` of portfolios ``h`` [D, N] on every date.

    ``stats`` is :attr:`XsResult.stats` of the same panel (cap-weighted style means, pooled
    sigma, n).  Absent / invalid stocks carry no exposure.
    """
    D, Q, N = X.shape
    K = 1 + P + Q
    h = h.to(torch.float64)
    if h.shape != (D, N):
        raise ValueError(f"h must be [D, N] = {(D, N)}, got {tuple(h.shape)}")
    if not X.is_cuda:
        return _portfolio_exposure_reference(X, cap, ret, ind, h, stats, P)
    dt = X.dtype if X.dtype == torch.float64 else torch.float32
    X = _native.check_device_tensor(X, dt, "X")
    cap = _native.check_device_tensor(cap, dt, "cap")
    ret = _native.check_device_tensor(ret, dt, "ret")
    if P > 0:
        ind = _native.check_device_tensor(ind, torch.int16, "ind")
    h = h.contiguous()
    stats = stats.to(torch.float64).contiguous()
    out = torch.empty(D, K, dtype=torch.float64, device=X.device)
    _native.call("mfa_portfolio_exposure_f64" if dt == torch.float64 else "mfa_portfolio_exposure",
                 _native.ptr(X), _native.ptr(cap), _native.ptr(ret),
                 _native.ptr(ind if P > 0 else None), _native.ptr(h), _native.ptr(stats), D, N, P,
                 Q, _native.ptr(out), _native.stream(X.device))
    return out


def _portfolio_exposure_reference(X, cap, ret, ind, h, stats, P):
    """Dense float64 oracle: builds X_d explicitly and computes X_d^T h."""
    D, Q, N = X.shape
    m = valid_mask(X, cap, ret, ind, P) & torch.isfinite(h)
    hm = torch.where(m, h, torch.zeros((), dtype=torch.float64))
    mu, sig = stats[:, :Q].double(), stats[:, Q].double()
    Z = (X.double() - mu[:, :, None]) / sig[:, None, None]
    Z = torch.where(m[:, None, :], Z, torch.zeros((), dtype=torch.float64))
    cols = [hm.sum(1, keepdim=True)]
    if P > 0:
        oh = torch.nn.functional.one_hot(ind.long().clamp(0, P - 1), P).double() * m[..., None]
        cols.append(torch.einsum("dnp,dn->dp", oh, hm))
    cols.append(torch.einsum("dqn,dn->dq", Z, hm))
    return torch.cat(cols, 1)


@dataclass
class RiskAttribution:
    """Per-date decomposition (all float64, leading dim D).

    total_var = factor_var + specific_var; mctr / contrib are in volatility units (contrib sums
    over factors to factor_var / sigma_p); pct_var = x_k (F x)_k / total_var.
    """
    exposure: torch.Tensor      # [D, K]
    factor_var: torch.Tensor    # [D]
    specific_var: torch.Tensor  # [D]
    total_var: torch.Tensor     # [D]
    mctr: torch.Tensor          # [D, K]
    contrib: torch.Tensor       # [D, K]
    pct_var: torch.Tensor       # [D, K]

    @property
    def total_vol(self) -> torch.Tensor:
        return torch.sqrt(self.total_var)

    def grouped(self, P: int) -> dict:
        """Share of total variance by factor group: country / industry / style / specific."""
        pv = self.pct_var
        return {"country": pv[:, 0], "industry": pv[:, 1:1 + P].sum(1),
                "style": pv[:, 1 + P:].sum(1), "specific": self.specific_var / self.total_var}


def risk_attribution(x: torch.Tensor, F: torch.Tensor,
                     specific_var: torch.Tensor | None = None) -> RiskAttribution:
    """Decompose portfolio risk given exposures ``x`` [D, K], factor covariances ``F`` [D, K, K]
    and (optionally) the portfolio's specific variance [D] (``sum_i h_i^2 s_i^2``)."""
    x = x.to(torch.float64)
    F = F.to(torch.float64)
    Fx = torch.einsum("dkl,dl->dk", F, x)
    fvar = (x * Fx).sum(1)
    svar = torch.zeros_like(fvar) if specific_var is None else specific_var.to(fvar)
    tvar = fvar + svar
    sig = torch.sqrt(tvar)
    mctr = Fx / sig[:, None]
    return RiskAttribution(exposure=x, factor_var=fvar, specific_var=svar, total_var=tvar,
                           mctr=mctr, contrib=x * mctr, pct_var=x * Fx / tvar[:, None])


def portfolio_specific_var(h: torch.Tensor, spec_vol: torch.Tensor) -> torch.Tensor:
    """``sum_i h_i^2 s_i^2`` per date; ``spec_vol`` [N] or [D, N] (NaN stocks contribute 0)."""
    h = h.to(torch.float64)
    s2 = spec_vol.to(torch.float64) ** 2
    v = h * h * (s2 if s2.dim() == 2 else s2[None, :])
    return torch.nan_to_num(v, nan=0.0).sum(-1)
