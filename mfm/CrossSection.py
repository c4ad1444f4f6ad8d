"""``mfm.CrossSection`` compatibility API (reference: Barra-master/mfm/CrossSection.py).

``style_factor_norm`` (:12-20) and ``CrossSection(...).reg()`` (:35-108) with the reference's
attributes and return types; the solve runs in the MI355X engine (one-date batch of the fused
CS-WLS kernels on the GPU, float64 reference path on the CPU).

``solver="pinv"`` (default) is the current reference (``CrossSection.py:76,98``);
``solver="inv"`` reproduces the stale copies / installed build (``build/lib/mfm/CrossSection.py``,
quirk Q4): an exactly singular normal matrix (e.g. an empty industry) raises
``numpy.linalg.LinAlgError: Singular matrix`` as in ``try_1024.ipynb#c3``.
"""
from __future__ import annotations

import numpy as np
import pandas as pd
import torch

from llm_driven_multi_factor_model_amd.ops import cross_section as _xs
from llm_driven_multi_factor_model_amd.ops.xs_reduce import style_norm as _style_norm

from ._device import device as _device, verbose as _verbose


def style_factor_norm(factors, capital):
    """Cap-weighted mean, ONE pooled ddof-0 std over all entries (CrossSection.py:12-20)."""
    f = np.asarray(factors, dtype=np.float64)
    c = np.asarray(capital, dtype=np.float64)
    w_mu = (f * c[:, None]).sum(0) / c.sum()
    return (f - w_mu) / np.std(f)


def check_inv_solvable(status, ind=None, valid=None, P: int = 0) -> None:
    """``np.linalg.inv`` semantics (quirk Q4): a date whose normal matrix is exactly singular
    raises LinAlgError -- an industry with no stock on the date (zero row / column of the
    reference's dense Gram) or an exactly rank-deficient style block."""
    st = torch.as_tensor(status).cpu()
    if bool(((st & (_xs.XS_ZERO_PIVOT | _xs.XS_PIVOT_EMPTY)) != 0).any()):
        raise np.linalg.LinAlgError("Singular matrix")
    if ind is not None and P > 0:
        ind = torch.as_tensor(ind).cpu().long()
        ok = torch.as_tensor(valid).cpu() if valid is not None else torch.ones_like(ind, dtype=torch.bool)
        ok = ok & (ind >= 0) & (ind < P)
        D = ind.shape[0]
        cnt = torch.zeros(D, P, dtype=torch.int64)
        cnt.scatter_add_(1, torch.where(ok, ind, 0), ok.long())
        if bool((cnt == 0).any()):
            raise np.linalg.LinAlgError("Singular matrix")


class CrossSection:
    """One cross-sectional regression (base_data columns: date, stocknames, capital, ret)."""

    def __init__(self, base_data: pd.DataFrame, style_factors: pd.DataFrame = pd.DataFrame(),
                 industry_factors: pd.DataFrame = pd.DataFrame(), pivot_mode: int = 0,
                 solver: str = "pinv"):
        if solver not in ("pinv", "inv"):
            raise ValueError("solver must be 'pinv' or 'inv'")
        self._solver = solver
        self.date = list(base_data.date)[0]
        self.stocknames = list(base_data.stocknames)
        self.capital = base_data.capital.values
        self.ret = base_data.ret.values
        self.style_factors_names = list(style_factors.columns)
        self.industry_factors_names = list(industry_factors.columns)
        self.N = base_data.shape[0]
        self.Q = style_factors.shape[1]
        self.P = industry_factors.shape[1]
        self._raw_styles = np.asarray(style_factors.values, dtype=np.float64)
        self.style_factors = style_factor_norm(self._raw_styles, self.capital)
        self.industry_factors = industry_factors.values
        self.country_factors = np.array(self.N * [[1]])
        sq = np.sqrt(self.capital)
        self.W = sq / sq.sum()
        self._pivot_mode = pivot_mode  # 1 = reference (last industry), 0 = last non-empty
        if _verbose():
            print(f"\rCross Section Regression, Date: {self.date}, {self.N} Stocks, {self.P} Industry "
                  f"Facotrs, {self.Q} Style Facotrs", end="")

    def _tensors(self, dev):
        if self.Q < 1:
            raise ValueError("at least one style factor is required")
        # float64 storage: the reference regresses its float64 inputs as they are
        X = torch.from_numpy(np.ascontiguousarray(self._raw_styles.T))[None].to(dev)
        cap = torch.from_numpy(np.asarray(self.capital, dtype=np.float64))[None].to(dev)
        ret = torch.from_numpy(np.asarray(self.ret, dtype=np.float64))[None].to(dev)
        ind = None
        if self.P > 0:
            oh = np.asarray(self.industry_factors)
            ids = np.where(oh.sum(1) > 0, oh.argmax(1), -1).astype(np.int16)
            ind = torch.from_numpy(ids)[None].to(dev)
        return X, cap, ret, ind

    def reg(self):
        """-> (factor_ret [K], specific_ret [N], pure_factor_portfolio_exposure np.matrix [K,K], R2)."""
        dev = _device()
        X, cap, ret, ind = self._tensors(dev)
        res = _xs.xs_wls(X, cap, ret, ind, self.P, pivot_mode=self._pivot_mode)
        if self._solver == "inv":
            check_inv_solvable(res.status[:1], ind, None, self.P)
        f = res.f[0].cpu().numpy()
        e = res.resid[0].double().cpu().numpy()
        # specific returns in float64 exactly as the reference: r - X f
        Xf = np.hstack([self.country_factors, self.industry_factors, self.style_factors]) if self.P > 0 \
            else np.hstack([self.country_factors, self.style_factors])
        e = self.ret - Xf @ f
        r2 = 1 - np.var(e) / np.var(self.ret)
        mu = res.stats[0, :self.Q]
        sig = float(res.stats[0, self.Q])
        pivot = None
        if self.P > 0 and self._pivot_mode == 0:  # last non-empty industry, as the solver
            present = np.nonzero(np.asarray(self.industry_factors).sum(0) > 0)[0]
            pivot = int(present[-1]) if present.size else self.P - 1
        _, expo = _xs.pure_factor_portfolio(X[0].cpu().double(), cap[0].cpu().double(),
                                            ind[0].cpu() if ind is not None else None, self.P,
                                            mu.cpu(), sig, pivot=pivot)
        return f, e, np.matrix(expo.numpy()), r2
