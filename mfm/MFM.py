"""``mfm.MFM`` compatibility API (reference: Barra-master/mfm/MFM.py:17-167).

Same constructor ``MFM(data, P, Q)`` (positional column contract, quirk Q13), attributes and
stage methods with the reference's return types and ordering exceptions.  Each stage is ONE
batched device call over all dates (the reference loops dates in Python); pandas objects are
built from the device results at the end of each stage.
"""
from __future__ import annotations

from collections.abc import MutableSequence

import numpy as np
import pandas as pd
import torch

from llm_driven_multi_factor_model_amd.models.risk_model import RiskModel
from llm_driven_multi_factor_model_amd.utils.config import RiskConfig
from llm_driven_multi_factor_model_amd.utils.io import panel_from_frame

from ._device import device as _device, verbose as _verbose


class LazyFrames(MutableSequence):
    """A list of per-date pandas objects built on first access.

    ``MFM``'s stages return Python lists of thousands of small DataFrames (MFM.py:66, :92-98,
    :117-123, :156-166); materialising them costs more than the batched GPU stage itself.  This
    sequence holds a builder and the dense device results instead, creates item t when it is
    first read and caches it.  It behaves as a list: len, index, negative index, slice,
    iteration, append / insert / del, ``pd.concat`` and ``==`` with a list.
    """

    def __init__(self, n: int, builder):
        self._build = builder
        self._items: list = [None] * n

    def _all(self):
        for j in range(len(self._items)):
            self[j]

    def __len__(self) -> int:
        return len(self._items)

    def __getitem__(self, i):
        if isinstance(i, slice):
            return [self[j] for j in range(*i.indices(len(self)))]
        if i < 0:
            i += len(self)
        if not 0 <= i < len(self):
            raise IndexError("list index out of range")
        if self._items[i] is None:
            self._items[i] = self._build(i)
        return self._items[i]

    def __setitem__(self, i, value):
        if isinstance(i, slice):
            self._all()  # materialise before a structural replace
        self._items[i] = value

    def __delitem__(self, i):
        self._all()
        del self._items[i]

    def insert(self, i, value):
        self._all()
        self._items.insert(i, value)

    def __eq__(self, other):
        return list(self) == list(other)

    def __repr__(self) -> str:
        done = sum(x is not None for x in self._items)
        return f"{type(self).__name__}({len(self)} items, {done} materialised)"


class SpecificReturns(LazyFrames):
    """``reg_by_time``'s per-date ``DataFrame[1, N_t]`` list; :meth:`dense` gives [T, N] directly."""

    def __init__(self, E: np.ndarray, valid: np.ndarray, stocks: np.ndarray, dates):
        self._E, self._valid, self._stocks, self._dates = E, valid, stocks, dates
        super().__init__(len(E), self._frame)

    def _frame(self, t: int) -> pd.DataFrame:
        v = self._valid[t]
        return pd.DataFrame([self._E[t][v].astype(np.float64)], columns=list(self._stocks[v]),
                            index=[self._dates[t]])

    def dense(self) -> pd.DataFrame:
        """[T, N] specific returns (NaN where a stock is absent) without per-date frames."""
        E = np.where(self._valid, self._E, np.nan).astype(np.float64)
        return pd.DataFrame(E, index=self._dates, columns=list(self._stocks))


class MFM:
    def __init__(self, data: pd.DataFrame, P: int, Q: int, pivot_mode: int = 0,
                 solver: str = "pinv", config: RiskConfig | None = None):
        """``solver="inv"`` reproduces the stale ``inv`` build (quirk Q4): reg_by_time raises
        LinAlgError at an exactly singular date.  ``config`` overrides the stage defaults."""
        if solver not in ("pinv", "inv"):
            raise ValueError("solver must be 'pinv' or 'inv'")
        self._solver = solver
        self.Q = Q
        self.P = P
        self.dates = pd.to_datetime(data.date.values)
        self.sorted_dates = pd.to_datetime(np.sort(pd.unique(self.dates)))
        self.T = len(self.sorted_dates)
        self.data = data
        self.columns = ["country"]
        self.columns.extend(list(data.columns[4:]))
        self.last_capital = None
        self.factor_ret = None
        self.specific_ret = None
        self.R2 = None
        self.Newey_West_cov = None
        self.eigen_risk_adj_cov = None
        self.vol_regime_adj_cov = None
        self._panel = panel_from_frame(data, P, Q, device=_device())
        cfg = config if config is not None else RiskConfig(pivot_mode=pivot_mode)
        self._model = RiskModel(self._panel, cfg)

    def _banner(self, title):
        if _verbose():
            print(f"\n\n{'=' * 35}{title}{'=' * 35}")

    def reg_by_time(self):
        self._banner("逐时间点进行横截面多因子回归")
        m = self._model
        f, e, r2 = m.regress()
        if self._solver == "inv":
            from .CrossSection import check_inv_solvable
            check_inv_solvable(m.status, m.panel.ind, m.panel.valid(), self.P)
        fr = f.cpu().numpy()
        self.factor_ret = pd.DataFrame(fr, columns=self.columns, index=self.sorted_dates)
        self.R2 = pd.DataFrame(r2.cpu().numpy(), columns=["R2"], index=self.sorted_dates)
        E = e.cpu().numpy()
        valid = m.panel.valid().cpu().numpy()
        stocks = np.asarray(m.panel.stocks)
        self.specific_ret = SpecificReturns(E, valid, stocks, self.sorted_dates)
        last = valid[-1]
        self.last_capital = m.panel.cap[-1].cpu().numpy()[last].astype(np.float64)
        return self.factor_ret, self.specific_ret, self.R2

    def _cov_list(self, V: torch.Tensor) -> LazyFrames:
        Vn = V.cpu().numpy()
        bad = np.isnan(Vn).any(axis=(1, 2))
        cols = self.columns
        return LazyFrames(Vn.shape[0], lambda t: pd.DataFrame() if bad[t] else
                          pd.DataFrame(Vn[t], columns=cols, index=cols))

    def Newey_West_by_time(self, q=2, tao=252):
        if self.factor_ret is None:
            raise Exception("please run reg_by_time to get factor returns first")
        self._banner("逐时间点进行Newey West调整")
        V = self._model.newey_west(q, tao)
        self.Newey_West_cov = self._cov_list(V)
        return self.Newey_West_cov

    def eigen_risk_adj_by_time(self, M=100, scale_coef=1.4):
        if self.Newey_West_cov is None:
            raise Exception("please run Newey_West_by_time to get factor return covariances after "
                            "Newey West adjustment first")
        self._banner("逐时间点进行Eigenfactor Risk调整")
        V = self._model.eigen_adjust(M=M, scale_coef=scale_coef, T_sim=self.T)
        self.eigen_risk_adj_cov = self._cov_list(V)
        return self.eigen_risk_adj_cov

    def vol_regime_adj_by_time(self, tao=84):
        if self.eigen_risk_adj_cov is None:
            raise Exception("please run eigen_risk_adj_by_time to get factor return covariances after "
                            "eigenfactor risk adjustment first")
        self._banner("逐时间点进行Volatility Regime调整")
        V, lam = self._model.vol_regime_adjust(tao)
        lam_h = [float(x) for x in lam.cpu().numpy()]
        er_list = self.eigen_risk_adj_cov

        def vra(t):
            er = er_list[t]
            return er * lam_h[t] ** 2 if not er.empty else er

        out = LazyFrames(self.T, vra)
        self.vol_regime_adj_cov = out
        return out, lam_h
