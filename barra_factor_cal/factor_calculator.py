"""``FactorCalculator`` compatibility API (reference: Barra_factor_cal/factor_calculator.py).

Each ``compute_*`` returns a DataFrame keyed by ``original_index`` like the reference; ``run``
returns ``[ts_code, trade_date, ret, circ_mv, <descriptors>]``.  All windows run as single
batched kernel launches (``FactorEngine``); names are case-insensitive.
"""
from __future__ import annotations

import pandas as pd

from llm_driven_multi_factor_model_amd.models.factor_engine import FactorEngine


class FactorCalculator:
    def __init__(self, prices_df: pd.DataFrame, index_df: pd.DataFrame, device=None):
        print("Initializing Factor Calculator...")
        self.prices_df = prices_df
        self.index_df = index_df
        self._engine = FactorEngine(prices_df, index_df, device=device)
        self.master_df = self._engine.master

    def _frame(self, res):
        if res is None:
            return None
        df = pd.DataFrame({"original_index": self.master_df["original_index"].values})
        for k, v in res.items():
            df[k] = v.double().cpu().numpy()
        return df

    def compute_size(self):
        return self._frame(self._engine.compute_size())

    def compute_beta_hsigma(self):
        return self._frame(self._engine.compute_beta_hsigma())

    def compute_rstr(self):
        return self._frame(self._engine.compute_rstr())

    def compute_dastd(self):
        return self._frame(self._engine.compute_dastd())

    def compute_cmra(self):
        return self._frame(self._engine.compute_cmra())

    def compute_nlsize(self):
        return self._frame(self._engine.compute_nlsize())

    def compute_bp(self):
        return self._frame(self._engine.compute_bp())

    def compute_liquidity(self):
        return self._frame(self._engine.compute_liquidity())

    def compute_earnings_yield(self):
        return self._frame(self._engine.compute_earnings_yield())

    def select_growth_factors(self):
        return self._frame(self._engine.select_growth_factors())

    def compute_leverage(self):
        return self._frame(self._engine.compute_leverage())

    def run(self, factors: list) -> pd.DataFrame:
        print(f"\nStarting factor calculation for: {factors}")
        out = self._engine.run(factors)
        print("Factor calculation complete.")
        return out
