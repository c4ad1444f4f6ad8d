"""Legacy ``factor.py`` compatibility (reference: ``/factor.py``, the CSV-era twin of
``Barra_factor_cal/factor_calculator.py`` + ``post_processing.py``).

Behavioural differences from :mod:`barra_factor_cal.factor_calculator` that this module keeps
(SURVEY.md §2.1 row 12, §2.2):

* CMRA over PARTIAL windows from a stock's first day (``factor.py:217``, quirk Q15);
* CETOP from a precomputed ``n_cashflow_act_ttm`` column (``factor.py:358-399``) instead of the
  statement-row TTM built from ``n_cashflow_act``;
* ``run`` returns ``[ts_code, trade_date, <descriptors>]`` only (``factor.py:505-530``: the
  ``reduce`` merge on ``original_index``), so ``ret`` / ``circ_mv`` are merged back AFTER
  post-processing in :func:`main` and are therefore NOT winsorized (contrast quirk Q23);
* :func:`main` is the script's ``__main__`` (``factor.py:604-733``): CSV in, ``ret`` shifted to
  t+1 per stock, INNER merge with the SW industry table, Barra renames, and
  ``result/barra_factors_1014.csv`` + ``result/industry_info_1014.csv`` out.

Descriptor kernels are the same batched HIP launches as the current calculator.
"""
from __future__ import annotations

import os
from dataclasses import replace

import numpy as np
import pandas as pd
import torch

from llm_driven_multi_factor_model_amd.models.factor_engine import (BARRA_OUTPUT_COLUMNS,
                                                                    BARRA_RENAME, FACTORS_TO_RUN,
                                                                    FactorEngine)
from llm_driven_multi_factor_model_amd.utils.config import FactorConfig

from .post_processing import (calculate_composite_factors, orthogonalize_factors,  # noqa: F401
                              winsorize_factors)

LEGACY_CONFIG = replace(FactorConfig(), cmra_partial=True)


class _LegacyEngine(FactorEngine):
    NUMERIC = FactorEngine.NUMERIC + ["n_cashflow_act_ttm"]

    def compute_earnings_yield(self):
        if not self._need("n_cashflow_act_ttm", "total_mv", "pe_ttm"):
            return None
        cf = self.cols["n_cashflow_act_ttm"].double()
        mv = self.cols["total_mv"].double()
        nan = torch.full_like(mv, float("nan"))
        cetop = torch.where((mv > 0) & (cf > 0), cf / mv, nan)
        pe = self.cols["pe_ttm"].double()
        etop = torch.where(pe > 0, 1.0 / pe, nan)
        return {"CETOP": cetop.float(), "ETOP": etop.float()}


class FactorCalculator:
    """``factor.py``'s ``FactorCalculator`` (string dates ``YYYY/MM/DD`` after preparation)."""

    def __init__(self, prices_df: pd.DataFrame, index_df: pd.DataFrame, device=None):
        print("Initializing Factor Calculator...")
        self._engine = _LegacyEngine(prices_df, index_df, device=device, config=LEGACY_CONFIG)
        self.master_df = self._engine.master
        m = self.master_df
        # prices_df as the legacy _prepare_data leaves it: sorted, string dates, ret / log_ret
        self.prices_df = m.drop(columns=["original_index", "market_ret"]).copy()
        self.prices_df["ret"] = self._engine.cols["ret"].double().cpu().numpy()
        self.prices_df["log_ret"] = self._engine.cols["log_ret"].double().cpu().numpy()
        self.index_df = index_df

    def __getattr__(self, name):
        if name.startswith("compute_") or name == "select_growth_factors":
            meth = getattr(self._engine, name)

            def call():
                res = meth()
                if res is None:
                    return None
                df = pd.DataFrame({"original_index": self.master_df["original_index"].values})
                for k, v in res.items():
                    df[k] = v.double().cpu().numpy()
                return df
            return call
        raise AttributeError(name)

    def run(self, factors: list) -> pd.DataFrame:
        res = self._engine.compute(factors)
        df = self.master_df[["ts_code", "trade_date"]].copy()
        for k, v in res.items():
            df[k] = v.double().cpu().numpy()
        print("Factor calculation complete.")
        return df


def main(stk_path: str, index_path: str, sw_industry_path: str, out_dir: str = "result",
         device=None, factors: list | None = None):
    """``factor.py __main__``: raw CSVs -> Barra table and industry info (legacy file names)."""
    from barra_factor_cal import config

    stk = pd.read_csv(stk_path)
    idx = pd.read_csv(index_path)
    calc = FactorCalculator(stk, idx, device=device)
    raw = calc.run(factors or list(FACTORS_TO_RUN))
    cols = [c for c in raw.columns if c not in ("ts_code", "trade_date")]
    win = winsorize_factors(raw, cols)
    comp = calculate_composite_factors(win, config.COMPOSITE_CONFIG)
    proc = orthogonalize_factors(comp, config.ORTHO_RULES)
    price = calc.prices_df[["ts_code", "trade_date", "ret", "circ_mv"]]
    fac = proc.merge(price, on=["ts_code", "trade_date"], how="left")
    fac["ret"] = fac.groupby("ts_code")["ret"].shift(-1)
    sw = pd.read_csv(sw_industry_path)
    fac = fac.merge(sw[["ts_code", "l1_code"]], on="ts_code")          # inner merge (legacy)
    fac = fac.rename(columns=dict(BARRA_RENAME))
    barra = fac[list(BARRA_OUTPUT_COLUMNS)]
    os.makedirs(out_dir, exist_ok=True)
    barra.to_csv(os.path.join(out_dir, "barra_factors_1014.csv"), index=False)
    info = price[["ts_code"]].drop_duplicates().merge(
        sw[["ts_code", "l1_code", "l1_name", "in_date"]], on="ts_code", how="left")
    info = info.drop_duplicates(subset=["l1_code", "l1_name"]).reset_index(drop=True)
    info = info.rename(columns={"l1_code": "code", "l1_name": "industry_names", "in_date": "start_date"})
    info = info[["code", "industry_names", "start_date"]]
    info.to_csv(os.path.join(out_dir, "industry_info_1014.csv"), index=False)
    return barra, info


if __name__ == "__main__":
    from barra_factor_cal import config as _cfg
    main(_cfg.STK_DATA_PATH, _cfg.INDEX_DATA_PATH, _cfg.INDUSTRY_DATA_PATH, _cfg.RESULT_DIR)
