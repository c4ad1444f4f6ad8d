"""post_processing.py compatibility API (winsorize / composite / orthogonalize per trade_date)."""
from __future__ import annotations

import pandas as pd

from llm_driven_multi_factor_model_amd.models import factor_engine as _fe


def winsorize_factors(factor_df: pd.DataFrame, factor_list: list, n_std: float = 2.5) -> pd.DataFrame:
    print(f"\n--- Starting Factor Winsorization (Boundary: Mean ± {n_std} * StdDev) ---")
    out = _fe.winsorize_frame(factor_df, factor_list, n_std)
    print("--- Factor Winsorization Complete ---")
    return out


def calculate_composite_factors(factor_df: pd.DataFrame, composite_factor_config: dict) -> pd.DataFrame:
    out = _fe.composite_frame(factor_df, composite_factor_config)
    print("\n--- Composite Factor Calculation Complete ---")
    return out


def orthogonalize_factors(factor_df: pd.DataFrame, ortho_config: dict) -> pd.DataFrame:
    print("\n--- Starting Factor Orthogonalization ---")
    out = _fe.orthogonalize_frame(factor_df, ortho_config)
    print("--- Factor Orthogonalization Complete ---")
    return out
