"""``load_data_v0.py`` compatibility (reference: Barra_factor_cal/load_data_v0.py, a module-level
script).  Differences from :mod:`barra_factor_cal.load_data` kept here:
CSI 300 (``000300.SH``, load_data_v0.py:42) instead of SSE 50 (quirk Q20), financial indicators
merged WITHOUT the ann_date dedupe (:231-236), and no forward-fill / fill step.
The reference runs at import time; here the same flow is one call.
"""
from __future__ import annotations

from .load_data import load_and_prepare_data, robust_merge_asof  # noqa: F401

INDEX_CODE = "000300.SH"


def load_and_prepare_data_v0(db=None, start_date: str = "20200101",
                             start_date_financial: str = "20190101", end_date: str | None = None):
    """Returns ``(stock_price_with_financials_df, index_df, sw_industry_df)``."""
    return load_and_prepare_data(db, index_code=INDEX_CODE, start_date=start_date,
                                 start_date_financial=start_date_financial, end_date=end_date,
                                 dedupe_indicators=False, fill=False)
