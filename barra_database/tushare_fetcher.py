"""Tushare Pro fetchers (reference: Barra_database/database/tushare_fetcher.py:17-315).

The token comes from TUSHARE_TOKEN; with no token or no ``tushare`` package every fetcher
returns an empty DataFrame.  The statement tables request the reference's full column sets
(``tushare_fields.py``: 167 fina_indicator, 158 balancesheet, 97 cashflow, 94 income fields)
with ``update_flag='1'`` (latest revision only), so the stored Mongo collections have the
reference's schema; pass ``fields=`` to request a different set.
"""
from __future__ import annotations

import os

import pandas as pd

from .tushare_fields import (BALANCESHEET_FIELDS, CASHFLOW_FIELDS, FINA_INDICATOR_FIELDS,
                             INCOME_FIELDS)

TOKEN = os.environ.get("TUSHARE_TOKEN")
try:  # optional dependency
    import tushare as ts  # noqa: F401
    pro = ts.pro_api(TOKEN) if TOKEN else None
except Exception:
    pro = None

DAILY_BASIC_FIELDS = ["ts_code", "trade_date", "close", "turnover_rate", "turnover_rate_f", "volume_ratio",
                      "pe", "pe_ttm", "pb", "ps", "ps_ttm", "dv_ratio", "dv_ttm", "total_share",
                      "float_share", "free_share", "total_mv", "circ_mv"]


def _call(api: str, **kw) -> pd.DataFrame:
    if pro is None:
        return pd.DataFrame()
    fields = kw.pop("fields", None)
    if fields is not None:
        kw["fields"] = ",".join(fields) if isinstance(fields, (list, tuple)) else fields
    return getattr(pro, api)(**kw)


def fetch_stock_info() -> pd.DataFrame:
    if pro is None:
        return pd.DataFrame()
    return pro.query("stock_basic", exchange="", list_status="L",
                     fields="ts_code,symbol,name,area,industry,list_date")


def fetch_trade_calendar(start_date: str, end_date: str) -> list:
    cal = _call("trade_cal", exchange="", start_date=start_date, end_date=end_date)
    return [] if cal.empty else cal[cal["is_open"] == 1]["cal_date"].tolist()


def fetch_daily_prices(start_date: str, end_date: str, fields=DAILY_BASIC_FIELDS) -> pd.DataFrame:
    return _call("daily_basic", start_date=start_date, end_date=end_date, fields=fields)


def fetch_daily_basic_by_stock(ts_code: str, start_date: str, end_date: str,
                               fields=DAILY_BASIC_FIELDS) -> pd.DataFrame:
    """One stock's daily_basic rows over [start_date, end_date] (the per-stock pull of
    Barra_database/database/backfill_data.py:56-60 and fill_missing_data.py:57)."""
    return _call("daily_basic", ts_code=ts_code, start_date=start_date, end_date=end_date,
                 fields=fields)


def fetch_daily_basic_by_date(trade_date: str, fields=DAILY_BASIC_FIELDS) -> pd.DataFrame:
    return _call("daily_basic", trade_date=trade_date, fields=fields)


def fetch_financial_indicators_by_stock(ts_code: str, fields=FINA_INDICATOR_FIELDS) -> pd.DataFrame:
    return _call("fina_indicator", ts_code=ts_code, update_flag="1", fields=fields)


def fetch_balancesheet_by_stock(ts_code: str, fields=BALANCESHEET_FIELDS) -> pd.DataFrame:
    return _call("balancesheet", ts_code=ts_code, update_flag="1", fields=fields)


def fetch_cashflow_by_stock(ts_code: str, fields=CASHFLOW_FIELDS) -> pd.DataFrame:
    return _call("cashflow", ts_code=ts_code, update_flag="1", fields=fields)


def fetch_income_by_stock(ts_code: str, fields=INCOME_FIELDS) -> pd.DataFrame:
    return _call("income", ts_code=ts_code, update_flag="1", fields=fields)


def fetch_index_info(market: str = "SSE") -> pd.DataFrame:
    return _call("index_basic", market=market)


def fetch_daily_index_prices(ts_code: str, start_date: str, end_date: str) -> pd.DataFrame:
    return _call("index_daily", ts_code=ts_code, start_date=start_date, end_date=end_date)


def fetch_index_components(ts_code: str, trade_date: str | None = None) -> pd.DataFrame:
    kw = {"index_code": ts_code}
    if trade_date:
        kw["trade_date"] = trade_date
    return _call("index_weight", **kw)


def fetch_sw_industries(src: str = "SW2021") -> pd.DataFrame:
    return _call("index_member_all", src=src) if pro is not None and hasattr(pro, "index_member_all") \
        else pd.DataFrame()
