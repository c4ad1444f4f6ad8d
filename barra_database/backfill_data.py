"""Backfill a historical window of daily_basic per stock (reference: backfill_data.py:19-83)."""
from __future__ import annotations

import time

from . import tushare_fetcher as _default_fetcher
from .ingest import update_per_stock

BACKFILL_START_DATE = "20190101"
BACKFILL_END_DATE = "20191231"


def backfill_historical_prices(db, stock_list=None, start=BACKFILL_START_DATE, end=BACKFILL_END_DATE,
                               fetcher=_default_fetcher, sleep=time.sleep, clock=time.time):
    if stock_list is None:
        stock_list = [d["ts_code"] for d in db["stock_info"].find({}, {"ts_code": 1, "_id": 0})]

    def fetch(code):
        df = fetcher.fetch_daily_prices(start, end)
        return df[df["ts_code"] == code] if not df.empty else df

    return update_per_stock(db, "daily_prices", stock_list, fetch, 480, sleep=sleep, clock=clock)
