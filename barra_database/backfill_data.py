"""Backfill a historical window of daily_basic per stock (reference: backfill_data.py:19-83).

One Tushare call per stock, ``daily_basic(ts_code=code, start_date, end_date)``
(backfill_data.py:56-60), under the reference's limiter: 480 calls per minute, 3 attempts with
a 5 s back-off, 0.125 s between successful calls, duplicate-key errors taken as success.
"""
from __future__ import annotations

import time

from . import tushare_fetcher as _default_fetcher
from .ingest import update_per_stock

BACKFILL_START_DATE = "20190101"
BACKFILL_END_DATE = "20191231"


def stock_codes(db) -> list:
    """``stock_info``'s codes (``distinct`` as in backfill_data.py:31, a find otherwise)."""
    coll = db["stock_info"]
    if hasattr(coll, "distinct"):
        return list(coll.distinct("ts_code"))
    return [d["ts_code"] for d in coll.find({}, {"ts_code": 1, "_id": 0})]


def backfill_historical_prices(db, stock_list=None, start=BACKFILL_START_DATE, end=BACKFILL_END_DATE,
                               fetcher=_default_fetcher, sleep=time.sleep, clock=time.time):
    """Returns the number of rows fetched (duplicates skipped by the unique index included)."""
    if stock_list is None:
        stock_list = stock_codes(db)
        if not stock_list:
            print("stock_info is empty: no stock list to backfill.")
            return 0

    def fetch(code):
        return fetcher.fetch_daily_basic_by_stock(code, start, end)

    return update_per_stock(db, "daily_prices", stock_list, fetch, 480, sleep=sleep, clock=clock)
