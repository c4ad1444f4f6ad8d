"""Repair stocks missing from daily_prices (reference: fill_missing_data.py:16-68).

The stocks of ``stock_info`` with no ``daily_prices`` row at all are pulled one call each,
``daily_basic(ts_code=code, start_date='20200101', end_date=yesterday)``
(fill_missing_data.py:51-58), through the shared limiter / retry loop of ``ingest``.
"""
from __future__ import annotations

import time
from datetime import date, timedelta

from . import tushare_fetcher as _default_fetcher
from .ingest import update_per_stock

FILL_START_DATE = "20200101"


def missing_stocks(db) -> list:
    have = set(db["daily_prices"].distinct("ts_code")) if hasattr(db["daily_prices"], "distinct") else \
        {d["ts_code"] for d in db["daily_prices"].find({}, {"ts_code": 1, "_id": 0})}
    allc = [d["ts_code"] for d in db["stock_info"].find({}, {"ts_code": 1, "_id": 0})]
    return sorted(set(allc) - have)


def yesterday(today: date | None = None) -> str:
    return ((today or date.today()) - timedelta(days=1)).strftime("%Y%m%d")


def fill_missing_daily_prices(db, start=FILL_START_DATE, end=None, fetcher=_default_fetcher,
                              sleep=time.sleep, clock=time.time, today: date | None = None):
    """``end`` defaults to yesterday (relative to ``today``, the real date by default)."""
    end = yesterday(today) if end is None else end
    todo = missing_stocks(db)
    print(f"missing stocks: {len(todo)}")
    if not todo:
        return 0

    def fetch(code):
        return fetcher.fetch_daily_basic_by_stock(code, start, end)

    return update_per_stock(db, "daily_prices", todo, fetch, 480, sleep=sleep, clock=clock)
