"""Repair stocks missing from daily_prices (reference: fill_missing_data.py:16-68)."""
from __future__ import annotations

import time

from . import tushare_fetcher as _default_fetcher
from .ingest import update_per_stock


def missing_stocks(db) -> list:
    have = set(db["daily_prices"].distinct("ts_code")) if hasattr(db["daily_prices"], "distinct") else \
        {d["ts_code"] for d in db["daily_prices"].find({}, {"ts_code": 1, "_id": 0})}
    allc = [d["ts_code"] for d in db["stock_info"].find({}, {"ts_code": 1, "_id": 0})]
    return sorted(set(allc) - have)


def fill_missing_daily_prices(db, start="20190101", end="20251231", fetcher=_default_fetcher,
                              sleep=time.sleep, clock=time.time):
    todo = missing_stocks(db)

    def fetch(code):
        df = fetcher.fetch_daily_prices(start, end)
        return df[df["ts_code"] == code] if not df.empty else df

    return update_per_stock(db, "daily_prices", todo, fetch, 480, sleep=sleep, clock=clock)
