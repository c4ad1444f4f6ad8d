"""Per-stock backfill and gap-fill jobs against a fake Tushare fetcher (CPU).

Reference: Barra_database/database/backfill_data.py:43-77 (one ``daily_basic(ts_code=code,
start_date, end_date)`` per stock, 480 calls / min, 3 attempts) and
Barra_database/database/fill_missing_data.py:24-64 (only the stocks with no daily_prices row,
window 20200101 -> yesterday).  No network: the fetcher records every call.
"""
from datetime import date

import pandas as pd

from barra_database import backfill_data, fill_missing_data
from tests._fakemongo import FakeDB


class FakeFetcher:
    def __init__(self, fail_first=()):
        self.calls = []
        self.fail_left = {c: 1 for c in fail_first}

    def fetch_daily_basic_by_stock(self, ts_code, start_date, end_date):
        self.calls.append((ts_code, start_date, end_date))
        if self.fail_left.get(ts_code):
            self.fail_left[ts_code] -= 1
            raise RuntimeError("transient API error")
        days = pd.date_range(pd.Timestamp(start_date), periods=3, freq="B").strftime("%Y%m%d")
        return pd.DataFrame({"ts_code": ts_code, "trade_date": days, "close": 10.0})

    def fetch_daily_prices(self, *a, **k):  # the whole-market call must not be used
        raise AssertionError("market-wide daily_basic called by a per-stock job")


class Clock:
    def __init__(self):
        self.t = 0.0
        self.sleeps = []

    def __call__(self):
        return self.t

    def sleep(self, s):
        self.sleeps.append(s)
        if s > 1:  # the per-call 0.125 s pauses do not advance this clock
            self.t += s


def _db(codes, have=()):
    db = FakeDB()
    db["stock_info"].docs = [{"ts_code": c} for c in codes]
    db["daily_prices"].unique = ("ts_code", "trade_date")
    db["daily_prices"].docs = [{"ts_code": c, "trade_date": "20200102"} for c in have]
    return db


def test_backfill_one_call_per_stock_with_its_code():
    codes = ["000001.SZ", "000002.SZ", "600000.SH"]
    db, f, clk = _db(codes), FakeFetcher(), Clock()
    n = backfill_data.backfill_historical_prices(db, fetcher=f, sleep=clk.sleep, clock=clk)
    assert f.calls == [(c, "20190101", "20191231") for c in codes]
    assert n == 9
    rows = db["daily_prices"].docs
    assert sorted({r["ts_code"] for r in rows}) == codes
    assert all(len([r for r in rows if r["ts_code"] == c]) == 3 for c in codes)
    assert clk.sleeps == [0.125] * 3  # per-call pause, no rate-limit wait below 480 calls


def test_backfill_retry_and_rate_limit():
    codes = [f"{i:06d}.SZ" for i in range(482)]
    db, f, clk = _db(codes), FakeFetcher(fail_first=["000005.SZ"]), Clock()
    backfill_data.backfill_historical_prices(db, fetcher=f, sleep=clk.sleep, clock=clk)
    assert len(f.calls) == 483                       # one retry
    assert f.calls[5] == f.calls[6] == ("000005.SZ", "20190101", "20191231")
    assert clk.sleeps.count(5.0) == 1                # the 5 s back-off
    waits = [s for s in clk.sleeps if s not in (0.125, 5.0)]
    assert len(waits) == 1                           # one rate-limit wait after 480 calls
    assert abs(waits[0] - (60 - 5.0 + 1)) < 1e-9     # 60 - elapsed + 1 (ingest.RateLimiter)
    assert clk.sleeps.index(waits[0]) == 481         # after the 480th success (+ the back-off)


def test_backfill_rerun_is_idempotent():
    codes = ["000001.SZ", "000002.SZ"]
    db, f, clk = _db(codes), FakeFetcher(), Clock()
    backfill_data.backfill_historical_prices(db, fetcher=f, sleep=clk.sleep, clock=clk)
    backfill_data.backfill_historical_prices(db, fetcher=f, sleep=clk.sleep, clock=clk)
    assert len(db["daily_prices"].docs) == 6         # duplicate-key inserts skipped
    assert len(f.calls) == 4                         # no retry on duplicate-key errors


def test_fill_missing_only_missing_stocks_reference_window():
    codes = ["000001.SZ", "000002.SZ", "300750.SZ", "600000.SH"]
    db, f, clk = _db(codes, have=["000002.SZ", "600000.SH"]), FakeFetcher(), Clock()
    n = fill_missing_data.fill_missing_daily_prices(db, fetcher=f, sleep=clk.sleep, clock=clk,
                                                    today=date(2025, 3, 1))
    assert f.calls == [("000001.SZ", "20200101", "20250228"), ("300750.SZ", "20200101", "20250228")]
    assert n == 6
    assert fill_missing_data.missing_stocks(db) == []
    f2 = FakeFetcher()
    assert fill_missing_data.fill_missing_daily_prices(db, fetcher=f2, sleep=clk.sleep, clock=clk) == 0
    assert f2.calls == []


def test_fill_missing_default_end_is_yesterday():
    assert fill_missing_data.yesterday(date(2024, 1, 1)) == "20231231"
