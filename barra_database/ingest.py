"""Rate limiting, retry and duplicate-tolerant bulk inserts shared by the updaters.

Semantics of update_mongo_db.py: per-minute call budgets (480 for statement endpoints, 190 for
index endpoints, :151 / :411), 3 attempts with a 5 s back-off (:172-184), duplicate-key errors
treated as success (:177-178), ``insert_many(ordered=False)`` so re-runs are idempotent under a
unique index (:119-128), and resume-from-last-date (:19-30).
"""
from __future__ import annotations

import time
from dataclasses import dataclass, field
from typing import Callable

import pandas as pd


@dataclass
class RateLimiter:
    calls_per_minute: int
    clock: Callable[[], float] = time.time
    sleep: Callable[[float], None] = time.sleep
    count: int = 0
    start: float = field(default=None)

    def __post_init__(self):
        self.start = self.clock() if self.start is None else self.start

    def acquire(self):
        if self.count >= self.calls_per_minute:
            elapsed = self.clock() - self.start
            if elapsed < 60:
                self.sleep(60 - elapsed + 1)
            self.count, self.start = 0, self.clock()

    def done(self):
        self.count += 1


def with_retry(fn: Callable[[], pd.DataFrame], attempts: int = 3, backoff: float = 5.0,
               sleep: Callable[[float], None] = time.sleep, label: str = ""):
    """Run ``fn`` up to ``attempts`` times; duplicate-key errors count as success (None)."""
    last = None
    for a in range(attempts):
        try:
            return fn()
        except Exception as e:  # network / API errors
            if "duplicate key error" in str(e).lower():
                return None
            last = e
            print(f"\nError {label} on attempt {a + 1}: {e}")
            if a < attempts - 1:
                sleep(backoff)
    print(f"Failed {label} after {attempts} attempts: {last}")
    return None


def insert_records(collection, df: pd.DataFrame | None) -> int:
    if df is None or df.empty:
        return 0
    records = df.to_dict("records")
    try:
        collection.insert_many(records, ordered=False)
    except Exception as e:
        print(f"An error occurred during bulk insert: {e}. Some duplicates may have been skipped.")
    return len(records)


def get_last_update_date(db, collection_name: str, date_col: str = "trade_date",
                         default: str = "20190101") -> pd.Timestamp:
    try:
        latest = db[collection_name].find_one(sort=[(date_col, -1)])
        if latest and date_col in latest:
            return pd.to_datetime(str(latest[date_col]))
    except Exception as e:
        print(f"Error reading last date from {collection_name}: {e}")
    return pd.to_datetime(default)


def update_per_stock(db, collection_name: str, stock_list, fetch: Callable[[str], pd.DataFrame],
                     calls_per_minute: int = 480, per_call_sleep: float = 0.125,
                     sleep: Callable[[float], None] = time.sleep, clock=time.time) -> int:
    """Per-stock statement pulls with the reference's rate limit / retry loop."""
    if not stock_list:
        print(f"Stock list is empty, skipping {collection_name} update.")
        return 0
    coll = db[collection_name]
    rl = RateLimiter(calls_per_minute, clock=clock, sleep=sleep)
    n = 0
    for code in stock_list:
        rl.acquire()

        def call(code=code):
            df = fetch(code)
            ins = insert_records(coll, df)
            return ins

        got = with_retry(call, sleep=sleep, label=f"fetching {collection_name} for {code}")
        if got is not None:
            n += got
            rl.done()
            if per_call_sleep:
                sleep(per_call_sleep)
    return n
