"""Incremental MongoDB updater (reference: Barra_database/database/update_mongo_db.py).

Every ``update_*`` takes ``db`` plus an optional ``fetcher`` module/object (defaults to
``tushare_fetcher``) and ``sleep``/``clock`` hooks so the rate-limit / retry / resume logic is
testable offline.
"""
from __future__ import annotations

import time
from datetime import date, timedelta

import pandas as pd

from . import tushare_fetcher as _default_fetcher
from .ingest import RateLimiter, get_last_update_date, insert_records, update_per_stock, with_retry

MONGO_CONNECTION_STRING = "mongodb://localhost:27017/"
DB_NAME = "barra_financial_data"


def update_stock_info(db, fetcher=_default_fetcher):
    coll = db["stock_info"]
    try:
        df = fetcher.fetch_stock_info()
        if df.empty:
            print("Warning: Fetched stock list is empty.")
            return []
        coll.drop()
        coll.insert_many(df.to_dict("records"))
        return df["ts_code"].tolist()
    except Exception as e:
        print(f"An error occurred while updating stock info: {e}")
        return []


def update_daily_prices(db, fetcher=_default_fetcher, sleep=time.sleep, today=None):
    name = "daily_prices"
    last = get_last_update_date(db, name, "trade_date")
    start = last.strftime("%Y%m%d") if last == pd.to_datetime("20190101") else \
        (last + timedelta(days=1)).strftime("%Y%m%d")
    end = (today or date.today()).strftime("%Y%m%d")
    if start > end:
        print("Daily prices are already up to date.")
        return 0
    try:
        days = fetcher.fetch_trade_calendar(start, end)
    except Exception as e:
        print(f"Error fetching trade calendar: {e}")
        return 0
    frames = []
    for d in days:
        df = with_retry(lambda d=d: fetcher.fetch_daily_basic_by_date(d), attempts=1, sleep=sleep,
                        label=f"daily prices {d}")
        if df is not None and not df.empty:
            frames.append(df)
        sleep(0.2)
    return insert_records(db[name], pd.concat(frames, ignore_index=True) if frames else None)


def _stmt(name, fetch_attr):
    def upd(db, stock_list, fetcher=_default_fetcher, sleep=time.sleep, clock=time.time):
        return update_per_stock(db, name, stock_list, getattr(fetcher, fetch_attr), 480,
                                sleep=sleep, clock=clock)
    upd.__name__ = f"update_{name}"
    return upd


update_financial_indicators = _stmt("financial_indicators", "fetch_financial_indicators_by_stock")
update_balancesheet = _stmt("balancesheet", "fetch_balancesheet_by_stock")
update_cashflow = _stmt("cashflow", "fetch_cashflow_by_stock")
update_income = _stmt("income", "fetch_income_by_stock")


def update_index_info(db, fetcher=_default_fetcher):
    df = fetcher.fetch_index_info()
    if df.empty:
        return 0
    db["index_info"].drop()
    return insert_records(db["index_info"], df)


def update_daily_index_prices(db, index_list, fetcher=_default_fetcher, sleep=time.sleep, clock=time.time,
                              today=None):
    name = "index_daily_prices"
    last = get_last_update_date(db, name, "trade_date")
    start = (last + timedelta(days=1)).strftime("%Y%m%d")
    end = ((today or date.today()) - timedelta(days=1)).strftime("%Y%m%d")
    if start > end:
        print("Index daily prices are already up to date.")
        return 0
    rl = RateLimiter(190, clock=clock, sleep=sleep)
    frames = []
    for code in index_list:
        rl.acquire()
        df = with_retry(lambda c=code: fetcher.fetch_daily_index_prices(c, start, end), sleep=sleep,
                        label=f"index prices {code}")
        if df is not None:
            frames.append(df)
            rl.done()
    return insert_records(db[name], pd.concat(frames, ignore_index=True) if frames else None)


def update_index_components(db, index_list, fetcher=_default_fetcher, sleep=time.sleep, clock=time.time):
    rl = RateLimiter(190, clock=clock, sleep=sleep)
    n = 0
    for code in index_list:
        rl.acquire()
        df = with_retry(lambda c=code: fetcher.fetch_index_components(c), sleep=sleep,
                        label=f"index components {code}")
        if df is not None:
            n += insert_records(db["index_components"], df)
            rl.done()
    return n


def update_sw_industries_from_csv(db, csv_file_path: str):
    try:
        df = pd.read_csv(csv_file_path)
    except FileNotFoundError:
        print(f"ERROR: The file was not found at the specified path: {csv_file_path}")
        return 0
    if df.empty:
        print("Warning: The CSV file is empty. No data was inserted.")
        return 0
    db["sw_industries"].drop()
    db["sw_industries"].insert_many(df.to_dict("records"))
    return len(df)


def main():
    from pymongo import MongoClient
    import os
    client = MongoClient(os.environ.get("MFA_MONGO_URI", MONGO_CONNECTION_STRING))
    db = client[os.environ.get("MFA_MONGO_DB", DB_NAME)]
    stocks = update_stock_info(db)
    update_daily_prices(db)
    update_daily_index_prices(db, ["000300.SH", "000016.SH", "000903.SH"])
    client.close()
    return stocks


if __name__ == "__main__":
    main()
