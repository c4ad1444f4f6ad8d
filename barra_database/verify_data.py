"""Coverage check (reference: verify_data.py:8-35)."""
from __future__ import annotations


def get_unique_stock_count(db, collection: str = "daily_prices") -> int:
    c = db[collection]
    if hasattr(c, "distinct"):
        return len(c.distinct("ts_code"))
    return len({d["ts_code"] for d in c.find({}, {"ts_code": 1, "_id": 0})})
