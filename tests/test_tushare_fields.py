"""The Tushare statement fetchers request the reference's full column sets (fake ``pro``)."""
import ast
import os

import pandas as pd
import pytest

import barra_database.tushare_fetcher as tf

REF = "/root/reference/Barra_database/database/tushare_fetcher.py"


class FakePro:
    def __init__(self):
        self.calls = []

    def __getattr__(self, api):
        def fn(**kw):
            self.calls.append((api, kw))
            return pd.DataFrame({"ts_code": ["000001.SZ"]})
        return fn


def _reference_fields():
    tree = ast.parse(open(REF, encoding="utf-8").read())
    out = {}
    for fn in tree.body:
        if isinstance(fn, ast.FunctionDef):
            for node in ast.walk(fn):
                if isinstance(node, ast.Assign) and getattr(node.targets[0], "id", None) == "fields_list":
                    out[fn.name] = [e.value for e in node.value.elts]
    return out


@pytest.mark.reference
def test_statement_fields_equal_reference(monkeypatch):
    if not os.path.exists(REF):
        pytest.skip("reference not mounted")
    fake = FakePro()
    monkeypatch.setattr(tf, "pro", fake)
    ref = _reference_fields()
    for name, api in [("fetch_financial_indicators_by_stock", "fina_indicator"),
                      ("fetch_balancesheet_by_stock", "balancesheet"),
                      ("fetch_cashflow_by_stock", "cashflow"),
                      ("fetch_income_by_stock", "income")]:
        getattr(tf, name)("000001.SZ")
        got_api, kw = fake.calls[-1]
        assert got_api == api and kw["ts_code"] == "000001.SZ" and kw["update_flag"] == "1"
        assert kw["fields"].split(",") == ref[name], name


def test_field_counts_and_factor_columns():
    assert len(tf.FINA_INDICATOR_FIELDS) == 167 and len(tf.BALANCESHEET_FIELDS) == 158
    assert len(tf.CASHFLOW_FIELDS) == 97 and len(tf.INCOME_FIELDS) == 94
    # every statement column the factor pipeline consumes is requested
    for col in ("debt_to_assets", "q_profit_yoy", "q_sales_yoy"):
        assert col in tf.FINA_INDICATOR_FIELDS
    for col in ("total_ncl", "total_hldr_eqy_inc_min_int"):
        assert col in tf.BALANCESHEET_FIELDS
    assert "n_cashflow_act" in tf.CASHFLOW_FIELDS
