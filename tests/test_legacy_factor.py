"""Legacy ``factor.py`` twin (barra_factor_cal.factor) vs the reference's /factor.py."""
import contextlib
import io
import os
import warnings

import numpy as np
import pytest

from llm_driven_multi_factor_model_amd.models import factor_engine as FE

COLS = ["SIZE", "BETA", "HSIGMA", "RSTR", "DASTD", "CMRA", "NLSIZE", "BP", "STOM", "STOQ", "STOA",
        "CETOP", "ETOP", "YOYProfit", "YOYSales", "MLEV", "DTOA", "BLEV"]


@pytest.fixture(scope="module")
def data():
    prices, index, sw = FE.synthetic_prices(N=8, T=300, seed=2, suspend_frac=0.03)
    # legacy CETOP reads a precomputed TTM column (factor.py:358-399)
    rng = np.random.default_rng(0)
    prices["n_cashflow_act_ttm"] = rng.normal(2e8, 1.5e8, len(prices))
    return prices, index, sw


def test_legacy_run_schema_and_cmra_partial(data):
    from barra_factor_cal import factor as legacy
    prices, index, _ = data
    with contextlib.redirect_stdout(io.StringIO()):
        calc = legacy.FactorCalculator(prices.copy(), index.copy(), device="cpu")
        out = calc.run(FE.FACTORS_TO_RUN)
        cur = FE.FactorEngine(prices.copy(), index.copy(), device="cpu").run(["CMRA"])
    assert list(out.columns) == ["ts_code", "trade_date"] + COLS     # no ret / circ_mv
    # partial windows: CMRA defined from a stock's 3rd row on, the full-window variant from 252
    first = out.groupby("ts_code").head(5)["CMRA"]
    assert first.notna().sum() > 0 and cur.groupby("ts_code").head(5)["CMRA"].isna().all()


@pytest.mark.reference
def test_legacy_descriptors_match_reference(ref, data):
    if ref.legacy_factor is None:
        pytest.skip("reference factor.py not present")
    from barra_factor_cal import factor as legacy
    prices, index, _ = data
    warnings.simplefilter("ignore")
    with contextlib.redirect_stdout(io.StringIO()), contextlib.redirect_stderr(io.StringIO()):
        r = ref.legacy_factor.FactorCalculator(prices.copy(), index.copy()).run(FE.FACTORS_TO_RUN)
        o = legacy.FactorCalculator(prices.copy(), index.copy(), device="cpu").run(FE.FACTORS_TO_RUN)
    assert list(o.columns) == list(r.columns)
    assert (o["ts_code"].values == r["ts_code"].values).all()
    for c in COLS:
        a, b = o[c].to_numpy(np.float64), r[c].to_numpy(np.float64)
        assert (np.isnan(a) == np.isnan(b)).all(), c
        m = np.isfinite(b)
        np.testing.assert_allclose(a[m], b[m], rtol=2e-4, atol=1e-6, err_msg=c)


def test_legacy_main_writes_barra_files(tmp_path, data):
    from barra_factor_cal import factor as legacy
    prices, index, sw = data
    paths = {}
    for name, df in (("stk", prices), ("idx", index), ("sw", sw)):
        paths[name] = os.path.join(tmp_path, f"{name}.csv")
        df.to_csv(paths[name], index=False)
    with contextlib.redirect_stdout(io.StringIO()):
        barra, info = legacy.main(paths["stk"], paths["idx"], paths["sw"], str(tmp_path / "result"),
                                  device="cpu")
    assert os.path.isfile(tmp_path / "result" / "barra_factors_1014.csv")
    assert os.path.isfile(tmp_path / "result" / "industry_info_1014.csv")
    assert list(barra.columns) == FE.BARRA_OUTPUT_COLUMNS
    assert list(info.columns) == ["code", "industry_names", "start_date"]
    assert barra.groupby("stocknames").tail(1)["ret"].isna().all()   # t+1 alignment
