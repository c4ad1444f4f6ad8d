"""End-to-end CLI (demo.py equivalent) and the native CSV reader."""
import os
import subprocess
import sys

import numpy as np
import pandas as pd
import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def _run(*args, env=None):
    e = dict(os.environ, PYTHONPATH=ROOT, MFA_DEVICE="cpu")
    e.update(env or {})
    return subprocess.run([sys.executable, "-m", "llm_driven_multi_factor_model_amd.cli", *args],
                          capture_output=True, text=True, env=e, timeout=600)


def test_synth_then_risk_writes_demo_outputs(tmp_path):
    d = str(tmp_path)
    r = _run("synth", "--out", d, "--dates", "60", "--stocks", "90", "--industries", "6")
    assert r.returncode == 0, r.stderr
    r = _run("risk", "--data", f"{d}/barra_data_csi.csv", "--industry", f"{d}/industry_info.csv",
             "--out", f"{d}/results", "--sims", "4", "--device", "cpu")
    assert r.returncode == 0, r.stderr
    for f in ["factor_returns.csv", "r_squared.csv", "specific_returns.csv",
              "final_vol_regime_adj_covariance.csv", "volatility_multiplier_lambda.csv"]:
        assert os.path.exists(f"{d}/results/{f}"), f
    fr = pd.read_csv(f"{d}/results/factor_returns.csv", index_col=0)
    assert fr.shape == (60, 1 + 6 + 10) and fr.columns[0] == "country"
    cov = pd.read_csv(f"{d}/results/final_vol_regime_adj_covariance.csv", index_col=0)
    assert np.allclose(cov.values, cov.values.T)


def test_cli_preset_kept_and_attribution(tmp_path):
    """Unset flags must not override the preset (use4l keeps its 168-day VRA half-life);
    --attribution equal writes the per-date decomposition."""
    d = str(tmp_path)
    r = _run("synth", "--out", d, "--dates", "70", "--stocks", "80", "--industries", "5")
    assert r.returncode == 0, r.stderr
    r = _run("risk", "--data", f"{d}/barra_data_csi.csv", "--industry", f"{d}/industry_info.csv",
             "--out", f"{d}/res", "--preset", "use4l", "--sims", "3", "--eigen-shard", "sims",
             "--eigen-chunk", "2", "--attribution", "equal", "--device", "cpu")
    assert r.returncode == 0, r.stderr
    att = pd.read_csv(f"{d}/res/risk_attribution.csv", index_col=0)
    assert len(att) == 70
    ok = att.dropna()
    assert len(ok) > 10
    shares = ok[["country_share", "industry_share", "style_share", "specific_share"]].sum(1)
    assert np.allclose(shares, 1.0)
    assert (ok["total_vol"] >= ok["factor_vol"]).all()
    # the resolved config (logged by cmd_risk): use4l's VRA half-life survives, --sims wins
    assert '"vra_half_life": 168.0' in r.stderr and '"eigen_sims": 3' in r.stderr
    assert '"eigen_shard": "sims"' in r.stderr


def test_native_csv_reader_matches_pandas(tmp_path):
    from llm_driven_multi_factor_model_amd.utils import native_io
    rng = np.random.default_rng(0)
    n = 5000
    df = pd.DataFrame({"date": np.repeat(["2020/01/02", "2020/01/03"], n // 2),
                       "stocknames": [f"{i % 2500:06d}.SZ" for i in range(n)],
                       "capital": rng.random(n) * 1e5, "ret": rng.normal(0, 0.02, n),
                       "industry": [f"80{i % 28:04d}.SI" for i in range(n)], "size": rng.normal(size=n)})
    df.loc[3, "size"] = np.nan
    p = str(tmp_path / "x.csv")
    df.to_csv(p, index=False)
    got = native_io.read_csv(p)
    pd.testing.assert_frame_equal(got, pd.read_csv(p), check_dtype=False)


def test_native_reader_float32_columns(tmp_path):
    """Type 3 columns parse to float64 and round to float32 -- exactly pandas' float64 read
    followed by the reference's astype(float32) load downcast (load_data.py:13-25, Q27)."""
    from llm_driven_multi_factor_model_amd.utils import native_io
    rng = np.random.default_rng(3)
    n = 4000
    df = pd.DataFrame({"ts_code": [f"{i % 900:06d}.SZ" for i in range(n)],
                       "trade_date": np.repeat(["2020-01-02", "2020-01-03"], n // 2),
                       "close": rng.lognormal(2, 1, n), "total_mv": rng.lognormal(14, 2, n) * 1e3,
                       "pe_ttm": rng.normal(20, 30, n)})
    df.loc[7, "close"] = np.nan
    p = str(tmp_path / "prices.csv")
    df.to_csv(p, index=False)
    got = native_io.read_columns(p, {"ts_code": 1, "trade_date": 2, "close": 3, "total_mv": 3,
                                     "pe_ttm": 3})
    ref = pd.read_csv(p)
    for c in ("close", "total_mv", "pe_ttm"):
        assert got[c].dtype == np.float32
        np.testing.assert_array_equal(got[c], ref[c].to_numpy().astype(np.float32), err_msg=c)
    assert (got["trade_date"][:2] == 20200102).all() and got["ts_code"][0] == b"000000.SZ"


def test_panel_from_barra_csv_native_equals_pandas(tmp_path, monkeypatch):
    from llm_driven_multi_factor_model_amd.utils.io import panel_from_barra_csv
    d = str(tmp_path)
    assert _run("synth", "--out", d, "--dates", "20", "--stocks", "50", "--industries", "5").returncode == 0
    a = panel_from_barra_csv(f"{d}/barra_data_csi.csv", f"{d}/industry_info.csv")
    monkeypatch.setenv("MFA_NO_NATIVE_IO", "1")
    b = panel_from_barra_csv(f"{d}/barra_data_csi.csv", f"{d}/industry_info.csv")
    import torch
    for k in ["styles", "cap", "ret", "ind"]:
        torch.testing.assert_close(getattr(a, k), getattr(b, k), equal_nan=True)
    assert list(a.stocks) == list(b.stocks) and (a.dates == b.dates).all()


def test_cli_checkpoint_resume(tmp_path):
    """risk --checkpoint on the first dates, then risk --resume on the full file runs only the
    new dates; their factor returns equal a single full run's."""
    d = str(tmp_path)
    assert _run("synth", "--out", d, "--dates", "50", "--stocks", "70", "--industries", "5").returncode == 0
    df = pd.read_csv(f"{d}/barra_data_csi.csv")
    dates = sorted(df.date.unique())
    df[df.date.isin(dates[:35])].to_csv(f"{d}/first.csv", index=False)
    common = ["--industry", f"{d}/industry_info.csv", "--sims", "3", "--device", "cpu"]
    r = _run("risk", "--data", f"{d}/first.csv", "--out", f"{d}/r1", "--checkpoint", f"{d}/ck.pt", *common)
    assert r.returncode == 0, r.stderr
    r = _run("risk", "--data", f"{d}/barra_data_csi.csv", "--out", f"{d}/r2", "--resume", f"{d}/ck.pt", *common)
    assert r.returncode == 0, r.stderr
    r = _run("risk", "--data", f"{d}/barra_data_csi.csv", "--out", f"{d}/full", *common)
    assert r.returncode == 0, r.stderr
    f2 = pd.read_csv(f"{d}/r2/factor_returns.csv", index_col=0)
    ff = pd.read_csv(f"{d}/full/factor_returns.csv", index_col=0)
    assert len(f2) == 15
    np.testing.assert_allclose(f2.values, ff.values[35:], rtol=1e-12, atol=1e-15)


def test_native_matrix_csv_writer_matches_pandas(tmp_path):
    """specific_returns.csv through the native writer is byte-identical to pandas to_csv
    (numpy float32 repr: positional / scientific switch, integral '.0', NaN -> empty)."""
    from llm_driven_multi_factor_model_amd.utils import native_io
    rng = np.random.default_rng(1)
    v = (rng.normal(0, 0.02, (37, 23)) * rng.choice([1, 1e-6, 1e3, 1e17], (37, 23))).astype(np.float32)
    v[0, :6] = [0.0, -0.0, 1.0, -3.0, 1e-4, 9.999e-5]
    v[1, :4] = [np.nan, np.inf, -np.inf, 123456.0]
    v[2, :2] = [1e16, 9.9e15]
    idx = pd.date_range("2021-01-04", periods=37, freq="B")
    cols = [f"{i:06d}.SZ" for i in range(23)]
    a, b = str(tmp_path / "a.csv"), str(tmp_path / "b.csv")
    assert native_io.write_matrix_csv(a, v, idx.strftime("%Y-%m-%d"), cols)
    pd.DataFrame(v, index=idx, columns=cols).to_csv(b)
    assert open(a).read() == open(b).read()
    assert not native_io.write_matrix_csv(a, v, idx.strftime("%Y-%m-%d"), ["a,b"] + cols[1:])


def test_upstream_barra_data1_schema(tmp_path):
    """Original upstream dataset schema (Barra-master/dda_0921.ipynb#c1-c2: data/Barra_data1.csv,
    same 15 columns, ``HY00x`` industry codes): the loader is code-agnostic, so relabelling the
    industries and re-reading gives the same panel through both the native and pandas readers."""
    from llm_driven_multi_factor_model_amd.utils.io import panel_from_barra_csv
    d = str(tmp_path)
    assert _run("synth", "--out", d, "--dates", "15", "--stocks", "40", "--industries", "4").returncode == 0
    df = pd.read_csv(f"{d}/barra_data_csi.csv")
    info = pd.read_csv(f"{d}/industry_info.csv")
    relabel = {c: f"HY{i + 1:03d}" for i, c in enumerate(info["code"])}
    df["industry"] = df["industry"].map(relabel)
    info["code"] = info["code"].map(relabel)
    df.to_csv(f"{d}/Barra_data1.csv", index=False)
    info.to_csv(f"{d}/industry_info_hy.csv", index=False)
    a = panel_from_barra_csv(f"{d}/barra_data_csi.csv", f"{d}/industry_info.csv")
    b = panel_from_barra_csv(f"{d}/Barra_data1.csv", f"{d}/industry_info_hy.csv")
    import torch
    for k in ["styles", "cap", "ret", "ind"]:
        torch.testing.assert_close(getattr(a, k), getattr(b, k), equal_nan=True)
    assert b.P == 4 and list(a.stocks) == list(b.stocks)
