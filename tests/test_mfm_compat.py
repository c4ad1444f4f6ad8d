"""Drop-in ``mfm`` package vs the reference ``mfm`` on the BASELINE toy config (CPU)."""
import contextlib
import io

import numpy as np
import pandas as pd
import pytest
import torch

import mfm
from llm_driven_multi_factor_model_amd.models.panel import synthetic_panel


def toy_frame(T=100, N=50, P=3, Q=3, seed=0, missing=0.05):
    """BASELINE.md recipe: [date(str), stocknames, capital, ret, ind0..ind{P-1}, sty0..sty{Q-1}].

    Raw, unrounded float64 values (what demo.py's pd.read_csv hands the reference)."""
    rng = np.random.default_rng(seed)
    dates = pd.bdate_range("2020-01-02", periods=T).strftime("%Y/%m/%d")
    rows = []
    for t, d in enumerate(dates):
        for i in range(N):
            if rng.random() < missing:
                continue
            rows.append([d, f"{i:06d}.SZ", float(rng.lognormal(12, 1)), float(rng.normal(0, 0.02))])
    df = pd.DataFrame(rows, columns=["date", "stocknames", "capital", "ret"])
    idx = df.stocknames.str[:6].astype(int).values
    for j in range(P):
        df[f"ind{j}"] = (idx % P == j).astype(np.int64)
    for q in range(Q):
        df[f"sty{q}"] = rng.normal(0.1 * q, 1, len(df))
    return df


def run_ref(ref, df, P, Q, M=5):
    with contextlib.redirect_stdout(io.StringIO()):
        m = ref.MFM.MFM(df, P, Q)
        f, e, r2 = m.reg_by_time()
        nw = m.Newey_West_by_time(q=2, tao=252)
    return m, f, e, r2, nw


@pytest.mark.reference
def test_mfm_reg_and_newey_west_parity(ref, monkeypatch):
    monkeypatch.setenv("MFA_DEVICE", "cpu")
    df = toy_frame()
    rm, rf, re_, rr2, rnw = run_ref(ref, df, 3, 3)
    m = mfm.MFM(df, 3, 3)
    f, e, r2 = m.reg_by_time()
    assert list(f.columns) == list(rf.columns) and (f.index == rf.index).all()
    np.testing.assert_allclose(f.values, rf.values, rtol=1e-9, atol=1e-13)
    np.testing.assert_allclose(r2.values, rr2.values, rtol=1e-9, atol=1e-12)
    for a, b in zip(e, re_):
        assert list(a.columns) == list(b.columns)
        np.testing.assert_allclose(a.values, b.values, rtol=1e-9, atol=1e-13)
    np.testing.assert_allclose(m.last_capital, rm.last_capital)
    nw = m.Newey_West_by_time(q=2, tao=252)
    assert len(nw) == len(rnw)
    for a, b in zip(nw, rnw):
        assert a.empty == b.empty
        if not a.empty:
            np.testing.assert_allclose(a.values, b.values, rtol=1e-9, atol=1e-16)


@pytest.mark.reference
def test_mfm_vra_parity_given_same_eigen_input(ref, monkeypatch):
    monkeypatch.setenv("MFA_DEVICE", "cpu")
    df = toy_frame(T=60, seed=1)
    rm, *_ = run_ref(ref, df, 3, 3)
    m = mfm.MFM(df, 3, 3)
    m.reg_by_time()
    m.Newey_West_by_time()
    er = m.eigen_risk_adj_by_time(M=8, scale_coef=1.4)
    assert sum(not x.empty for x in er) > 40
    vr, lam = m.vol_regime_adj_by_time(tao=42)
    rm.eigen_risk_adj_cov = er  # feed our eigen-adjusted series to the reference VRA
    with contextlib.redirect_stdout(io.StringIO()):
        rvr, rlam = rm.vol_regime_adj_by_time(tao=42)
    np.testing.assert_allclose(lam, rlam, rtol=1e-12)
    for a, b in zip(vr, rvr):
        if not a.empty:
            np.testing.assert_allclose(a.values, b.values, rtol=1e-12)


def test_mfm_stage_order_exceptions():
    m = mfm.MFM(toy_frame(T=20, N=30), 3, 3)
    with pytest.raises(Exception):
        m.Newey_West_by_time()
    with pytest.raises(Exception):
        m.eigen_risk_adj_by_time()


@pytest.mark.reference
def test_crosssection_compat(ref, monkeypatch):
    monkeypatch.setenv("MFA_DEVICE", "cpu")
    df = toy_frame(T=1, N=80, seed=3, missing=0.0)
    base, sty, ind = df.iloc[:, :4], df.iloc[:, -3:], df.iloc[:, 4:7]
    with contextlib.redirect_stdout(io.StringIO()):
        rf, re_, rex, rr2 = ref.CrossSection.CrossSection(base, sty, ind).reg()
    f, e, ex, r2 = mfm.CrossSection(base, sty, ind).reg()
    np.testing.assert_allclose(f, rf, rtol=1e-9, atol=1e-13)
    np.testing.assert_allclose(e, re_, rtol=1e-9, atol=1e-13)
    np.testing.assert_allclose(np.asarray(ex), np.asarray(rex), rtol=1e-7, atol=1e-9)
    assert abs(r2 - rr2) < 1e-12


@pytest.mark.reference
def test_utils_newey_west_and_bayes(ref, monkeypatch):
    monkeypatch.setenv("MFA_DEVICE", "cpu")
    rng = np.random.default_rng(0)
    F = pd.DataFrame(rng.normal(0, 0.01, (80, 5)), columns=list("abcde"))
    np.testing.assert_allclose(mfm.utils.Newey_West(F, 2, 60).values, ref.utils.Newey_West(F, 2, 60).values,
                               rtol=1e-10)
    with pytest.raises(Exception):
        mfm.utils.Newey_West(F[:4], 2, 60)
    vol, cap = rng.random(200) * 0.05, rng.lognormal(10, 1, 200)
    np.testing.assert_allclose(mfm.utils.bayes_shrink(vol, cap), ref.utils.bayes_shrink(vol, cap), rtol=1e-5)


def test_inv_solver_raises_on_singular(monkeypatch):
    """solver='inv' (stale build, quirk Q4): an empty industry raises LinAlgError; pinv does not."""
    monkeypatch.setenv("MFA_DEVICE", "cpu")
    df = toy_frame(T=1, N=60, seed=4, missing=0.0)
    df["ind2"] = 0
    df.loc[df.stocknames.str[:6].astype(int) % 3 == 2, "ind1"] = 1  # industry 2 now empty
    base, sty, ind = df.iloc[:, :4], df.iloc[:, -3:], df.iloc[:, 4:7]
    f, *_ = mfm.CrossSection(base, sty, ind).reg()
    assert np.isfinite(f).all() and abs(f[3]) < 1e-12  # pinv semantics: empty industry -> 0
    with pytest.raises(np.linalg.LinAlgError):
        mfm.CrossSection(base, sty, ind, solver="inv").reg()
    good = toy_frame(T=1, N=60, seed=4, missing=0.0)
    fi, *_ = mfm.CrossSection(good.iloc[:, :4], good.iloc[:, -3:], good.iloc[:, 4:7], solver="inv").reg()
    fp, *_ = mfm.CrossSection(good.iloc[:, :4], good.iloc[:, -3:], good.iloc[:, 4:7]).reg()
    np.testing.assert_allclose(fi, fp)
    m = mfm.MFM(pd.concat([good.assign(date="2020/01/02"), df.assign(date="2020/01/03")]), 3, 3,
                solver="inv")
    with pytest.raises(np.linalg.LinAlgError):
        with contextlib.redirect_stdout(io.StringIO()):
            m.reg_by_time()


@pytest.mark.gpu
def test_mfm_gpu_matches_cpu(cuda, monkeypatch):
    """The drop-in mfm.MFM on the MI355X (HIP kernels) == the CPU float64 path: factor returns,
    R^2 and the Newey-West series (the eigen adjustment draws device-specific sims and is
    covered statistically in test_eigen.py)."""
    df = toy_frame(T=120, N=60, P=4, Q=3, seed=2)
    out = {}
    for dev in ("cpu", "cuda:0"):
        monkeypatch.setenv("MFA_DEVICE", dev)
        with contextlib.redirect_stdout(io.StringIO()):
            m = mfm.MFM(df, 4, 3)
            f, e, r2 = m.reg_by_time()
            nw = m.Newey_West_by_time(q=2, tao=252)
        out[dev] = (f, r2, nw)
    fc, rc, nc = out["cpu"]
    fg, rg, ng = out["cuda:0"]
    np.testing.assert_allclose(fg.values, fc.values, rtol=1e-9, atol=1e-13)
    np.testing.assert_allclose(rg.values, rc.values, rtol=1e-9, atol=1e-12)
    for a, b in zip(ng[-5:], nc[-5:]):
        np.testing.assert_allclose(a.values, b.values, rtol=1e-9, atol=1e-15)


def test_specific_returns_lazy_list_semantics(monkeypatch):
    """reg_by_time's specific returns are built lazily but behave as the reference's list of
    one-row DataFrames (len / index / negative index / slice / iteration / pd.concat)."""
    monkeypatch.setenv("MFA_DEVICE", "cpu")
    df = toy_frame(T=12, N=20, P=3, Q=2, seed=5)
    with contextlib.redirect_stdout(io.StringIO()):
        m = mfm.MFM(df, 3, 2)
        f, e, r2 = m.reg_by_time()
    assert len(e) == 12 and all(x is None for x in e._items)
    first = e[0]
    assert first.shape[0] == 1 and first.index[0] == f.index[0] and e[0] is first
    assert e[-1].index[0] == f.index[-1]
    assert [x.index[0] for x in e[2:5]] == list(f.index[2:5])
    cat = pd.concat(list(e))
    assert cat.shape[0] == 12
    dense = e.dense()
    for t in (0, 7, 11):
        row = e[t].iloc[0]
        np.testing.assert_array_equal(row.values, dense.loc[e[t].index[0], row.index].values)
    e.append(e[0])
    assert len(e) == 13
    with pytest.raises(IndexError):
        e[20]
