"""Descriptor engine vs the reference FactorCalculator; HIP rolling kernels vs CPU oracles."""
import contextlib
import io
import warnings

import numpy as np
import pandas as pd
import pytest
import torch

from llm_driven_multi_factor_model_amd.models import factor_engine as FE
from llm_driven_multi_factor_model_amd.ops import rolling as RL

COLS = ["SIZE", "BETA", "HSIGMA", "RSTR", "DASTD", "CMRA", "NLSIZE", "BP", "STOM", "STOQ", "STOA",
        "CETOP", "ETOP", "YOYProfit", "YOYSales", "MLEV", "DTOA", "BLEV"]


@pytest.fixture(scope="module")
def data():
    return FE.synthetic_prices(N=10, T=330, seed=1, suspend_frac=0.03)


@pytest.fixture(scope="module")
def ref_out(ref, data):
    prices, index, _ = data
    warnings.simplefilter("ignore")
    with contextlib.redirect_stdout(io.StringIO()), contextlib.redirect_stderr(io.StringIO()):
        fc = ref.factor_calculator.FactorCalculator(prices.copy(), index.copy())
        return fc.run(FE.FACTORS_TO_RUN)


@pytest.mark.reference
def test_descriptors_match_reference(ref_out, data, monkeypatch):
    prices, index, _ = data
    eng = FE.FactorEngine(prices, index, device="cpu")
    with contextlib.redirect_stdout(io.StringIO()):
        out = eng.run(FE.FACTORS_TO_RUN)
    assert list(out.columns) == list(ref_out.columns)
    assert (out["ts_code"].values == ref_out["ts_code"].values).all()
    assert (out["trade_date"].values == ref_out["trade_date"].values).all()
    for c in ["ret", "circ_mv"] + COLS:
        a, b = out[c].to_numpy(np.float64), ref_out[c].to_numpy(np.float64)
        assert (np.isnan(a) == np.isnan(b)).all(), c
        m = np.isfinite(b)
        np.testing.assert_allclose(a[m], b[m], rtol=2e-4, atol=1e-6, err_msg=c)


@pytest.mark.reference
def test_post_processing_pipeline_matches_reference(ref, ref_out, data):
    pp = ref.post_processing
    cols = [c for c in ref_out.columns if c not in ("ts_code", "trade_date")]
    with contextlib.redirect_stdout(io.StringIO()):
        rw = pp.winsorize_factors(ref_out, cols)
        from llm_driven_multi_factor_model_amd.utils.config import FactorConfig
        cfg = FactorConfig()
        rc = pp.calculate_composite_factors(rw, cfg.composite)
        ro = pp.orthogonalize_factors(rc, cfg.ortho)
    w = FE.winsorize_frame(ref_out, cols, device="cpu")
    c = FE.composite_frame(w, cfg.composite, device="cpu")
    o = FE.orthogonalize_frame(c, cfg.ortho, device="cpu")
    for col in cols + list(cfg.composite):
        np.testing.assert_allclose(o[col].to_numpy(np.float64), ro[col].to_numpy(np.float64), rtol=5e-4,
                                   atol=5e-5, equal_nan=True, err_msg=col)


@pytest.mark.reference
def test_multivalued_statement_multiplies_rows_like_reference(ref, data):
    """One (stock, end_date) statement with two cash-flow values: the reference's TTM left merge
    (factor_calculator.py:403-410) multiplies those rows and run() carries the extra rows into
    every column (:561-566); the engine reproduces the frame row for row."""
    prices, index, _ = data
    p = prices.copy()
    r = int(np.flatnonzero((p["ts_code"] == p["ts_code"].iloc[0]).to_numpy())[200])
    p.iloc[r, p.columns.get_loc("n_cashflow_act")] *= 1.5
    warnings.simplefilter("ignore")
    with contextlib.redirect_stdout(io.StringIO()), contextlib.redirect_stderr(io.StringIO()):
        want = ref.factor_calculator.FactorCalculator(p.copy(), index.copy()).run(FE.FACTORS_TO_RUN)
        got = FE.FactorEngine(p, index, device="cpu").run(FE.FACTORS_TO_RUN)
    assert len(want) > len(p) and len(got) == len(want)
    assert (got["ts_code"].values == want["ts_code"].values).all()
    assert (got["trade_date"].values == want["trade_date"].values).all()
    for c in ["ret", "CETOP", "ETOP", "BETA", "RSTR", "STOM"]:
        a, b = got[c].to_numpy(np.float64), want[c].to_numpy(np.float64)
        assert (np.isnan(a) == np.isnan(b)).all(), c
        m = np.isfinite(b)
        np.testing.assert_allclose(a[m], b[m], rtol=2e-4, atol=1e-6, err_msg=c)


def test_barra_export_schema(data):
    prices, index, sw = data
    with contextlib.redirect_stdout(io.StringIO()):
        final, info, t = FE.factor_pipeline(prices, index, sw, device="cpu")
    assert list(final.columns) == FE.BARRA_OUTPUT_COLUMNS
    assert list(info.columns) == ["code", "industry_names", "start_date"]
    # t+1 return alignment: ret on the last row of each stock is NaN
    last = final.groupby("stocknames").tail(1)
    assert last["ret"].isna().all()


@pytest.mark.gpu
def test_hip_rolling_kernels_match_cpu(cuda):
    prices, index, _ = FE.synthetic_prices(N=24, T=600, seed=3, suspend_frac=0.05)
    cpu = FE.FactorEngine(prices, index, device="cpu")
    gpu = FE.FactorEngine(prices, index, device=cuda)
    with contextlib.redirect_stdout(io.StringIO()):
        a = cpu.compute(FE.FACTORS_TO_RUN)
        b = gpu.compute(FE.FACTORS_TO_RUN)
    for k in a:
        torch.testing.assert_close(b[k].cpu().float(), a[k].float(), rtol=2e-5, atol=1e-6, equal_nan=True,
                                   msg=k)
    lr = cpu.cols["log_ret"]
    torch.testing.assert_close(RL.cmra(lr.to(cuda), cpu.seg_lo.to(cuda), partial=True).cpu(),
                               RL.cmra(lr, cpu.seg_lo, partial=True), rtol=1e-5, atol=1e-6, equal_nan=True)


@pytest.mark.gpu
def test_hip_sliding_window_kernels_match_direct(cuda):
    """Segment-anchored kernels == the direct per-row kernels (suspensions, stock edges)."""
    g = torch.Generator().manual_seed(4)
    N, T = 37, 700                      # T not a multiple of the 64-row chunk
    R = N * T
    mkt = torch.randn(T, generator=g) * 0.012
    ret = (mkt[None, :] * 1.1 + torch.randn(N, T, generator=g) * 0.02).reshape(-1).float()
    ret[torch.rand(R, generator=g) < 0.05] = float("nan")
    mret = mkt[None, :].expand(N, T).reshape(-1).contiguous().float()
    lr = torch.log1p(ret)
    turn = torch.rand(R, generator=g) * 5
    turn[torch.rand(R, generator=g) < 0.3] = 0.0
    lens = torch.randint(50, T, (N,), generator=g)   # ragged stock lengths via NaN-free cut
    stock = torch.arange(N, dtype=torch.int32).repeat_interleave(T)
    seg = RL.seg_lo_from_codes(stock).to(cuda)
    args = [t.to(cuda) for t in (ret, mret, lr, turn)]
    r_, m_, l_, t_ = args
    fns = {
        "beta": lambda: RL.beta_hsigma(r_, m_, seg, 252, 63.0, 42),
        "rstr": lambda: RL.rstr(l_, seg, 504, 21, 126.0, 42),
        "dastd": lambda: RL.dastd(r_, m_, seg, 252, 42.0, 42),
        "stom": lambda: RL.rolling_sum(t_, seg, 21, 15, 0.01, log=True),
        "stoa": lambda: RL.rolling_sum(t_, seg, 252, 126, 0.01, log=True),
        "cmra": lambda: RL.cmra(l_, seg, 252),
        "cmra_partial": lambda: RL.cmra(l_, seg, 252, partial=True),
    }
    with RL.direct_kernels():
        direct = {k: f() for k, f in fns.items()}
    scan = {k: f() for k, f in fns.items()}
    del lens
    for k in fns:
        a = direct[k] if isinstance(direct[k], tuple) else (direct[k],)
        b = scan[k] if isinstance(scan[k], tuple) else (scan[k],)
        for x, y in zip(a, b):
            torch.testing.assert_close(y.cpu(), x.cpu(), rtol=2e-5, atol=2e-7, equal_nan=True, msg=k)


_FIXTURE = __import__("pathlib").Path(__file__).parent / "fixtures" / "ref_descriptors_n50_t800_seed5.npz"


def _check_against_fixture(out):
    """Descriptors vs the reference FactorCalculator's output for synthetic_prices(N=50, T=800,
    seed=5, suspend_frac=0.03), computed once by running the reference source and stored as
    npz (tests/fixtures; loaded with allow_pickle=False)."""
    fx = np.load(_FIXTURE, allow_pickle=False)
    assert (out["ts_code"].astype(str).to_numpy() == fx["ts_code"]).all()
    assert (out["trade_date"].astype(str).to_numpy() == fx["trade_date"]).all()
    for c in ["ret", "circ_mv"] + COLS:
        a, b = out[c].to_numpy(np.float64), fx["col_" + c]
        assert (np.isnan(a) == np.isnan(b)).all(), c
        m = np.isfinite(b)
        np.testing.assert_allclose(a[m], b[m], rtol=2e-4, atol=1e-6, err_msg=c)


def test_descriptors_match_reference_fixture_n50_t800():
    prices, index, _ = FE.synthetic_prices(N=50, T=800, seed=5, suspend_frac=0.03)
    eng = FE.FactorEngine(prices, index, device="cpu")
    with contextlib.redirect_stdout(io.StringIO()):
        _check_against_fixture(eng.run(FE.FACTORS_TO_RUN))


@pytest.mark.gpu
def test_hip_descriptors_match_reference_fixture_n50_t800(cuda):
    prices, index, _ = FE.synthetic_prices(N=50, T=800, seed=5, suspend_frac=0.03)
    eng = FE.FactorEngine(prices, index, device=cuda)
    with contextlib.redirect_stdout(io.StringIO()):
        _check_against_fixture(eng.run(FE.FACTORS_TO_RUN))


@pytest.mark.gpu
def test_hip_rolling_kernels_large_ragged_panel(cuda):
    """500 stocks with ragged histories of 300..9000 rows (2.3 M flat rows; many stocks longer
    than a 2048-row tile, stock starts anywhere inside tiles), 2 % suspensions: the default
    (segment-anchored) kernels == the direct per-row kernels, including the three turnover sums
    of one window_sums pass."""
    g = torch.Generator().manual_seed(11)
    N = 500
    lens = torch.randint(300, 9000, (N,), generator=g)
    R = int(lens.sum())
    stock = torch.repeat_interleave(torch.arange(N, dtype=torch.int32), lens)
    day = torch.cat([torch.arange(int(n)) for n in lens])
    T = int(lens.max())
    mkt = torch.randn(T, generator=g) * 0.012
    ret = (mkt[day] * 1.1 + torch.randn(R, generator=g) * 0.02).float()
    ret[torch.rand(R, generator=g) < 0.02] = float("nan")
    mret = mkt[day].float().contiguous()
    lr = torch.log1p(ret)
    turn = torch.rand(R, generator=g) * 5
    turn[torch.rand(R, generator=g) < 0.2] = 0.0
    seg = RL.seg_lo_from_codes(stock).to(cuda)
    r_, m_, l_, t_ = (x.to(cuda) for x in (ret, mret, lr, turn))
    fns = {
        "beta": lambda: RL.beta_hsigma(r_, m_, seg, 252, 63.0, 42),
        "dastd": lambda: RL.dastd(r_, m_, seg, 252, 42.0, 42),
        "beta_short": lambda: RL.beta_hsigma(r_, m_, seg, 20, 5.0, 10),
        "dastd_short": lambda: RL.dastd(r_, m_, seg, 17, 7.0, 5),
        "rstr": lambda: RL.rstr(l_, seg, 504, 21, 126.0, 42),
        "stom": lambda: RL.rolling_sum(t_, seg, 21, 15, 0.01, log=True),
        "stoa": lambda: RL.rolling_sum(t_, seg, 252, 126, 0.01, log=True),
        "cmra": lambda: RL.cmra(l_, seg, 252),
        "cmra_partial": lambda: RL.cmra(l_, seg, 252, partial=True),
        "sto3": lambda: tuple(RL.window_sums(t_, seg, [(21, 15), (63, 42), (252, 126)], 0.01, log=True)),
    }
    with RL.direct_kernels():
        direct = {k: f() for k, f in fns.items()}
        direct["sto3"] = (direct["stom"], RL.rolling_sum(t_, seg, 63, 42, 0.01, log=True), direct["stoa"])
    fast = {k: f() for k, f in fns.items()}
    for k in fns:
        a = direct[k] if isinstance(direct[k], tuple) else (direct[k],)
        b = fast[k] if isinstance(fast[k], tuple) else (fast[k],)
        for x, y in zip(a, b):
            # full-window CMRA needs 252 NaN-free rows: rare at 2 % suspensions
            assert int(torch.isfinite(x).sum()) > (1000 if k == "cmra" else R // 2), k
            torch.testing.assert_close(y.cpu(), x.cpu(), rtol=2e-5, atol=2e-7, equal_nan=True, msg=k)


def _pipeline_paths_equal(device):
    prices, index, sw = FE.synthetic_prices(N=40, T=420, seed=6, suspend_frac=0.03)
    sw = sw.iloc[1:].reset_index(drop=True)  # one stock without an industry row
    with contextlib.redirect_stdout(io.StringIO()):
        f1, i1, t1 = FE.factor_pipeline(prices, index, sw, device=device)
        f0, i0, _ = FE.factor_pipeline(prices, index, sw, device=device, columnar=False)
    assert "export_s" in t1
    pd.testing.assert_frame_equal(f1, f0.reset_index(drop=True))
    pd.testing.assert_frame_equal(i1, i0)


def test_columnar_pipeline_equals_frame_pipeline():
    """The single-process columnar fast path (device tensors through post-processing, one
    export frame) gives exactly the frame-by-frame pipeline's output frames."""
    _pipeline_paths_equal("cpu")


@pytest.mark.gpu
def test_hip_columnar_pipeline_equals_frame_pipeline(cuda):
    _pipeline_paths_equal(cuda)


def test_barra_export_fast_path_equals_merge_path(data):
    """The index-lookup export (unique industry rows) equals the pandas merge / groupby-shift
    path it replaces, including suspended stocks and a stock missing from the industry table."""
    prices, index, sw = data
    eng = FE.FactorEngine(prices, index, device="cpu")
    raw = eng.run(FE.FACTORS_TO_RUN)
    for table in (sw, sw.iloc[1:].reset_index(drop=True)):
        fast, info_f = FE.barra_export(raw, table)
        slow, info_s = FE.barra_export(raw, table, _merge_path=True)
        pd.testing.assert_frame_equal(fast, slow.reset_index(drop=True), check_dtype=False)
        pd.testing.assert_frame_equal(info_f, info_s)


def test_cetop_ttm_code_path_equals_merge_path():
    """CETOP's statement-row TTM on integer keys equals the drop_duplicates / merge path,
    with missing cash flows and NaT statement dates (no statement yet) in the panel."""
    prices, index, _ = FE.synthetic_prices(N=60, T=400, seed=2, suspend_frac=0.05)
    ed = prices["end_date"].unique()
    prices.loc[prices.end_date.isin(ed[::3]) & (prices.ts_code < "000030"), "n_cashflow_act"] = np.nan
    m = prices.end_date.isin(ed[1::5]) & (prices.ts_code > "600010")
    prices.loc[m, "end_date"] = np.datetime64("NaT")
    prices.loc[m, "n_cashflow_act"] = np.nan
    eng = FE.FactorEngine(prices, index, device="cpu")
    a, b = eng._ttm_by_codes(eng.master), eng._ttm_by_merge(eng.master)
    assert a is not None and int(torch.isfinite(a).sum()) > 1000
    torch.testing.assert_close(a, b, rtol=0, atol=0, equal_nan=True)


def test_cetop_ttm_run_path_equals_merge_path_and_falls_back():
    """O(n) run-start TTM (end_date non-decreasing within each stock after the PIT join) equals
    the merge path; a restatement that moves end_date backwards disables it (fallback)."""
    prices, index, _ = FE.synthetic_prices(N=50, T=400, seed=4, suspend_frac=0.05)
    ed = prices["end_date"].unique()
    prices.loc[prices.end_date.isin(ed[::4]) & (prices.ts_code < "000020"), "n_cashflow_act"] = np.nan
    eng = FE.FactorEngine(prices, index, device="cpu")
    a = eng._ttm_runs(eng.master)
    assert a is not None and int(torch.isfinite(a).sum()) > 1000
    torch.testing.assert_close(a, eng._ttm_by_merge(eng.master), rtol=0, atol=0, equal_nan=True)
    code = prices.ts_code.iloc[0]
    rows = prices.index[prices.ts_code == code]
    prices.loc[rows[-5:], "end_date"] = prices.loc[rows[0], "end_date"]   # backwards restatement
    eng2 = FE.FactorEngine(prices, index, device="cpu")
    assert eng2._ttm_runs(eng2.master) is None
    b = eng2._ttm_by_codes(eng2.master)
    if b is None:
        b = eng2._ttm_by_merge(eng2.master)
    torch.testing.assert_close(b, eng2._ttm_by_merge(eng2.master), rtol=0, atol=0, equal_nan=True)


@pytest.mark.gpu
def test_hip_cmra_rstr_window_edges(cuda):
    """The segment-anchored CMRA and RSTR kernels at the edges of their window ranges (CMRA W =
    65 / 128 / 129 / 200 / 257: just above one 64-row segment, whole segments, the 256-row tile
    halo; RSTR reach W + L - 1 = 512 = its tile halo, W = 1, L = 1, a short half-life; a sum
    window of 513 rows = the 512 reach) == the direct per-row kernels, on ragged stocks with
    NaNs."""
    g = torch.Generator().manual_seed(21)
    lens = torch.randint(30, 3000, (300,), generator=g)
    R = int(lens.sum())
    stock = torch.repeat_interleave(torch.arange(300, dtype=torch.int32), lens)
    lr = (torch.randn(R, generator=g) * 0.02).float()
    lr[torch.rand(R, generator=g) < 0.003] = float("nan")
    seg = RL.seg_lo_from_codes(stock).to(cuda)
    l_ = lr.to(cuda)
    fns = {
        "cmra65": lambda: RL.cmra(l_, seg, 65),
        "cmra128": lambda: RL.cmra(l_, seg, 128),
        "cmra129": lambda: RL.cmra(l_, seg, 129),
        "cmra200": lambda: RL.cmra(l_, seg, 200),
        "cmra257": lambda: RL.cmra(l_, seg, 257),
        "rstr_max_reach": lambda: RL.rstr(l_, seg, 512, 21, 126.0, 42),
        "rstr_w1": lambda: RL.rstr(l_, seg, 2, 1, 5.0, 1),
        "rstr_short_hl": lambda: RL.rstr(l_, seg, 100, 3, 2.0, 10),
        "sum513": lambda: RL.rolling_sum(l_.abs(), seg, 513, 10),
        "sum1": lambda: RL.rolling_sum(l_, seg, 1, 1),
    }
    with RL.direct_kernels():
        direct = {k: f() for k, f in fns.items()}
    fast = {k: f() for k, f in fns.items()}
    for k in fns:
        assert int(torch.isfinite(direct[k]).sum()) > R // 4, k
        torch.testing.assert_close(fast[k].cpu(), direct[k].cpu(), rtol=2e-5, atol=2e-7, equal_nan=True, msg=k)


@pytest.mark.gpu
def test_seg_kernels_rank_invariant(cuda):
    """Every segment-anchored descriptor (BETA/HSIGMA, DASTD, RSTR, CMRA, the turnover sums) on
    a ragged panel: a slice of every stock that starts halo_rows() rows (or fewer, at the stock
    start) before its first output row, with the rows' full-history ordinals, reproduces the
    full-panel outputs BIT FOR BIT -- a shard boundary anywhere relative to the segments."""
    from llm_driven_multi_factor_model_amd.utils.config import FactorConfig
    g = torch.Generator().manual_seed(21)
    lens = torch.randint(300, 2600, (60,), generator=g)
    lens[:4] = torch.tensor([1, 40, 700, 2049])
    R = int(lens.sum())
    stock = torch.repeat_interleave(torch.arange(lens.numel(), dtype=torch.int32), lens)
    ret = (torch.randn(R, generator=g) * 0.02).float()
    ret[torch.rand(R, generator=g) < 0.002] = float("nan")
    mret = (torch.randn(R, generator=g) * 0.012).float()
    lr = torch.log1p(ret)
    turn = torch.rand(R, generator=g) * 5
    turn[torch.rand(R, generator=g) < 0.1] = 0.0
    seg = RL.seg_lo_from_codes(stock).to(cuda)
    r_, m_, l_, t_ = (x.to(cuda) for x in (ret, mret, lr, turn))
    ordv = torch.arange(R, device=cuda, dtype=torch.int32) - seg

    def run(r, m, lg, tt, sg, ro):
        lay = RL.SegLayout(sg, ro)
        out = [*RL.beta_hsigma(r, m, sg, 252, 63.0, 42, row_ord=lay),
               RL.dastd(r, m, sg, 252, 42.0, 42, row_ord=lay),
               RL.rstr(lg, sg, 504, 21, 126.0, 42, row_ord=lay),
               RL.cmra(lg, sg, 252, row_ord=lay),
               *RL.window_sums(tt, sg, [(21, 15), (63, 42), (252, 126)], 0.01, log=True, row_ord=lay)]
        return out

    full = run(r_, m_, l_, t_, seg, ordv)
    halo = FE.FactorEngine.halo_rows(type("C", (), {"cfg": FactorConfig()})())
    assert halo == 566
    starts = torch.cumsum(lens, 0) - lens
    for trial in range(3):
        keep, own = [], []
        for s_, n_ in zip(starts.tolist(), lens.tolist()):
            o = int(torch.randint(0, n_, (1,), generator=g))
            t0 = max(0, o - halo)
            keep.append(torch.arange(s_ + t0, s_ + n_))
            own.append(torch.arange(s_ + o, s_ + n_))
        keep = torch.cat(keep).to(cuda)
        own = torch.cat(own).to(cuda)
        sseg = RL.seg_lo_from_codes(stock.to(cuda)[keep])
        part = run(r_[keep], m_[keep], l_[keep], t_[keep], sseg, ordv[keep])
        pos = torch.searchsorted(keep, own)   # owned rows inside the slice
        for k, (a, b) in enumerate(zip(full, part)):
            assert int(torch.isfinite(a[own]).sum()) > own.numel() // 4, k
            assert torch.equal(a[own].nan_to_num(7.0), b[pos].nan_to_num(7.0)), (trial, k)


@pytest.mark.gpu
def test_seg_layout_kernels_equal_torch_build(cuda):
    """The GPU segment layout (seg_count / seg_place kernels around one prefix sum) equals the
    tensor-op build: the same Rv, virtual stock starts, output map and NaN-padded series, for
    full histories and for a slice whose rows start mid-history (ordinals not multiples of
    256, one stock with a gap in its ordinals)."""
    g = torch.Generator().manual_seed(3)
    lens = torch.randint(1, 1500, (40,), generator=g)
    lens[:3] = torch.tensor([1, 256, 257])
    R = int(lens.sum())
    stock = torch.repeat_interleave(torch.arange(lens.numel(), dtype=torch.int32), lens)
    seg = RL.seg_lo_from_codes(stock)
    x = torch.randn(R, generator=g)
    y = torch.randn(R, generator=g)
    ordv = torch.arange(R, dtype=torch.int32) - seg
    keep = torch.nonzero((ordv % 7 != 3) | (stock != 5)).flatten()   # stock 5: ordinal gaps
    keep = keep[ordv[keep] >= (stock[keep] % 3) * 300]               # slices start mid-history
    cases = [(seg, None, x, y), (RL.seg_lo_from_codes(stock[keep]), ordv[keep], x[keep], y[keep])]
    for sl, ro, a, b in cases:
        cpu = RL.SegLayout(sl, ro if ro is not None else torch.arange(sl.numel(), dtype=torch.int32) - sl)
        gpu = RL.SegLayout(sl.to(cuda), None if ro is None else ro.to(cuda), series=[a.to(cuda)])
        assert gpu.Rv == cpu.Rv
        assert torch.equal(gpu.seg_v.cpu(), cpu.seg_v) and torch.equal(gpu.omap.cpu(), cpu.omap)
        ag = gpu._virt[next(iter(gpu._virt))][1]
        assert torch.equal(ag.cpu().nan_to_num(7.0), cpu.virt(a).nan_to_num(7.0))
        bg = gpu.virt(b.to(cuda))   # a later series-only pass
        assert torch.equal(bg.cpu().nan_to_num(7.0), cpu.virt(b).nan_to_num(7.0))
