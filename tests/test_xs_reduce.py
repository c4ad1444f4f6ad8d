"""Post-processing reductions vs the reference's pandas/statsmodels code and HIP vs CPU."""
import numpy as np
import pandas as pd
import pytest
import torch

from llm_driven_multi_factor_model_amd.ops import xs_reduce as R


def _panel(D=6, N=120, seed=0, nan_frac=0.1):
    g = torch.Generator().manual_seed(seed)
    x = torch.randn(D, N, generator=g) * 2 + 1
    x[torch.rand(D, N, generator=g) < nan_frac] = float("nan")
    x[0, :3] = torch.tensor([50.0, -40.0, 30.0])  # outliers
    x[D - 1, 1:] = float("nan")                    # single valid value -> no clipping
    return x


def _long(cols: dict):
    D, N = next(iter(cols.values())).shape
    data = {"trade_date": np.repeat(np.arange(D), N), "ts_code": np.tile(np.arange(N), D)}
    for k, v in cols.items():
        data[k] = v.double().numpy().reshape(-1)
    return pd.DataFrame(data)


@pytest.mark.reference
def test_winsorize_matches_reference(ref, capsys):
    x = _panel()
    df = ref.post_processing.winsorize_factors(_long({"a": x}), ["a"], n_std=2.5)
    exp = df["a"].values.reshape(x.shape)
    np.testing.assert_allclose(R.winsorize(x).double().numpy(), exp, rtol=1e-6, atol=1e-6, equal_nan=True)


@pytest.mark.reference
def test_composite_matches_reference(ref, capsys):
    a, b, c = _panel(seed=1), _panel(seed=2), _panel(seed=3)
    cfg = {"v": {"components": ["a", "b", "c"], "weights": [0.7, 0.15, 0.15]}}
    df = ref.post_processing.calculate_composite_factors(_long({"a": a, "b": b, "c": c}), cfg)
    out = R.composite([a, b, c], [0.7, 0.15, 0.15])
    np.testing.assert_allclose(out.double().numpy(), df["v"].values.reshape(a.shape), rtol=1e-6, equal_nan=True)


@pytest.mark.reference
def test_orthogonalize_matches_reference(ref, capsys):
    y, b, s = _panel(seed=4), _panel(seed=5), _panel(seed=6)
    y[2, :100] = float("nan")  # date with too few rows -> NaN
    df = ref.post_processing.orthogonalize_factors(_long({"y": y, "b": b, "s": s}), {"y": ["b", "s"]})
    out = R.ols_resid(y, [b, s])
    np.testing.assert_allclose(out.double().numpy(), df["y"].values.reshape(y.shape), rtol=1e-4, atol=1e-5,
                               equal_nan=True)


@pytest.mark.reference
def test_bayes_shrink_matches_reference(ref):
    g = torch.Generator().manual_seed(7)
    vol = torch.rand(300, generator=g) * 0.05 + 0.01
    cap = torch.exp(torch.randn(300, generator=g) * 1.3 + 10)
    exp = ref.utils.bayes_shrink(vol.double().numpy(), cap.double().numpy(), ngroup=10, q=1)
    out = R.bayes_shrink(vol, cap, 10, 1.0)
    np.testing.assert_allclose(out.double().numpy(), exp, rtol=1e-5)


@pytest.mark.reference
def test_style_norm_matches_reference(ref):
    g = torch.Generator().manual_seed(8)
    X = torch.randn(2, 4, 50, generator=g)
    cap = torch.exp(torch.randn(2, 50, generator=g))
    Z, mu, sig = R.style_norm(X, cap)
    for d in range(2):
        exp = ref.CrossSection.style_factor_norm(X[d].T.double().numpy(), cap[d].double().numpy())
        np.testing.assert_allclose(Z[d].T.double().numpy(), exp, rtol=1e-5, atol=1e-6)


@pytest.mark.gpu
def test_hip_reductions_match_cpu(cuda):
    x, y, b, s = _panel(D=9, N=1000, seed=10), _panel(D=9, N=1000, seed=11), _panel(D=9, N=1000, seed=12), \
        _panel(D=9, N=1000, seed=13)
    torch.testing.assert_close(R.winsorize(x.to(cuda)).cpu(), R.winsorize(x), rtol=1e-6, atol=1e-6, equal_nan=True)
    torch.testing.assert_close(R.composite([x.to(cuda), y.to(cuda)], [0.5, 0.5]).cpu(), R.composite([x, y], [0.5, 0.5]),
                               equal_nan=True)
    torch.testing.assert_close(R.ols_resid(y.to(cuda), [b.to(cuda), s.to(cuda)]).cpu(), R.ols_resid(y, [b, s]),
                               rtol=1e-4, atol=1e-5, equal_nan=True)
    torch.testing.assert_close(R.ols_resid(y.to(cuda), [b.to(cuda)], min_rows=2, sign=-1).cpu(),
                               R.ols_resid(y, [b], min_rows=2, sign=-1), rtol=1e-4, atol=1e-5, equal_nan=True)
    X = torch.randn(5, 10, 2000)
    cap = torch.exp(torch.randn(5, 2000))
    Zg, mug, sg = R.style_norm(X.to(cuda), cap.to(cuda))
    Zc, muc, sc = R.style_norm(X, cap)
    torch.testing.assert_close(Zg.cpu(), Zc, rtol=1e-5, atol=1e-5)
    vol = torch.rand(4, 3000) * 0.05 + 0.01
    cap2 = torch.exp(torch.randn(4, 3000))
    torch.testing.assert_close(R.bayes_shrink(vol.to(cuda), cap2.to(cuda)).cpu(),
                               R.bayes_shrink(vol, cap2), rtol=1e-5, atol=1e-6)


def test_bayes_shrink_all_nan_date_cpu():
    """A date without any finite (vol, cap) pair (the first date of a resumed panel: its
    trailing-vol halo is all NaN) stays a NaN row instead of failing np.quantile."""
    vol = torch.rand(3, 200) * 0.05 + 0.01
    cap = torch.exp(torch.randn(3, 200))
    vol[0] = float("nan")
    out, g = R.bayes_shrink(vol, cap, 10, 1.0, return_groups=True)
    assert torch.isnan(out[0]).all() and (g[0] == -1).all()
    torch.testing.assert_close(out[1:], R.bayes_shrink(vol[1:], cap[1:], 10, 1.0))


@pytest.mark.gpu
def test_hip_bayes_shrink_all_nan_date(cuda):
    vol = torch.rand(3, 500) * 0.05 + 0.01
    cap = torch.exp(torch.randn(3, 500))
    vol[0] = float("nan")
    got = R.bayes_shrink(vol.to(cuda), cap.to(cuda)).cpu()
    assert torch.isnan(got[0]).all()
    torch.testing.assert_close(got[1:], R.bayes_shrink(vol, cap)[1:], rtol=1e-5, atol=1e-6)


@pytest.mark.gpu
@pytest.mark.parametrize("dtype", [torch.float32, torch.float64])
def test_grid_map_transpose_equals_index_scatter(cuda, dtype):
    """GridMap (csrc/gather.hip, LDS-tiled rows <-> grid transpose): on ragged (stock, date)
    rows -- stocks with gaps, a stock with one row, grid edges not multiples of 64 -- the
    scatter equals an index scatter bitwise (NaN in empty cells), a strided layout (column
    stride / date stride of a [D, Q, N] panel) lands every value where the index formula says,
    and the gather inverts the scatter."""
    from llm_driven_multi_factor_model_amd.ops import xs_reduce as XR
    g = torch.Generator().manual_seed(5)
    Dg, Ng, C = 203, 131, 3
    keep = torch.rand(Ng, Dg, generator=g) < 0.8
    keep[7] = False
    keep[7, 100] = True
    sid, did = torch.nonzero(keep, as_tuple=True)          # sorted by (stock, date)
    R = sid.numel()
    X = torch.randn(C, R, generator=g, dtype=torch.float64).to(dtype)
    gm = XR.GridMap(sid.to(cuda), did.to(cuda), Dg, Ng)
    G = gm.scatter(X.to(cuda))
    ref = torch.full((C, Dg * Ng), float("nan"), dtype=dtype)
    ref[:, did * Ng + sid] = X
    assert torch.equal(G.cpu().nan_to_num(7.0), ref.nan_to_num(7.0))
    assert torch.equal(gm.gather(G, C).cpu(), X)
    Q = C
    P = torch.full((Dg, Q, Ng), float("nan"), dtype=dtype, device=cuda)
    gm.scatter(X.to(cuda), out=P.view(-1), gs=Ng, ds=Q * Ng)
    for q in range(Q):
        assert torch.equal(P[did, q, sid].cpu(), X[q])
    assert int(torch.isfinite(P).sum()) == C * R
    assert torch.equal(gm.gather(P.view(-1), C, gs=Ng, ds=Q * Ng).cpu(), X)


@pytest.mark.gpu
def test_grid_map_duplicate_rows_take_index_path(cuda):
    """the tile kernel covers one row per (stock, date) cell.  A stock with a
    duplicated row inside a fully populated 64-date block (the pandas engine's fall-back input)
    makes the map non-strict: scatter / gather then take the index path, so no row is left out
    of the gather (every row reads its cell) -- identical to the CPU map."""
    from llm_driven_multi_factor_model_amd.ops import xs_reduce as XR
    Dg, Ng = 130, 5
    sid, did = torch.nonzero(torch.ones(Ng, Dg, dtype=torch.bool), as_tuple=True)
    dup = 2 * Dg + 10                                       # stock 2, date 10: full 64-date block
    sid = torch.cat([sid[:dup + 1], sid[dup:dup + 1], sid[dup + 1:]])
    did = torch.cat([did[:dup + 1], did[dup:dup + 1], did[dup + 1:]])
    X = torch.randn(2, sid.numel(), dtype=torch.float32)
    X[:, dup + 1] = X[:, dup]                              # same values: the winner is irrelevant
    gm = XR.GridMap(sid.to(cuda), did.to(cuda), Dg, Ng)
    gc = XR.GridMap(sid, did, Dg, Ng)
    assert not gm.strict and not gc.strict
    G = gm.scatter(X.to(cuda))
    assert torch.equal(G.cpu().nan_to_num(7.0), gc.scatter(X).nan_to_num(7.0))
    assert torch.equal(gm.gather(G, 2).cpu(), X)


def test_factor_pipeline_duplicate_rows_columnar_equals_frame_path():
    """Duplicate (stock, date) rows: the single-process pipeline routes them to the frame path
    (its per-date grids give each row its own column), whichever ``columnar`` says."""
    import contextlib
    import io
    from llm_driven_multi_factor_model_amd.models import factor_engine as FE
    prices, index, sw = FE.synthetic_prices(N=8, T=140, seed=4)
    prices = pd.concat([prices, prices.iloc[[300]]]).reset_index(drop=True)
    with contextlib.redirect_stdout(io.StringIO()):
        a, ia, _ = FE.factor_pipeline(prices, index, sw, device="cpu", columnar=True)
        b, ib, _ = FE.factor_pipeline(prices, index, sw, device="cpu", columnar=False)
    assert len(a) == len(prices)
    pd.testing.assert_frame_equal(a, b)
    pd.testing.assert_frame_equal(ia, ib)
