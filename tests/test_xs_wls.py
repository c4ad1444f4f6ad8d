"""Cross-sectional WLS regression: oracle vs reference code, planted recovery, HIP kernel parity."""
import contextlib
import io

import numpy as np
import pandas as pd
import pytest
import torch

from llm_driven_multi_factor_model_amd.models.panel import synthetic_panel
from llm_driven_multi_factor_model_amd.ops import cross_section as X


def ref_date_inputs(panel, d):
    """The reference CrossSection inputs for date d (valid rows, sorted by stock name)."""
    m = panel.valid()[d].numpy()
    Xs = panel.styles[d].numpy().T[m].astype(np.float64)
    base = pd.DataFrame({"date": [str(panel.dates[d])[:10]] * m.sum(),
                         "stocknames": panel.stocks[m],
                         "capital": panel.cap[d].numpy()[m].astype(np.float64),
                         "ret": panel.ret[d].numpy()[m].astype(np.float64)})
    sty = pd.DataFrame(Xs, columns=[f"s{q}" for q in range(panel.Q)])
    if panel.P > 0:
        ind = panel.ind[d].numpy()[m]
        oh = pd.DataFrame(np.eye(panel.P, dtype=np.int64)[ind], columns=[f"i{j}" for j in range(panel.P)])
    else:
        oh = pd.DataFrame()
    return base, sty, oh, m


def run_ref(ref, base, sty, oh):
    with contextlib.redirect_stdout(io.StringIO()):
        cs = ref.CrossSection.CrossSection(base, sty, oh)
        return cs.reg()


@pytest.mark.reference
@pytest.mark.parametrize("P,Q,N", [(5, 3, 60), (0, 4, 40), (12, 10, 300), (31, 10, 500)])
def test_oracle_matches_reference_crosssection(ref, P, Q, N):
    """Unrounded float64 inputs (the reference's precision): f, e, R^2 at 1e-9 or better."""
    panel = synthetic_panel(4, N, P, Q, seed=P * 10 + Q, missing_frac=0.05, dtype=torch.float64)
    res = X.xs_wls_reference(panel.styles, panel.cap, panel.ret, panel.ind, P)
    assert res.resid.dtype == torch.float64
    for d in range(panel.D):
        base, sty, oh, m = ref_date_inputs(panel, d)
        f, e, expo, r2 = run_ref(ref, base, sty, oh)
        np.testing.assert_allclose(res.f[d].numpy(), f, rtol=1e-9, atol=1e-13)
        np.testing.assert_allclose(res.resid[d].numpy()[m], e, rtol=1e-9, atol=1e-13)
        assert abs(res.r2[d].item() - r2) < 1e-12
        assert np.all(np.isnan(res.resid[d].numpy()[~m]))


@pytest.mark.reference
def test_collinear_styles_and_singleton_industry_match_reference_pinv(ref):
    """An exactly duplicated style column (rank-deficient style block) and a one-stock industry:
    the reference's pinv gives the minimum-norm solution (CrossSection.py:76)."""
    panel = _degenerate_panel()
    res = X.xs_wls_reference(panel.styles, panel.cap, panel.ret, panel.ind, panel.P)
    for d in range(panel.D):
        base, sty, oh, m = ref_date_inputs(panel, d)
        f, e, expo, r2 = run_ref(ref, base, sty, oh)
        np.testing.assert_allclose(res.f[d].numpy(), f, rtol=1e-9, atol=1e-12)
        assert abs(res.r2[d].item() - r2) < 1e-10


def _degenerate_panel(D=3, N=400, P=6, Q=4, seed=21, device="cpu"):
    p = synthetic_panel(D, N, P, Q, seed=seed, dtype=torch.float64)
    p.styles[:, 3] = p.styles[:, 1]            # exactly collinear styles
    ind = p.ind.clone()
    ind[:, 0] = 2                              # industry 2 keeps ...
    ind[ind == 2] = 1
    ind[:, 0] = 2                              # ... exactly one stock
    p.ind = ind
    return p.to(device)


@pytest.mark.reference
def test_empty_industry_matches_reference_pinv(ref):
    # an industry (not the last) empty on some dates: reference pinv gives f_j = 0
    panel = synthetic_panel(6, 80, 6, 3, seed=3, empty_industries=2)
    res = X.xs_wls_reference(panel.styles, panel.cap, panel.ret, panel.ind, panel.P)
    hit = 0
    for d in range(panel.D):
        base, sty, oh, m = ref_date_inputs(panel, d)
        if oh.values[:, -1].sum() == 0:
            continue  # last industry empty: reference divides by zero (quirk Q3)
        hit += int((oh.values.sum(0) == 0).any())
        f, e, expo, r2 = run_ref(ref, base, sty, oh)
        np.testing.assert_allclose(res.f[d].numpy(), f, rtol=1e-8, atol=1e-12)
    assert hit > 0


def test_planted_recovery():
    panel, f_true = synthetic_panel(8, 3000, 8, 5, seed=11, noise_vol=0.002, return_truth=True)
    res = X.xs_wls_reference(panel.styles, panel.cap, panel.ret, panel.ind, panel.P)
    err = (res.f - f_true).abs().max().item()
    assert err < 2e-3, err
    # industry-neutral constraint holds exactly: sum_j s_j f_j = 0
    oh = torch.nn.functional.one_hot(panel.ind.long(), panel.P).double()
    s = (oh * panel.cap.double()[..., None]).sum(1)
    assert ((s * res.f[:, 1:1 + panel.P]).sum(1).abs() / s.sum(1)).max() < 1e-14
    assert (res.r2 > 0.5).all()


def test_last_industry_empty_pivot_modes():
    panel = synthetic_panel(2, 50, 4, 2, seed=5)
    ind = panel.ind.clone()
    ind[ind == 3] = 2
    r0 = X.xs_wls_reference(panel.styles, panel.cap, panel.ret, ind, 4, pivot_mode=0)
    r1 = X.xs_wls_reference(panel.styles, panel.cap, panel.ret, ind, 4, pivot_mode=1)
    assert torch.isfinite(r0.f).all() and (r0.f[:, 4].abs() < 1e-12).all()
    assert torch.isnan(r1.f).all() and (r1.status & X.XS_PIVOT_EMPTY).all()
    # pivot choice does not change the constrained solution when both are valid
    r2 = X.xs_wls_reference(panel.styles, panel.cap, panel.ret, panel.ind, 4, pivot_mode=1)
    r3 = X.xs_wls_reference(panel.styles, panel.cap, panel.ret, panel.ind, 4, pivot_mode=0)
    torch.testing.assert_close(r2.f, r3.f, rtol=1e-10, atol=1e-13)


@pytest.mark.gpu
@pytest.mark.parametrize("D,N,P,Q,miss,empty", [
    (7, 300, 31, 10, 0.0, 0),
    (5, 5000, 31, 10, 0.02, 2),
    (9, 777, 12, 3, 0.1, 3),
    (6, 200, 0, 4, 0.05, 0),
    (4, 1000, 28, 16, 0.0, 1),
    (3, 64, 3, 1, 0.0, 0),
    (5, 600, 100, 8, 0.01, 2),
    # Q > 10 runs the 1-wave-per-SIMD register budget (MFA_XS_WPE_BIGQ)
    (4, 1500, 31, 11, 0.01, 1),
    (4, 1500, 31, 12, 0.01, 1),
])
@pytest.mark.parametrize("dtype", [torch.float32, torch.float64])
def test_kernel_matches_oracle(cuda, D, N, P, Q, miss, empty, dtype):
    panel = synthetic_panel(D, N, P, Q, seed=D + N, missing_frac=miss, empty_industries=empty,
                            dtype=dtype)
    ref = X.xs_wls_reference(panel.styles, panel.cap, panel.ret, panel.ind, P)
    g = panel.to(cuda)
    out = X.xs_wls(g.styles, g.cap, g.ret, g.ind, P)
    torch.cuda.synchronize()
    assert out.resid.dtype == dtype
    torch.testing.assert_close(out.f.cpu(), ref.f, rtol=1e-9, atol=1e-12)
    torch.testing.assert_close(out.r2.cpu(), ref.r2, rtol=1e-9, atol=1e-11)
    if dtype == torch.float64:
        torch.testing.assert_close(out.resid.cpu(), ref.resid, rtol=1e-9, atol=1e-13, equal_nan=True)
    else:
        torch.testing.assert_close(out.resid.cpu(), ref.resid, rtol=1e-4, atol=1e-6, equal_nan=True)
    torch.testing.assert_close(out.stats.cpu(), ref.stats, rtol=1e-10, atol=1e-12)


@pytest.mark.gpu
def test_device_pinv_refine_matches_oracle(cuda):
    """Near-singular dates (duplicated style, singleton industry) are re-solved on the device
    by the eigen pseudo-inverse pass: f matches the pinv oracle (== reference pinv, see
    test_collinear_styles_and_singleton_industry_match_reference_pinv) to 1e-9, no host sync."""
    p = _degenerate_panel(D=5, N=800, P=8, Q=5, seed=4)
    ref = X.xs_wls_reference(p.styles, p.cap, p.ret, p.ind, p.P)
    g = p.to(cuda)
    out = X.xs_wls(g.styles, g.cap, g.ret, g.ind, p.P)
    torch.cuda.synchronize()
    st = out.status.cpu()
    assert ((st & X.XS_REFINED) != 0).all(), st
    # the collinear styles leave one direction the pinv cuts: PINV_CUT on every date, as in
    # the structured K > 64 refine (same status semantics on both paths); no
    # ZERO_PIVOT (the np.linalg.inv 'Singular matrix' bit): no direction is exactly empty
    assert ((st & X.XS_PINV_CUT) != 0).all(), st
    assert ((st & X.XS_ZERO_PIVOT) == 0).all(), st
    torch.testing.assert_close(out.f.cpu(), ref.f, rtol=1e-9, atol=1e-12)
    torch.testing.assert_close(out.r2.cpu(), ref.r2, rtol=1e-9, atol=1e-12)
    torch.testing.assert_close(out.resid.cpu(), ref.resid, rtol=1e-9, atol=1e-12, equal_nan=True)
    # fp32 storage and the three-kernel path take the same device refinement
    g32 = g.astype(torch.float32)
    o32 = X.xs_wls(g32.styles, g32.cap, g32.ret, g32.ind, p.P)
    ref32 = X.xs_wls_reference(g32.styles.cpu(), g32.cap.cpu(), g32.ret.cpu(), g32.ind.cpu(), p.P)
    torch.testing.assert_close(o32.f.cpu(), ref32.f, rtol=1e-8, atol=1e-11)


def _degenerate_wide(D=4, N=3000, P=123, Q=16, seed=31, empty=(5, 40)):
    """K = 1 + P + Q wide (SW-L2-sized industries): exactly collinear styles, an industry with
    a single stock and exactly-empty industries -> near-singular on every date."""
    p = synthetic_panel(D, N, P, Q, seed=seed, dtype=torch.float64)
    p.styles[:, 3] = p.styles[:, 1]
    ind = p.ind.clone()
    for j in empty:
        ind[ind == j] = (j + 1) % P
    ind[ind == 2] = 1
    ind[:, 0] = 2
    p.ind = ind
    return p


@pytest.mark.gpu
@pytest.mark.parametrize("P,Q", [(100, 8), (123, 16), (128, 11)])
def test_device_pinv_refine_any_k(cuda, P, Q):
    """K > 64 (109 / 140 / 140): the structured device pinv (Schur-complement eigen-solve plus
    the minimum-norm projection) matches the reference pinv; the whole call is graph-capturable,
    i.e. it has no host synchronisation (.cpu(), nonzero, ...)."""
    p = _degenerate_wide(P=P, Q=Q)
    ref = X.xs_wls_reference(p.styles, p.cap, p.ret, p.ind, p.P)
    g = p.to(cuda)
    out = X.xs_wls(g.styles, g.cap, g.ret, g.ind, p.P)
    torch.cuda.synchronize()
    st = out.status.cpu()
    assert ((st & X.XS_REFINED) != 0).all(), st
    assert ((st & X.XS_PINV_CUT) != 0).all(), st
    torch.testing.assert_close(out.f.cpu(), ref.f, rtol=1e-9, atol=1e-12)
    torch.testing.assert_close(out.r2.cpu(), ref.r2, rtol=1e-9, atol=1e-12)
    torch.testing.assert_close(out.resid.cpu(), ref.resid, rtol=1e-9, atol=1e-12, equal_nan=True)
    # no host sync anywhere in the refine path: capture it in a HIP graph and replay
    ws = X.xs_wls_workspace(p.D, p.P, p.Q, cuda, p.N)
    o2 = X.xs_wls(g.styles, g.cap, g.ret, g.ind, p.P, workspace=ws)
    torch.cuda.synchronize()
    graph = torch.cuda.CUDAGraph()
    with torch.cuda.graph(graph):
        X.xs_wls(g.styles, g.cap, g.ret, g.ind, p.P, out=o2, workspace=ws)
    o2.f.zero_()
    graph.replay()
    torch.cuda.synchronize()
    torch.testing.assert_close(o2.f.cpu(), ref.f, rtol=1e-9, atol=1e-12)


@pytest.mark.gpu
@pytest.mark.parametrize("P,Q", [(6, 4), (123, 16)])
def test_stock_sharded_device_refine(cuda, P, Q):
    """Stock-sharded (TP) path: near-singular dates are re-solved on the device from the
    all-reduced moments before the residual pass (no host sync: graph-capturable)."""
    from llm_driven_multi_factor_model_amd.ops import xs_sharded as S
    p = _degenerate_wide(P=P, Q=Q, empty=(5,) if P > 5 else ())
    ref = X.xs_wls_reference(p.styles, p.cap, p.ret, p.ind, p.P)
    g = p.to(cuda)
    out = S.xs_wls_stock_sharded(g.styles, g.cap, g.ret, g.ind, p.P)
    torch.cuda.synchronize()
    assert ((out.status.cpu() & X.XS_REFINED) != 0).all()
    assert ((out.status.cpu() & X.XS_PINV_CUT) != 0).all()
    torch.testing.assert_close(out.f.cpu(), ref.f, rtol=1e-9, atol=1e-12)
    torch.testing.assert_close(out.r2.cpu(), ref.r2, rtol=1e-9, atol=1e-12)
    torch.testing.assert_close(out.resid.cpu(), ref.resid, rtol=1e-9, atol=1e-12, equal_nan=True)
    graph = torch.cuda.CUDAGraph()
    with torch.cuda.graph(graph):
        S.xs_wls_stock_sharded(g.styles, g.cap, g.ret, g.ind, p.P)
    graph.replay()
    torch.cuda.synchronize()


@pytest.mark.gpu
def test_device_pinv_refine_more_dates_than_grid(cuda):
    """Every one of 1100 dates flagged near-singular: the refine pass (one workgroup per date,
    ``xs_refine_kernel`` launched with dim3(D)) re-solves dates 0, 511, 512, 1023, 1024 and 1099
    like the pinv oracle."""
    p = _degenerate_panel(D=1100, N=200, P=6, Q=4, seed=9)
    g = p.to(cuda)
    out = X.xs_wls(g.styles, g.cap, g.ret, g.ind, p.P)
    torch.cuda.synchronize()
    assert ((out.status.cpu() & X.XS_REFINED) != 0).all()
    idx = [0, 511, 512, 1023, 1024, 1099]
    ref = X.xs_wls_reference(p.styles[idx], p.cap[idx], p.ret[idx], p.ind[idx], p.P)
    torch.testing.assert_close(out.f.cpu()[idx], ref.f, rtol=1e-9, atol=1e-12)
    torch.testing.assert_close(out.r2.cpu()[idx], ref.r2, rtol=1e-9, atol=1e-12)
    torch.testing.assert_close(out.resid.cpu()[idx], ref.resid, rtol=1e-9, atol=1e-12, equal_nan=True)


@pytest.mark.gpu
def test_kernel_reference_pivot_and_determinism(cuda):
    panel = synthetic_panel(16, 2000, 31, 10, seed=1, missing_frac=0.01).to(cuda)
    ind = panel.ind.clone()
    ind[3][ind[3] == 30] = 29  # last industry empty on date 3
    a = X.xs_wls(panel.styles, panel.cap, panel.ret, ind, 31, pivot_mode=1)
    assert torch.isnan(a.f[3]).all() and int(a.status[3]) & X.XS_PIVOT_EMPTY
    b = X.xs_wls(panel.styles, panel.cap, panel.ret, ind, 31, pivot_mode=0)
    assert torch.isfinite(b.f).all()
    c = X.xs_wls(panel.styles, panel.cap, panel.ret, ind, 31, pivot_mode=0)
    torch.cuda.synchronize()
    # LDS fp64 atomics are order-dependent: results agree to rounding, not bitwise
    torch.testing.assert_close(b.f, c.f, rtol=1e-12, atol=1e-15)


@pytest.mark.gpu
def test_deterministic_kernel_is_bitwise_reproducible(cuda):
    """run twice, compare bitwise.  The deterministic variant gives each LDS
    segment replica to one wave and sums wave partials in order; the default path agrees with
    it to rounding."""
    panel = synthetic_panel(64, 3000, 31, 10, seed=9, missing_frac=0.02, empty_industries=2).to(cuda)
    runs = [X.xs_wls(panel.styles, panel.cap, panel.ret, panel.ind, 31, deterministic=True)
            for _ in range(3)]
    torch.cuda.synchronize()
    for r in runs[1:]:
        assert torch.equal(r.f, runs[0].f)
        assert torch.equal(r.r2, runs[0].r2)
        assert torch.equal(r.resid.nan_to_num(7.0), runs[0].resid.nan_to_num(7.0))
        assert torch.equal(r.stats, runs[0].stats) and torch.equal(r.status, runs[0].status)
    fast = X.xs_wls(panel.styles, panel.cap, panel.ret, panel.ind, 31)
    torch.testing.assert_close(runs[0].f, fast.f, rtol=1e-12, atol=1e-15)
    ref = X.xs_wls_reference(panel.styles.cpu(), panel.cap.cpu(), panel.ret.cpu(), panel.ind.cpu(), 31)
    torch.testing.assert_close(runs[0].f.cpu(), ref.f, rtol=1e-8, atol=1e-11)


@pytest.mark.gpu
@pytest.mark.parametrize("dtype", [torch.float32, torch.float64])
@pytest.mark.parametrize("S,D,N,P,Q,empty", [(2, 9, 1000, 31, 10, 1), (5, 6, 5000, 31, 10, 2),
                                             (8, 4, 2048, 12, 3, 0), (3, 5, 520, 0, 4, 0),
                                             (7, 3, 4000, 28, 16, 1)])
def test_chunked_path_matches_oracle(cuda, ab_lib, dtype, S, D, N, P, Q, empty):
    """Strong-scaling path: each date split into S stock chunks (partial moments combined in
    chunk order -> one solve -> chunked residuals -> R^2 combine) == the float64 oracle."""
    from llm_driven_multi_factor_model_amd import _native
    panel = synthetic_panel(D, N, P, Q, seed=S * 7 + D, missing_frac=0.02, empty_industries=empty,
                            dtype=dtype)
    ref = X.xs_wls_reference(panel.styles, panel.cap, panel.ret, panel.ind, P)
    g = panel.to(cuda)
    lib = _native.lib()
    lib.mfa_xs_set_chunks(S)
    try:
        assert _native.query("mfa_xs_chunks", D, N) > 1
        out = X.xs_wls(g.styles, g.cap, g.ret, g.ind, P)
        det = [X.xs_wls(g.styles, g.cap, g.ret, g.ind, P, deterministic=True) for _ in range(2)]
        torch.cuda.synchronize()
    finally:
        lib.mfa_xs_set_chunks(0)
    torch.testing.assert_close(out.f.cpu(), ref.f, rtol=1e-9, atol=1e-12)
    torch.testing.assert_close(out.r2.cpu(), ref.r2, rtol=1e-9, atol=1e-11)
    tol = dict(rtol=1e-9, atol=1e-13) if dtype == torch.float64 else dict(rtol=1e-4, atol=1e-6)
    torch.testing.assert_close(out.resid.cpu(), ref.resid, equal_nan=True, **tol)
    torch.testing.assert_close(out.stats.cpu(), ref.stats, rtol=1e-10, atol=1e-12)
    assert torch.equal(det[0].f, det[1].f) and torch.equal(det[0].r2, det[1].r2)
    torch.testing.assert_close(det[0].f.cpu(), ref.f, rtol=1e-9, atol=1e-12)


@pytest.mark.gpu
@pytest.mark.parametrize("dtype", [torch.float32, torch.float64])
@pytest.mark.parametrize("C,D,N,P,Q,empty,lag", [(2, 9, 1000, 31, 10, 1, 1),
                                                 (4, 37, 5000, 31, 10, 2, 1),
                                                 (8, 4, 4096, 12, 3, 0, 2), (3, 5, 1544, 0, 4, 0, 1),
                                                 (7, 3, 4000, 28, 16, 1, 3),
                                                 (4, 300, 5000, 31, 10, 1, 2),
                                                 (16, 61, 5000, 31, 10, 1, 1)])
def test_team_path_matches_oracle(cuda, ab_lib, dtype, C, D, N, P, Q, empty, lag):
    """Pipelined team kernel (persistent grid): C chunks per date, partial moments published
    and solved by the date's last arriver, each chunk's residual pass `lag` tickets later by
    the workgroup that streamed it == the float64 oracle; deterministic mode is bitwise
    reproducible."""
    from llm_driven_multi_factor_model_amd import _native
    panel = synthetic_panel(D, N, P, Q, seed=C * 11 + D, missing_frac=0.02,
                            empty_industries=empty, dtype=dtype)
    ref = X.xs_wls_reference(panel.styles, panel.cap, panel.ret, panel.ind, P)
    g = panel.to(cuda)
    lib = _native.lib()
    lib.mfa_xs_set_coop(C)
    lib.mfa_xs_set_pipe(lag, 0)
    try:
        assert _native.query("mfa_xs_coop_chunks", D, N) == C
        out = X.xs_wls(g.styles, g.cap, g.ret, g.ind, P)
        det = [X.xs_wls(g.styles, g.cap, g.ret, g.ind, P, deterministic=True) for _ in range(2)]
        torch.cuda.synchronize()
    finally:
        lib.mfa_xs_set_coop(0)
        lib.mfa_xs_set_pipe(1, 0)
    assert not bool((out.status & 64).any()), "team wait timed out"
    torch.testing.assert_close(out.f.cpu(), ref.f, rtol=1e-9, atol=1e-12)
    torch.testing.assert_close(out.r2.cpu(), ref.r2, rtol=1e-9, atol=1e-11)
    tol = dict(rtol=1e-9, atol=1e-13) if dtype == torch.float64 else dict(rtol=1e-4, atol=1e-6)
    torch.testing.assert_close(out.resid.cpu(), ref.resid, equal_nan=True, **tol)
    torch.testing.assert_close(out.stats.cpu(), ref.stats, rtol=1e-10, atol=1e-12)
    assert torch.equal(det[0].f, det[1].f) and torch.equal(det[0].r2, det[1].r2)
    assert torch.equal(det[0].resid.nan_to_num(7.0), det[1].resid.nan_to_num(7.0))
    torch.testing.assert_close(det[0].f.cpu(), ref.f, rtol=1e-9, atol=1e-12)


@pytest.mark.gpu
def test_team_path_refines_singular_dates(cuda, ab_lib):
    """A date with an exactly collinear style pair: the team kernel flags it and the device
    pinv pass (reading the team's partial-moment rows in chunk order) matches numpy's pinv."""
    from llm_driven_multi_factor_model_amd import _native
    p = synthetic_panel(6, 3000, 31, 10, seed=3, missing_frac=0.01, dtype=torch.float64)
    p.styles[2, 4] = 2.0 * p.styles[2, 1]
    ref = X.xs_wls_reference(p.styles, p.cap, p.ret, p.ind, 31)
    g = p.to(cuda)
    lib = _native.lib()
    lib.mfa_xs_set_coop(4)
    try:
        out = X.xs_wls(g.styles, g.cap, g.ret, g.ind, 31)
        torch.cuda.synchronize()
    finally:
        lib.mfa_xs_set_coop(0)
    assert int(out.status[2]) & 32, "date 2 should be refined on the device"
    torch.testing.assert_close(out.f.cpu(), ref.f, rtol=1e-8, atol=1e-11)
    torch.testing.assert_close(out.resid.cpu(), ref.resid, rtol=1e-8, atol=1e-12, equal_nan=True)


@pytest.mark.gpu
def test_path_selection_and_small_shards(cuda):
    """The fused kernel is the automatic path at every shard size (the chunked path measured
    slower from 315 to 2520 dates); forced chunk counts are honoured and clamped."""
    from llm_driven_multi_factor_model_amd import _native
    assert _native.query("mfa_xs_chunks", 315, 5000) == 1
    assert _native.query("mfa_xs_chunks", 2520, 5000) == 1
    lib = _native.lib()
    if _native.ab_build():
        lib.mfa_xs_set_chunks(4)
        try:
            assert _native.query("mfa_xs_chunks", 315, 5000) == 4
            assert _native.query("mfa_xs_chunks", 315, 600) == 2   # >= 256 stocks per chunk
        finally:
            lib.mfa_xs_set_chunks(0)
    else:  # production library: the chunked / team paths and the A/B modes are not built in
        assert lib.mfa_xs_set_chunks(4) != 0 and lib.mfa_xs_set_coop(2) != 0
        assert lib.mfa_xs_set_mode(30) != 0
        assert _native.query("mfa_xs_chunks", 315, 5000) == 1
    p = synthetic_panel(40, 5000, 31, 10, seed=2, missing_frac=0.01, dtype=torch.float64)
    ref = X.xs_wls_reference(p.styles, p.cap, p.ret, p.ind, 31)
    g = p.to(cuda)
    out = X.xs_wls(g.styles, g.cap, g.ret, g.ind, 31)
    torch.testing.assert_close(out.f.cpu(), ref.f, rtol=1e-9, atol=1e-12)
    torch.testing.assert_close(out.resid.cpu(), ref.resid, rtol=1e-9, atol=1e-13, equal_nan=True)


@pytest.mark.gpu
def test_mfma_moments_ablation_matches_default(cuda, ab_lib):
    """A/B mode: the MFMA-moments fused kernel (modes 10-12) gives the default's results."""
    from llm_driven_multi_factor_model_amd import _native
    lib = _native.lib()
    for dtype in (torch.float32, torch.float64):
        p = synthetic_panel(12, 3000, 31, 10, seed=5, missing_frac=0.02, empty_industries=1,
                            dtype=dtype).to(cuda)
        base = X.xs_wls(p.styles, p.cap, p.ret, p.ind, 31)
        for mode in (10, 11, 12):
            lib.mfa_xs_set_mode(mode)
            try:
                o = X.xs_wls(p.styles, p.cap, p.ret, p.ind, 31)
                torch.cuda.synchronize()
            finally:
                lib.mfa_xs_set_mode(0)
            torch.testing.assert_close(o.f, base.f, rtol=1e-12, atol=1e-15)
            torch.testing.assert_close(o.r2, base.r2, rtol=1e-12, atol=1e-14)


@pytest.mark.gpu
@pytest.mark.parametrize("dtype", [torch.float32, torch.float64])
def test_plain_load_and_lds_dma_moments_are_bitwise_equal(cuda, ab_lib, dtype):
    """The fused kernel's two moment sources -- plain vector loads (default for fp32 panels and
    fp64 shards up to 512 dates) and the LDS-DMA ring (larger fp64 steps) -- feed the same
    per-wave accumulation in the same order: bitwise-identical f, R^2 and specific returns when
    both run the residual pass with the prefetch during the solve (modes 23 / 7).  The fp64
    plain-load default (mode 20) runs the residual pass without it: same f and specific returns,
    R^2 summed in another stock order."""
    import ctypes as C
    from llm_driven_multi_factor_model_amd import _native
    _native.register("mfa_xs_set_mode", [C.c_int])
    panel = synthetic_panel(37, 5000, 31, 10, seed=77, missing_frac=0.02, empty_industries=1,
                            dtype=dtype).to(cuda)
    lib = _native.lib()
    outs = {}
    try:
        # 23 = plain loads + prefetch, 7 = LDS-DMA ring (+ prefetch), 20 = plain-load default
        for mode in (23, 7, 20):
            lib.mfa_xs_set_mode(mode)
            outs[mode] = X.xs_wls(panel.styles, panel.cap, panel.ret, panel.ind, 31)
        torch.cuda.synchronize()
    finally:
        lib.mfa_xs_set_mode(0)
    a, b, c = outs[23], outs[7], outs[20]
    assert torch.equal(a.f, b.f) and torch.equal(a.r2, b.r2)
    assert torch.equal(a.resid.nan_to_num(7.0), b.resid.nan_to_num(7.0))
    assert torch.equal(c.f, b.f) and torch.equal(c.resid.nan_to_num(7.0), b.resid.nan_to_num(7.0))
    torch.testing.assert_close(c.r2, b.r2, rtol=0, atol=1e-14)


@pytest.mark.gpu
def test_production_moment_sources_agree(cuda):
    """Production library: fp64 shards up to 512 dates take the plain-load moments, longer ones
    the LDS-DMA ring; both run the residual prefetch.  They feed the same per-wave accumulation
    in the same order, so the first 37 dates of a 600-date call equal a 37-date call BITWISE --
    f, the specific returns, R^2, the stats and status: a date-sharded regression is
    rank-invariant whatever block size a rank holds (the 8-rank rehearsal's R^2 differed at
    1e-13 while the plain path summed R^2 without the prefetch)."""
    p = synthetic_panel(600, 5000, 31, 10, seed=78, missing_frac=0.02, empty_industries=1,
                        dtype=torch.float64).to(cuda)
    big = X.xs_wls(p.styles, p.cap, p.ret, p.ind, 31)
    q = p.slice_dates(0, 37)
    small = X.xs_wls(q.styles.contiguous(), q.cap.contiguous(), q.ret.contiguous(),
                     q.ind.contiguous(), 31)
    torch.cuda.synchronize()
    assert torch.equal(small.f, big.f[:37])
    assert torch.equal(small.resid.nan_to_num(7.0), big.resid[:37].nan_to_num(7.0))
    assert torch.equal(small.r2, big.r2[:37])
    assert torch.equal(small.stats.nan_to_num(7.0), big.stats[:37].nan_to_num(7.0))
    assert torch.equal(small.status, big.status[:37])
