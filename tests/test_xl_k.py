"""Factor sets beyond the register / LDS-resident solvers (160 < K <= 1024; VERDICT r05 Missing 2).

The reference estimators work at any K (`/root/reference/Barra-master/mfm/utils.py:55-92`).  Here
every piece of the eigen adjustment above K = 160 runs on the XL kernels -- output-tiled MFMA draw
covariances (`csrc/eigen.hip: mc_cov_xl_kernel`), the persistent global-slot eigen solver
(`csrc/eigen_xl.hip`), the any-K finalize -- instead of rocSOLVER / rocBLAS behind a host sync.
Each is compared with the CPU fp64 path (LAPACK through torch) on shared draws.
"""
import numpy as np
import pytest
import torch

from llm_driven_multi_factor_model_amd.models.panel import synthetic_panel
from llm_driven_multi_factor_model_amd.models.risk_model import RiskModel
from llm_driven_multi_factor_model_amd.ops import eigen
from llm_driven_multi_factor_model_amd.utils.config import preset

from tests.test_wide_k import _clustered, _spd


@pytest.mark.gpu
def test_xl_mc_cov_draws_extend_the_wide_ones(cuda):
    """K = 200 / 257 draws: factor k of a sim is the same Philox number at every K, so the leading
    140 x 140 block equals the K = 140 wide kernel's matrix (to summation order); any partition
    of the sims gives bitwise the same matrices; every entry is numpy's cov of the draws."""
    from tests.test_eigen import _philox_normals
    T = 300
    wide = eigen.mc_cov(4, 140, T, seed=3, device=cuda)
    for K in (200, 257):
        xl = eigen.mc_cov(4, K, T, seed=3, device=cuda)
        torch.testing.assert_close(xl[:, :140, :140], wide, rtol=1e-11, atol=1e-13)
        assert torch.equal(xl, xl.transpose(1, 2))
        parts = torch.cat([eigen.mc_cov(1, K, T, seed=3, device=cuda),
                           eigen.mc_cov(3, K, T, seed=3, device=cuda, m0=1)])
        assert torch.equal(parts, xl)
    Z = _philox_normals(2, T, 257, 3)
    np.testing.assert_allclose(xl[2].cpu().numpy(), np.cov(Z.T), rtol=1e-11, atol=1e-13)


@pytest.mark.gpu
@pytest.mark.parametrize("K", [165, 200, 260])
def test_xl_eigh_matches_lapack(cuda, K):
    """eigen.eigh above K = 144 on the XL solver: LAPACK eigenvalues (1e-10 relative), A U = U
    diag(w), U orthonormal; a NaN matrix gives NaN; no matrix needs the Jacobi re-solve."""
    g = torch.Generator().manual_seed(K)
    B = 5
    X = torch.randn(B, 2 * K, K, generator=g, dtype=torch.float64)
    F = X.transpose(1, 2) @ X / (2 * K) * 1e-4
    F[2] = float("nan")
    w, U = eigen.eigh(F.to(cuda))
    flags = eigen.LAST_EIGH_FLAGS.cpu()
    ok = [b for b in range(B) if b != 2]
    wr = torch.linalg.eigvalsh(F[ok]).flip(-1)
    torch.testing.assert_close(w.cpu()[ok], wr, rtol=1e-10, atol=1e-18)
    Fg = F.to(cuda)[ok]
    R = Fg @ U[ok] - U[ok] * w[ok][:, None, :]
    assert float(R.abs().max()) < 1e-10 * float(Fg.abs().max())
    G = U[ok].transpose(-1, -2) @ U[ok] - torch.eye(K, dtype=torch.float64, device=cuda)
    assert float(G.abs().max()) < 1e-10
    assert torch.isnan(w[2]).all() and torch.isnan(U[2]).all()
    assert int(flags[ok].sum()) == 0


@pytest.mark.gpu
def test_xl_eigh_clustered_spectra_resolved_on_device(cuda):
    """Repeated eigenvalues at K = 170: the XL solver's orthogonality check flags the matrices
    whose twisted-factorisation vectors are not orthonormal and re-solves them in their slot by the
    Jacobi; every output is orthonormal with LAPACK eigenvalues."""
    K = 170
    A = torch.cat([_clustered(3, K, seed=K), _spd(2, K, seed=K + 1, spread=2.0)])
    w, U = eigen.eigh(A.to(cuda))
    flags = eigen.LAST_EIGH_FLAGS.cpu()
    w, U = w.cpu(), U.cpu()
    assert flags[-1] == 0 and flags[-2] == 0 and int(flags[:3].sum()) >= 1
    eye = torch.eye(K, dtype=torch.float64)
    scale = A.abs().amax((-1, -2))
    for b in range(A.shape[0]):
        assert (U[b].T @ U[b] - eye).abs().max() < 1e-10, (b, int(flags[b]))
        r = (A[b] @ U[b] - U[b] * w[b]).abs().max() / scale[b]
        assert r < 1e-10, (b, float(r))
        torch.testing.assert_close(w[b], torch.linalg.eigvalsh(A[b]).flip(-1), rtol=1e-10,
                                   atol=1e-14 * float(scale[b]))


@pytest.mark.gpu
@pytest.mark.parametrize("K", [163, 213])
def test_xl_eigen_adjust_matches_cpu(cuda, K):
    """The eigen adjustment above K = 144: bias multipliers and adjusted covariances equal the CPU
    fp64 path on the GPU's own draws (1e-8), an invalid date is NaN, the sims-sharded
    accumulation equals the one-shot call, and the rocSOLVER path agrees."""
    D, M = 4, 3
    F = _spd(D, K, seed=K, spread=2.0) * 1e-4
    F[1] = float("nan")
    Cz = eigen.mc_cov(M, K, 2 * K, seed=2, device=cuda)
    Fg, vg = eigen.eigen_risk_adjust(F.to(cuda), Cz=Cz, return_bias=True)
    Fc, vc = eigen.eigen_risk_adjust(F, Cz=Cz.cpu(), return_bias=True)
    torch.testing.assert_close(vg.cpu(), vc, rtol=1e-8, atol=1e-10, equal_nan=True)
    torch.testing.assert_close(Fg.cpu(), Fc, rtol=1e-8, atol=1e-16, equal_nan=True)
    assert torch.isnan(vg[1]).all() and torch.isfinite(vg[[0, 2, 3]]).all()
    Fs, vs = eigen.eigen_risk_adjust_sharded(F.to(cuda), M=M, T_sim=2 * K, seed=2, chunk=2,
                                             return_bias=True)
    torch.testing.assert_close(vs.cpu(), vc, rtol=1e-10, atol=1e-12, equal_nan=True)
    with eigen.using_wide_bias_solver("rocsolver"):
        Fr, vr = eigen.eigen_risk_adjust(F.to(cuda), Cz=Cz, return_bias=True)
    torch.testing.assert_close(vg, vr, rtol=1e-8, atol=1e-10, equal_nan=True)


@pytest.mark.gpu
def test_xl_risk_model_matches_cpu(cuda):
    """RiskModel.run at P = 163, Q = 16 (K = 180) on the GPU: the CS-WLS takes the split kernels
    (P > 128), the eigen stage the XL kernels and equals the CPU fp64 path on the GPU's own draw
    covariances.  Run twice it agrees to rounding only: above 57 industries at Q = 10 the
    moments' industry table is one shared LDS replica (order-dependent fp64 atomics), and the
    eigen adjustment amplifies that ~1e-16 to ~1e-9."""
    D, N, P, Q, M = 230, 1200, 163, 16, 3
    p = synthetic_panel(D, N, P, Q, seed=21, missing_frac=0.01, dtype=torch.float64)
    cfg = preset("reference", eigen_sims=M, nw_half_life=1000.0, vra_half_life=10.0,
                 eigen_sim_length=400)
    g = RiskModel(p.to(cuda), cfg).run()
    assert g.K == 180
    g2 = RiskModel(p.to(cuda), cfg).run()
    torch.testing.assert_close(g.factor_ret, g2.factor_ret, rtol=1e-12, atol=1e-15)
    torch.testing.assert_close(g.eigen_bias, g2.eigen_bias, rtol=1e-7, atol=1e-10, equal_nan=True)
    fin = torch.isfinite(g.nw_cov.reshape(D, -1)).all(-1).cpu()
    assert fin[180:].all()
    Cz = eigen.mc_cov(M, 180, 400, seed=cfg.eigen_seed, device=cuda).cpu()
    Fh, vb = eigen.eigen_risk_adjust(g.nw_cov.cpu(), Cz=Cz, scale_coef=cfg.eigen_scale,
                                     return_bias=True)
    torch.testing.assert_close(g.eigen_bias.cpu(), vb, rtol=1e-8, atol=1e-10, equal_nan=True)
    # F^ = U diag(v^2 w) U^T is not defined by the eigenvalues alone where F0 has a nearly
    # degenerate pair with different multipliers (any rotation inside the pair is an eigenbasis):
    # compare the dates whose F0 eigenvalue gaps exceed 1e-7 of the largest eigenvalue
    w0 = torch.linalg.eigvalsh(torch.nan_to_num(g.nw_cov.cpu()))
    gap = (w0[:, 1:] - w0[:, :-1]).min(-1).values / w0.abs().amax(-1).clamp_min(1e-300)
    ok = (gap > 1e-7) & fin
    assert int(ok.sum()) >= 20
    torch.testing.assert_close(g.eigen_cov.cpu()[ok], Fh[ok], rtol=1e-8, atol=1e-16, equal_nan=True)
    assert torch.isfinite(g.eigen_cov.reshape(D, -1)[-10:]).all()   # not vacuously NaN


@pytest.mark.gpu
@pytest.mark.parametrize("P,Q", [(129, 10), (163, 16), (256, 16)])
def test_xs_wls_many_industries(cuda, P, Q):
    """CS-WLS beyond the fused kernel's 128 industries (the K > 145 risk models): the split
    kernels (moments -> constrained solve -> structured device pinv -> residuals) against the
    fp64 oracle, near-singular dates included (two industries empty)."""
    from llm_driven_multi_factor_model_amd.ops import cross_section as X
    p = synthetic_panel(4, 6000, P, Q, seed=P, missing_frac=0.01, empty_industries=2,
                        dtype=torch.float64)
    ref = X.xs_wls_reference(p.styles, p.cap, p.ret, p.ind, P)
    g = p.to(cuda)
    out = X.xs_wls(g.styles, g.cap, g.ret, g.ind, P)
    torch.testing.assert_close(out.f.cpu(), ref.f, rtol=1e-9, atol=1e-12)
    torch.testing.assert_close(out.r2.cpu(), ref.r2, rtol=1e-9, atol=1e-11)
    torch.testing.assert_close(out.resid.cpu(), ref.resid, rtol=1e-9, atol=1e-13, equal_nan=True)


@pytest.mark.gpu
def test_xl_occupancy_variants_bitwise(cuda):
    """The XL solver compiled for 2 and for 4 waves per SIMD runs the same arithmetic: eigh and
    bias sums are bitwise equal."""
    K = 190
    F = _spd(6, K, seed=3, spread=2.0).to(cuda) * 1e-4
    Cz = eigen.mc_cov(3, K, 400, seed=5, device=cuda)
    out = []
    try:
        for w in (2, 4):
            eigen.set_xl_waves_per_simd(w)
            ww, U = eigen.eigh(F)
            valid = torch.isfinite(ww).all(-1)
            out.append((ww, U, eigen._bias_sum_xl(ww.clamp_min(0.0).contiguous(), valid, Cz)))
    finally:
        eigen.set_xl_waves_per_simd(0)
    for a, b in zip(out[0], out[1]):
        assert torch.equal(a, b)


@pytest.mark.gpu
@pytest.mark.parametrize("wpe", [2, 4])
def test_xl_bias_many_problems_per_slot(cuda, wpe):
    """More (date, sim) problems than resident workgroups: each persistent workgroup solves many
    problems in its slot one after another; the sums equal the CPU fp64 path at both occupancies."""
    K, D, M = 150, 60, 12          # 720 problems > 2 x 256 slots
    g = torch.Generator().manual_seed(11)
    X = torch.randn(D, 2 * K, K, generator=g, dtype=torch.float64)
    F = X.transpose(1, 2) @ X / (2 * K) * 1e-4
    w, _ = torch.linalg.eigh(F)
    w = w.flip(-1).clamp_min(0.0).contiguous()
    valid = torch.ones(D, dtype=torch.bool)
    valid[7] = False
    Cz = eigen.mc_cov(M, K, 400, seed=4, device=cuda)
    try:
        eigen.set_xl_waves_per_simd(wpe)
        S = eigen._bias_sum_xl(w.to(cuda), valid.to(cuda), Cz).cpu()
    finally:
        eigen.set_xl_waves_per_simd(0)
    ref = eigen._bias_sum_reference(w, valid, Cz.cpu())
    torch.testing.assert_close(S, ref, rtol=1e-9, atol=1e-12, equal_nan=True)


@pytest.mark.gpu
def test_xl_eigh_close_pairs_warm_resolve(cuda):
    """Eigenvalue pairs 1e-9 apart (relative) at K = 180: the twisted-factorisation vectors of a
    pair are not orthogonal to 1e-10, so the matrix is re-solved -- warm-started from its own
    vectors made orthonormal by Newton-Schulz steps, the Jacobi rotating only inside the pairs;
    the result is orthonormal with LAPACK eigenvalues."""
    K, B = 180, 3
    g = torch.Generator().manual_seed(8)
    out = []
    for b in range(B):
        Q, _ = torch.linalg.qr(torch.randn(K, K, generator=g, dtype=torch.float64))
        lam = torch.exp(torch.linspace(0.0, -6.0, K, dtype=torch.float64))
        lam[1::7] = lam[0::7][:lam[1::7].numel()] * (1 + 1e-9)   # close pairs
        out.append((Q * lam) @ Q.T)
    A = torch.stack(out)
    w, U = eigen.eigh(A.to(cuda))
    flags = eigen.LAST_EIGH_FLAGS.cpu()
    w, U = w.cpu(), U.cpu()
    assert int((flags == 1).sum()) >= 1, flags
    eye = torch.eye(K, dtype=torch.float64)
    for b in range(B):
        assert (U[b].T @ U[b] - eye).abs().max() < 1e-10, (b, int(flags[b]))
        assert (A[b] @ U[b] - U[b] * w[b]).abs().max() < 1e-12, b
        torch.testing.assert_close(w[b], torch.linalg.eigvalsh(A[b]).flip(-1), rtol=1e-10,
                                   atol=1e-15)


def test_cpu_paths_take_any_industry_and_style_count():
    """The CPU fp64 paths (the oracles, and the reference's own range: any K) are not bound by
    the GPU kernels' P <= 256 / Q <= 16: the dense oracle and the moment-space path agree at
    P = 300 industries, Q = 18 styles (K = 319)."""
    from llm_driven_multi_factor_model_amd.ops import cross_section as X
    from llm_driven_multi_factor_model_amd.ops.xs_sharded import xs_wls_stock_sharded
    p = synthetic_panel(3, 900, 300, 18, seed=2, missing_frac=0.01, dtype=torch.float64)
    a = X.xs_wls(p.styles, p.cap, p.ret, p.ind, 300)
    b = xs_wls_stock_sharded(p.styles, p.cap, p.ret, p.ind, 300)
    assert a.f.shape == (3, 319) and torch.isfinite(a.f).all()
    torch.testing.assert_close(b.f, a.f, rtol=1e-8, atol=1e-10)
    torch.testing.assert_close(b.r2, a.r2, rtol=1e-9, atol=1e-11)
