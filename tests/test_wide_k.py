"""Risk model beyond one wave of factors (K > 64).

SW-L2-sized factor sets (P = 123 industries, Q = 16 styles: K = 140) run every stage on the
device: the CS-WLS regression (structured device pinv), the Newey-West scan, the eigen adjustment
(Philox draws + rocBLAS GEMM covariances, rocSOLVER batched eigen-decompositions), VRA, the
eigenfactor bias statistic, and the attribution kernels (portfolio exposures for any P / Q,
cap-decile shrinkage for any N).  Each is compared with the CPU fp64 path on shared draws.
"""
import numpy as np
import pytest
import torch

from llm_driven_multi_factor_model_amd.models.panel import synthetic_panel
from llm_driven_multi_factor_model_amd.models.risk_model import RiskModel
from llm_driven_multi_factor_model_amd.ops import attribution as A
from llm_driven_multi_factor_model_amd.ops import eigen
from llm_driven_multi_factor_model_amd.ops import xs_reduce as R
from llm_driven_multi_factor_model_amd.utils.config import preset


def _spd(B, K, seed=0, spread=3.0):
    g = torch.Generator().manual_seed(seed)
    Q, _ = torch.linalg.qr(torch.randn(B, K, K, generator=g, dtype=torch.float64))
    lam = torch.exp(torch.linspace(0, -spread * 2.3, K, dtype=torch.float64))[None] * \
        (1 + 0.1 * torch.rand(B, K, generator=g, dtype=torch.float64))
    return (Q * lam[:, None, :]) @ Q.transpose(1, 2)


def test_wide_eigen_adjust_cpu_runs():
    """The CPU fp64 path (oracle) handles any K."""
    F = _spd(3, 70, seed=1) * 1e-4
    F[1] = float("nan")
    Cz = eigen.mc_cov(5, 70, 120, seed=2, device="cpu")
    Fh, v = eigen.eigen_risk_adjust(F, Cz=Cz, return_bias=True)
    assert torch.isnan(Fh[1]).all() and torch.isfinite(Fh[[0, 2]]).all()


@pytest.mark.gpu
def test_hip_wide_mc_cov_same_draws(cuda):
    """K = 140 draws: factor k < 64 of a sim is the same Philox number as in the one-wave
    kernel (the leading block of the covariance agrees to summation order), and any partition
    of the sims gives the same matrices."""
    T = 600
    wide = eigen.mc_cov(6, 140, T, seed=3, device=cuda)
    narrow = eigen.mc_cov(6, 42, T, seed=3, device=cuda)
    torch.testing.assert_close(wide[:, :42, :42], narrow, rtol=1e-11, atol=1e-13)
    assert torch.allclose(wide, wide.transpose(1, 2))
    d = torch.diagonal(wide, dim1=1, dim2=2)
    assert abs(d.mean().item() - 1.0) < 0.02
    parts = torch.cat([eigen.mc_cov(2, 140, T, seed=3, device=cuda),
                       eigen.mc_cov(4, 140, T, seed=3, device=cuda, m0=2)])
    assert torch.equal(parts, wide)


@pytest.mark.gpu
@pytest.mark.parametrize("K", [65, 140, 145, 160])
def test_hip_wide_eigh_and_adjust_match_cpu(cuda, K):
    D, M = 6, 5
    F = _spd(D, K, seed=K, spread=2.0) * 1e-4
    F[2] = float("nan")
    w, U = eigen.eigh(F.to(cuda))
    wr = torch.linalg.eigvalsh(F[[0, 1, 3, 4, 5]]).flip(-1)
    torch.testing.assert_close(w.cpu()[[0, 1, 3, 4, 5]], wr, rtol=1e-10, atol=1e-18)
    assert torch.isnan(w[2]).all()
    Cz = eigen.mc_cov(M, K, 400, seed=2, device=cuda)
    Fg, vg = eigen.eigen_risk_adjust(F.to(cuda), Cz=Cz, return_bias=True)
    Fc, vc = eigen.eigen_risk_adjust(F, Cz=Cz.cpu(), return_bias=True)
    torch.testing.assert_close(vg.cpu(), vc, rtol=1e-8, atol=1e-10, equal_nan=True)
    torch.testing.assert_close(Fg.cpu(), Fc, rtol=1e-8, atol=1e-16, equal_nan=True)
    # sims-sharded accumulation == one shot
    Fs, vs = eigen.eigen_risk_adjust_sharded(F.to(cuda), M=M, T_sim=400, seed=2, chunk=2,
                                             return_bias=True)
    torch.testing.assert_close(vs.cpu(), vc, rtol=1e-10, atol=1e-12, equal_nan=True)


@pytest.mark.gpu
def test_hip_risk_model_k140_matches_cpu(cuda):
    """RiskModel.run + eigenfactor_bias at P = 123, Q = 16 (K = 140) on the GPU; every stage
    matches the CPU fp64 path (the eigen stage on the GPU's own draw covariances).  300 dates:
    the Newey-West covariance needs more dates than factors (utils.py:29-30), so dates >= 140
    carry finite covariances; a long half-life keeps them positive definite (a 30-day half-life
    leaves < 140 effective dates: negative eigenvalues, an all-NaN eigen stage)."""
    D, N, P, Q, M = 300, 1200, 123, 16, 6
    p = synthetic_panel(D, N, P, Q, seed=13, missing_frac=0.01, dtype=torch.float64)
    cfg = preset("reference", eigen_sims=M, nw_half_life=1000.0, vra_half_life=10.0,
                 eigen_sim_length=300)   # T_sim > K: full-rank draw covariances
    g = RiskModel(p.to(cuda), cfg).run()
    assert g.K == 140
    c = RiskModel(p, cfg)
    c.regress()
    c.newey_west()
    torch.testing.assert_close(g.factor_ret.cpu(), c.factor_ret, rtol=1e-9, atol=1e-12)
    torch.testing.assert_close(g.nw_cov.cpu(), c.nw_cov, rtol=1e-8, atol=1e-15, equal_nan=True)
    fin = torch.isfinite(g.nw_cov.reshape(D, -1)).all(-1).cpu()
    assert fin[140:].all() and not fin[:139].any()
    Cz = eigen.mc_cov(M, 140, 300, seed=cfg.eigen_seed, device=cuda).cpu()
    Fh, vb = eigen.eigen_risk_adjust(g.nw_cov.cpu(), Cz=Cz, scale_coef=cfg.eigen_scale,
                                     return_bias=True)
    torch.testing.assert_close(g.eigen_bias.cpu(), vb, rtol=1e-8, atol=1e-10, equal_nan=True)
    torch.testing.assert_close(g.eigen_cov.cpu(), Fh, rtol=1e-8, atol=1e-16, equal_nan=True)
    assert torch.isfinite(g.eigen_cov.reshape(D, -1)[140:]).all()   # not vacuously NaN
    assert torch.isfinite(g.vra_cov[-1]).all()
    bias = g.eigenfactor_bias("eigen", start=150, predlen=2)
    assert bias.shape == (140,) and torch.isfinite(bias).all()


@pytest.mark.gpu
def test_hip_portfolio_exposure_wide(cuda):
    """P = 150 industries (> 128) and Q = 20 styles (> 16): block launches and dynamic LDS."""
    p = synthetic_panel(5, 1500, 150, 20, seed=3, missing_frac=0.02, dtype=torch.float64)
    g = p.to(cuda)
    # stats [D, Q + 2] (cap-weighted style means, pooled sigma, n) are inputs of the kernel;
    # the regression's own are not needed to compare the two paths
    st = torch.rand(p.D, p.Q + 2, dtype=torch.float64)
    st[:, p.Q] += 0.5
    h = torch.rand(p.D, p.N, dtype=torch.float64)
    got = A.portfolio_exposure(g.styles, g.cap, g.ret, g.ind, h.to(cuda), st.to(cuda), p.P)
    ref = A.portfolio_exposure(p.styles, p.cap, p.ret, p.ind, h, st, p.P)
    torch.testing.assert_close(got.cpu(), ref, rtol=1e-10, atol=1e-12)


@pytest.mark.gpu
def test_hip_bayes_shrink_wide_universe(cuda):
    """N = 20000 stocks (> the 16384 LDS sort): device sort + the same shrink kernel."""
    g = torch.Generator().manual_seed(5)
    vol = torch.rand(3, 20000, generator=g) * 0.05 + 0.01
    cap = torch.exp(torch.randn(3, 20000, generator=g))
    vol[1, ::7] = float("nan")
    got = R.bayes_shrink(vol.to(cuda), cap.to(cuda)).cpu()
    ref = R.bayes_shrink(vol, cap)
    torch.testing.assert_close(got, ref, rtol=1e-5, atol=1e-6, equal_nan=True)
    assert np.isnan(got[1, ::7].numpy()).all()


def test_rocsolver_wrapper_rejects_host_tensors():
    from llm_driven_multi_factor_model_amd.ops import rocsolver
    with pytest.raises(TypeError):
        rocsolver.syev_batched(torch.eye(3, dtype=torch.float64)[None])


@pytest.mark.gpu
def test_rocsolver_strided_batched_eigh(cuda):
    """ops/rocsolver.py (the K > 64 probe utility): rocSOLVER's strided-batched syevd / syevj on
    140 x 140 sample covariances == LAPACK eigenvalues, A V = V diag(w)."""
    from llm_driven_multi_factor_model_amd.ops import rocsolver
    g = torch.Generator().manual_seed(5)
    X = torch.randn(6, 300, 140, generator=g, dtype=torch.float64)
    A = (X.transpose(1, 2) @ X / 300).to(cuda)
    wr = torch.linalg.eigvalsh(A.cpu())
    for method, tol in (("syevd", 1e-11), ("syevj", 1e-9)):
        w, V, info = rocsolver.syev_batched(A, method)
        assert int(info.abs().sum()) == 0, method
        torch.testing.assert_close(w.cpu(), wr, rtol=tol, atol=1e-13, msg=method)
        R = A @ V - V * w[:, None, :]
        assert float(R.abs().max()) < 1e-9, method


@pytest.mark.gpu
@pytest.mark.parametrize("layout", ["row", "mixed", "pair"])
def test_hip_wide_bias_solver_matches_oracle(cuda, layout):
    """csrc/eigen_wide.hip (the "hip" wide solver): K = 42 on the multi-wave kernels equals the
    one-wave mode-5 kernel, K = 80 / 100 / 140 equal the CPU fp64 oracle, with one lane per row,
    two lanes per row (every K, the default) and the round-5 mix (one lane per row up to K = 96);
    an invalid date gives NaN."""
    from llm_driven_multi_factor_model_amd import _native
    if layout == "row" and not _native.ab_build():
        pytest.skip("one lane per row at K > 96: A/B layout, not in the production library")
    g = torch.Generator().manual_seed(9)
    eigen.set_wide_kernel_layout(layout)
    try:
        _wide_oracle_cases(cuda, g, _native)
    finally:
        eigen.set_wide_kernel_layout("pair")


def _wide_oracle_cases(cuda, g, _native):
    for K, D, M in ((42, 12, 8), (80, 5, 4), (100, 5, 4), (140, 6, 5)):
        X = torch.randn(D, 400, K, generator=g, dtype=torch.float64)
        F = X.transpose(1, 2) @ X / 400
        F[2] = float("nan")
        w, _ = eigen.eigh(F.to(cuda))
        valid = torch.isfinite(w).all(-1)
        w = torch.where(valid[:, None], w.clamp_min(0.0), w).contiguous()
        Cz = eigen.mc_cov(M, K, 300, seed=3, device=cuda)
        S = eigen._bias_sum_wide_hip(w, valid, Cz)
        ref = eigen._bias_sum_reference(w.cpu(), valid.cpu(), Cz.cpu())
        torch.testing.assert_close(S.cpu(), ref, rtol=1e-9, atol=1e-12, equal_nan=True, msg=str(K))
        assert torch.isnan(S[2]).all() and torch.isfinite(S[valid]).all()
        if K <= 64:
            S5 = torch.zeros_like(S)
            ws = torch.empty(D * M * K, dtype=torch.float64, device=cuda)
            _native.call("mfa_eigen_bias_accumulate", _native.ptr(w),
                         _native.ptr(valid.to(torch.int32).contiguous()), D, K, M, _native.ptr(Cz),
                         eigen.MAX_SWEEPS, eigen.TOL, _native.ptr(ws), _native.ptr(S5),
                         _native.stream(cuda))
            torch.testing.assert_close(S, S5, rtol=1e-12, atol=1e-14, equal_nan=True)


@pytest.mark.gpu
def test_hip_wide_bias_solver_in_risk_model(cuda):
    """RiskModel at K = 140: the "hip" wide solver (default) == the rocSOLVER path."""
    D, N, P, Q, M = 200, 1000, 123, 16, 4
    p = synthetic_panel(D, N, P, Q, seed=17, missing_frac=0.01, dtype=torch.float64)
    cfg = preset("reference", eigen_sims=M, nw_half_life=1000.0, eigen_sim_length=300)
    with eigen.using_wide_bias_solver("rocsolver"):
        a = RiskModel(p.to(cuda), cfg).run()
    with eigen.using_wide_bias_solver("hip"):
        b = RiskModel(p.to(cuda), cfg).run()
    assert torch.isfinite(a.eigen_bias[-1]).all()
    # 1e-8: at the first full-rank dates the smallest eigenvalue's ratio is ill-conditioned
    # (measured 1.2e-9 between the two solvers at date 143, k = 139)
    torch.testing.assert_close(b.eigen_bias, a.eigen_bias, rtol=1e-8, atol=1e-12, equal_nan=True)
    torch.testing.assert_close(b.eigen_cov, a.eigen_cov, rtol=1e-8, atol=1e-16, equal_nan=True)


def test_wide_bias_solver_selection():
    with pytest.raises(ValueError):
        eigen.set_wide_bias_solver("lapack")
    with eigen.using_wide_bias_solver("hip"):
        assert eigen._wide_solver == "hip"
    assert eigen._wide_solver in eigen.WIDE_BIAS_SOLVERS


def test_wide_bias_env_is_validated():
    """A misspelt MFA_WIDE_BIAS fails the import instead of silently selecting rocSOLVER."""
    import os
    import subprocess
    import sys
    env = dict(os.environ, MFA_WIDE_BIAS="hipp", CUDA_VISIBLE_DEVICES="", HIP_VISIBLE_DEVICES="")
    root = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
    r = subprocess.run([sys.executable, "-c", "import llm_driven_multi_factor_model_amd.ops.eigen"],
                       capture_output=True, text=True, env=env, timeout=300, cwd=root)
    assert r.returncode != 0 and "MFA_WIDE_BIAS" in r.stderr


@pytest.mark.gpu
def test_hip_wide_eigh_native(cuda):
    """eigen.eigh at 96 < K <= 144 on the multi-wave HIP solver == LAPACK (values 1e-10 relative,
    A U = U diag(w), U orthonormal); a NaN matrix gives NaN; the rocSOLVER path agrees."""
    g = torch.Generator().manual_seed(12)
    K, B = 140, 7
    X = torch.randn(B, 400, K, generator=g, dtype=torch.float64)
    F = X.transpose(1, 2) @ X / 400
    F[3] = float("nan")
    w, U = eigen.eigh(F.to(cuda))
    ok = [b for b in range(B) if b != 3]
    wr = torch.linalg.eigvalsh(F[ok]).flip(-1)
    torch.testing.assert_close(w.cpu()[ok], wr, rtol=1e-10, atol=1e-13)
    Fg = F.to(cuda)[ok]
    R = Fg @ U[ok] - U[ok] * w[ok][:, None, :]
    assert float(R.abs().max()) < 1e-10
    G = U[ok].transpose(-1, -2) @ U[ok] - torch.eye(K, dtype=torch.float64, device=cuda)
    assert float(G.abs().max()) < 1e-10
    assert torch.isnan(w[3]).all() and torch.isnan(U[3]).all()
    with eigen.using_wide_bias_solver("rocsolver"):
        w2, _ = eigen.eigh(F.to(cuda))
    torch.testing.assert_close(w2.cpu()[ok], w.cpu()[ok], rtol=1e-10, atol=1e-13)


@pytest.mark.gpu
@pytest.mark.parametrize("K", [80, 101, 140, 157])
def test_hip_wide_mc_cov_is_fp64_cov_of_its_philox_draws(cuda, K):
    """K > 64 draw covariances (mc_cov_wide_kernel, fp64 matrix cores): every entry equals
    numpy's fp64 cov of the same Philox normals (tile layout, odd K, centring)."""
    from tests.test_eigen import _philox_normals
    T, M, seed = 300, 2, 7
    Cz = eigen.mc_cov(M, K, T, seed=seed, device=cuda).cpu().numpy()
    for m in range(M):
        Z = _philox_normals(m, T, K, seed)
        np.testing.assert_allclose(Cz[m], np.cov(Z.T), rtol=1e-11, atol=1e-13)


def _clustered(B, K, seed=0):
    """SPD matrices with exactly repeated eigenvalues (clusters of 1..6) and a scaled identity."""
    g = torch.Generator().manual_seed(seed)
    out = []
    for b in range(B):
        Q, _ = torch.linalg.qr(torch.randn(K, K, generator=g, dtype=torch.float64))
        lam, k = [], 0
        while len(lam) < K:
            lam += [float(np.exp(-0.05 * k))] * (1 + (k * 7 + b) % 6)
            k += 1
        lam = torch.tensor(lam[:K], dtype=torch.float64)
        out.append((Q * lam) @ Q.T)
    out[-1] = 3e-4 * torch.eye(K, dtype=torch.float64)
    return torch.stack(out)


@pytest.mark.gpu
@pytest.mark.parametrize("K", [80, 140])
def test_hip_wide_eigh_clustered_spectra_resolved_on_device(cuda, K):
    """Finite matrices with repeated eigenvalues: the tridiagonal solver's vectors
    are checked on the device (max |U^T U - I| <= 1e-10) and the failures re-solved by the device
    Jacobi -- orthonormal U, A U = U diag(w), LAPACK eigenvalues; no host sync, no rocSOLVER."""
    from llm_driven_multi_factor_model_amd import _native
    A = torch.cat([_clustered(4, K, seed=K), _spd(2, K, seed=K + 1, spread=2.0)])
    Ag = A.to(cuda).contiguous()
    B = A.shape[0]
    w = torch.empty(B, K, dtype=torch.float64, device=cuda)
    U = torch.empty(B, K, K, dtype=torch.float64, device=cuda)
    ws = torch.empty(B * K * K, dtype=torch.float64, device=cuda)
    fixed = torch.full((B,), -1, dtype=torch.int32, device=cuda)
    _native.call("mfa_eigh_wide_fix", _native.ptr(Ag), B, K, eigen.ORTHO_TOL, _native.ptr(w),
                 _native.ptr(U), _native.ptr(ws), _native.ptr(fixed), _native.stream(cuda))
    torch.cuda.synchronize()
    w, U, fixed = w.cpu(), U.cpu(), fixed.cpu()
    assert (fixed >= 0).all()
    assert fixed[-1] == 0 and fixed[-2] == 0          # distinct spectra pass the check
    eye = torch.eye(K, dtype=torch.float64)
    scale = A.abs().amax((-1, -2))
    for b in range(B):
        assert (U[b].T @ U[b] - eye).abs().max() < 1e-10, (b, int(fixed[b]))
        r = (A[b] @ U[b] - U[b] * w[b]).abs().max() / scale[b]
        assert r < 1e-10, (b, float(r))
        torch.testing.assert_close(w[b], torch.linalg.eigvalsh(A[b]).flip(-1), rtol=1e-10,
                                   atol=1e-14 * float(scale[b]))
    # the public entry point takes the same path
    w2, U2 = eigen.eigh(Ag)
    torch.testing.assert_close(w2.cpu(), w, rtol=0, atol=0)
    # a NaN input stays NaN (not "re-solved")
    An = Ag.clone()
    An[1, 3, 5] = float("nan")
    wn, Un = eigen.eigh(An)
    assert torch.isnan(wn[1]).all() and torch.isfinite(wn[0]).all()


@pytest.mark.gpu
@pytest.mark.parametrize("K", [80, 170])
def test_hip_eigh_skips_resolve_of_indefinite_dates(cuda, K):
    """The eigen adjustment passes resolve_psd_tol: a clustered (re-solve-needing) matrix with a
    negative eigenvalue -- an invalid date, whose eigenvectors are never read -- is flagged 2 and
    not re-solved; without the tolerance it is re-solved (flag 1).  Eigenvalues agree both ways."""
    A = _clustered(2, K, seed=K)
    g = torch.Generator().manual_seed(K)
    Q, _ = torch.linalg.qr(torch.randn(K, K, generator=g, dtype=torch.float64))
    lam = torch.linalg.eigvalsh(A[0]).flip(-1)
    lam[-3:] = -1e-6                                     # indefinite, with a repeated value
    A[0] = (Q * lam) @ Q.T
    Ag = A.to(cuda)
    w1, _ = eigen.eigh(Ag)
    f1 = eigen.LAST_EIGH_FLAGS.cpu()
    w2, _ = eigen.eigh(Ag, resolve_psd_tol=0.0)
    f2 = eigen.LAST_EIGH_FLAGS.cpu()
    assert int(f1[0]) == 1 and int(f2[0]) == 2, (f1, f2)
    assert int(f2[1]) == int(f1[1])                       # the PSD matrix is handled alike
    torch.testing.assert_close(w2[0].cpu(), torch.linalg.eigvalsh(A[0]).flip(-1), rtol=1e-9,
                               atol=1e-13)
