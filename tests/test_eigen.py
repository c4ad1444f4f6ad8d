"""Batched Jacobi eigh, MC draw covariances and the eigenfactor risk adjustment."""
import numpy as np
import pandas as pd
import pytest
import torch

from llm_driven_multi_factor_model_amd.ops import eigen


def _spd(B, K, seed=0, spread=3.0):
    g = torch.Generator().manual_seed(seed)
    Q, _ = torch.linalg.qr(torch.randn(B, K, K, generator=g, dtype=torch.float64))
    lam = torch.exp(torch.linspace(0, -spread * 2.3, K, dtype=torch.float64))[None] * \
        (1 + 0.1 * torch.rand(B, K, generator=g, dtype=torch.float64))
    return (Q * lam[:, None, :]) @ Q.transpose(1, 2)


def test_eigh_reference_descending():
    A = _spd(3, 6)
    w, U = eigen.eigh(A)
    assert (w[:, :-1] >= w[:, 1:]).all()
    torch.testing.assert_close((U * w[:, None, :]) @ U.transpose(1, 2), A, rtol=1e-10, atol=1e-14)


def test_eigen_adjust_cpu_shapes_and_nan():
    F = _spd(4, 5, seed=2) * 1e-4
    F[1] = float("nan")
    Cz = eigen.mc_cov(20, 5, 200, seed=3, device="cpu")
    Fh, v = eigen.eigen_risk_adjust(F, Cz=Cz, return_bias=True)
    assert torch.isnan(Fh[1]).all() and torch.isfinite(Fh[[0, 2, 3]]).all()
    # the adjustment only rescales eigenvalues: eigenvectors of F and F_hat coincide
    w0, U0 = eigen.eigh(F[0])
    w1, U1 = eigen.eigh(Fh[0])
    assert torch.allclose((U0.T @ Fh[0] @ U0).diagonal(), (v[0] ** 2) * w0, rtol=1e-9)


@pytest.mark.reference
def test_eigen_adjust_statistical_parity_with_reference(ref):
    K, T, M = 5, 400, 300
    F = _spd(1, K, seed=5, spread=1.5)[0] * 1e-4
    df = pd.DataFrame(F.numpy(), columns=list("abcde"), index=list("abcde"))
    R = ref.utils.eigen_risk_adj(df, T=T, M=M, scale_coef=1.4).values
    Cz = eigen.mc_cov(M, K, T, seed=11, device="cpu")
    Fh = eigen.eigen_risk_adjust(F[None], Cz=Cz, scale_coef=1.4)[0].numpy()
    w0 = np.linalg.eigvalsh(F.numpy())[::-1]
    wr = np.linalg.eigvalsh(R)[::-1]
    wo = np.linalg.eigvalsh(Fh)[::-1]
    # multipliers v^2 agree within Monte-Carlo noise (both > 1 for the small eigenvalues)
    np.testing.assert_allclose(wo / w0, wr / w0, rtol=0.03)


def _parity_k42(ref, sorted_eig):
    """Multipliers v^2 of the 42 eigenvalues (ours / reference's eigen_risk_adj at K = 42,
    M = 100, T = 400, independent Monte-Carlo draws)."""
    K, T, M = 42, 400, 100
    F = _spd(1, K, seed=5, spread=1.5)[0] * 1e-4
    cols = [f"f{i}" for i in range(K)]
    df = pd.DataFrame(F.numpy(), columns=cols, index=cols)
    eig = np.linalg.eig
    if sorted_eig:
        np.linalg.eig = lambda a: tuple(x[..., ::-1] for x in np.linalg.eigh(a))
    try:
        R = ref.utils.eigen_risk_adj(df, T=T, M=M, scale_coef=1.4).values
    finally:
        np.linalg.eig = eig
    Cz = eigen.mc_cov(M, K, T, seed=11, device="cpu")
    Fh = eigen.eigen_risk_adjust(F[None], Cz=Cz, scale_coef=1.4)[0].numpy()
    w0 = np.linalg.eigvalsh(F.numpy())[::-1]
    return np.linalg.eigvalsh(Fh)[::-1] / w0, np.linalg.eigvalsh(R)[::-1] / w0


@pytest.mark.reference
def test_eigen_adjust_statistical_parity_with_reference_k42(ref):
    """VERDICT r05 item 5, at the headline K = 42.  The reference pairs simulated and real
    eigenvalues by np.linalg.eig's UNSORTED output order (quirk Q7, utils.py:64,79); with that
    order fixed to descending (an eigh shim) every multiplier agrees within Monte-Carlo noise
    (3 %).  Against the raw reference the bulk agrees the same way; the tail of the spectrum,
    where eig's order is not descending (F0's smallest eigenvalues come out ascending), pairs
    differently and differs by up to ~15 % -- a reference artefact, not noise."""
    ours, want = _parity_k42(ref, sorted_eig=True)
    np.testing.assert_allclose(ours, want, rtol=0.03)
    ours, raw = _parity_k42(ref, sorted_eig=False)
    rel = np.abs(ours - raw) / raw
    assert np.median(rel) < 0.02 and rel[:21].max() < 0.04
    assert rel[-2:].min() > 0.05      # the eig-order pairing of the two smallest is visible


@pytest.mark.gpu
@pytest.mark.parametrize("K,B", [(42, 50), (7, 10), (64, 5), (1, 3), (33, 9)])
def test_hip_eigh_matches_torch(cuda, K, B):
    A = _spd(B, K, seed=K)
    w, U = eigen.eigh(A.to(cuda))
    w, U = w.cpu(), U.cpu()
    wr = torch.linalg.eigvalsh(A).flip(-1)
    torch.testing.assert_close(w, wr, rtol=1e-10, atol=1e-14 * wr.abs().max().item())
    torch.testing.assert_close((U * w[:, None, :]) @ U.transpose(1, 2), A, rtol=1e-9, atol=1e-13)
    torch.testing.assert_close(U.transpose(1, 2) @ U, torch.eye(K, dtype=torch.float64).expand(B, K, K),
                               rtol=0, atol=1e-12)


@pytest.mark.gpu
@pytest.mark.parametrize("K", [42, 12, 33])
def test_hip_eigh_clustered_spectrum(cuda, K):
    """Exactly repeated and 1e-9-close eigenvalues: the tridiagonal eigh's eigenvectors of such
    clusters are not orthogonal, so those matrices are flagged and re-solved by the Jacobi in
    the same call; well-separated matrices of the batch keep the fast path."""
    g = torch.Generator().manual_seed(K)
    Q, _ = torch.linalg.qr(torch.randn(4, K, K, generator=g, dtype=torch.float64))
    lam = torch.exp(torch.linspace(0, -6, K, dtype=torch.float64)).repeat(4, 1)
    lam[0, 3:8] = lam[0, 3]                    # 5-fold exact cluster
    lam[1, 1] = lam[1, 0] * (1 + 1e-9)         # near pair
    lam[2] = 1e-4                              # scaled identity
    A = (Q * lam[:, None, :]) @ Q.transpose(1, 2)
    w, U = eigen.eigh(A.to(cuda))
    w, U = w.cpu(), U.cpu()
    wr = torch.linalg.eigvalsh(A).flip(-1)
    torch.testing.assert_close(w, wr, rtol=1e-10, atol=1e-14 * wr.abs().max().item())
    torch.testing.assert_close((U * w[:, None, :]) @ U.transpose(1, 2), A, rtol=1e-9, atol=1e-13)
    torch.testing.assert_close(U.transpose(1, 2) @ U, torch.eye(K, dtype=torch.float64).expand(4, K, K),
                               rtol=0, atol=1e-12)


@pytest.mark.gpu
def test_hip_eigh_nan_input(cuda):
    A = _spd(2, 8).to(cuda)
    A[1, 0, 0] = float("nan")
    w, U = eigen.eigh(A)
    assert torch.isfinite(w[0]).all() and torch.isnan(w[1]).all()


@pytest.mark.gpu
def test_hip_mc_cov_statistics(cuda):
    Cz = eigen.mc_cov(64, 42, 2520, seed=1, device=cuda).cpu()
    assert torch.allclose(Cz, Cz.transpose(1, 2))
    d = torch.diagonal(Cz, dim1=1, dim2=2)
    assert abs(d.mean().item() - 1.0) < 0.01
    off = Cz - torch.diag_embed(d)
    assert off.abs().mean().item() < 0.03  # ~ sqrt(2/(pi T))
    assert not torch.equal(Cz[0], Cz[1])
    again = eigen.mc_cov(64, 42, 2520, seed=1, device=cuda).cpu()
    assert torch.equal(Cz, again)  # counter-based RNG: bitwise reproducible


def _need_solver(solver):
    if solver not in eigen.available_bias_solvers():
        pytest.skip(f"{solver}: A/B variant, not in the production library")


@pytest.mark.gpu
@pytest.mark.parametrize("solver", sorted(eigen.BIAS_SOLVERS))
@pytest.mark.parametrize("K", [42, 5, 17, 64, 37, 43, 9, 16, 25, 32, 45, 48, 49])
def test_hip_eigen_adjust_matches_reference_path(cuda, solver, K):
    """Every instantiated register width of the tridiagonal bias solver (KP = 8 / 16 / 24 / 32 /
    42 / 44 / 48 / 64: K at and just past each width) against the CPU path at 1e-8."""
    _need_solver(solver)
    D, M = 12, 16
    F = _spd(D, K, seed=9 + K, spread=2.0) * 1e-4
    F[3] = float("nan")
    Cz = eigen.mc_cov(M, K, 500, seed=2, device=cuda)
    with eigen.using_bias_solver(solver):
        Fg, vg = eigen.eigen_risk_adjust(F.to(cuda), Cz=Cz, return_bias=True)
    Fc, vc = eigen.eigen_risk_adjust(F, Cz=Cz.cpu(), return_bias=True)
    torch.testing.assert_close(vg.cpu(), vc, rtol=1e-8, atol=1e-10, equal_nan=True)
    torch.testing.assert_close(Fg.cpu(), Fc, rtol=1e-8, atol=1e-16, equal_nan=True)


@pytest.mark.gpu
def test_hip_bias_solvers_agree_on_pipeline_like_inputs(cuda):
    """Every GPU solver gives the same per-sim bias ratios on graded, nearly-diagonal draw
    covariances (the shape of the MC problem: C_b = S C_z S, S spanning decades)."""
    D, K, M = 40, 42, 24
    g = torch.Generator().manual_seed(7)
    Q, _ = torch.linalg.qr(torch.randn(D, K, K, generator=g, dtype=torch.float64))
    lam = torch.exp(torch.randn(D, K, generator=g, dtype=torch.float64) * 1.5 - 9.0)
    F = ((Q * lam[:, None, :]) @ Q.transpose(1, 2)).to(cuda)
    Cz = eigen.mc_cov(M, K, 2520, seed=3, device=cuda)
    out = {}
    for solver in eigen.available_bias_solvers():
        with eigen.using_bias_solver(solver):
            out[solver] = eigen.eigen_risk_adjust(F, Cz=Cz, return_bias=True)[1].cpu()
    for solver in out:
        torch.testing.assert_close(out[solver], out["jacobi"], rtol=1e-10, atol=0)


@pytest.mark.gpu
def test_bias_mode13_four_accumulators_matches_mode5(cuda, ab_lib):
    """A/B mode 13 (mode 5 with four accumulators per matvec / back-transform dot product): the
    same bias ratios as mode 5 to rounding, on graded draw covariances and with a NaN date."""
    import ctypes as C
    from llm_driven_multi_factor_model_amd import _native
    _native.register("mfa_eigen_set_bias_mode", [C.c_int])
    F = _spd(9, 42, seed=11, spread=2.5) * 1e-4
    F[4] = float("nan")
    Cz = eigen.mc_cov(16, 42, 2520, seed=5, device=cuda)
    lib = _native.lib()
    out = {}
    try:
        for mode in (0, 5, 13):
            lib.mfa_eigen_set_bias_mode(mode)
            out[mode] = eigen.eigen_risk_adjust(F.to(cuda), Cz=Cz, return_bias=True)[1].cpu()
    finally:
        lib.mfa_eigen_set_bias_mode(5)
    assert torch.equal(out[5].isnan(), out[13].isnan())
    torch.testing.assert_close(out[13], out[5], rtol=1e-12, atol=0, equal_nan=True)
    # a different kernel ran (not a fallback to the Jacobi, mode 0): different rounding
    assert not torch.equal(out[13].nan_to_num(0), out[0].nan_to_num(0))


@pytest.mark.gpu
@pytest.mark.parametrize("K", [42, 37, 44])
def test_bias_padded_eigenvectors_bitwise_unpadded(cuda, ab_lib, K):
    """Mode 5 pads the tridiagonal to 44 rows with decoupled rows, so its eigenvector
    recurrences carry no `i < K` tests; mode 14 is the unpadded kernel.  Same arithmetic on every
    real row and the same twist index: bitwise the same bias ratios; NaN dates stay NaN."""
    import ctypes as C
    from llm_driven_multi_factor_model_amd import _native
    _native.register("mfa_eigen_set_bias_mode", [C.c_int])
    F = _spd(7, K, seed=K, spread=2.5) * 1e-4
    F[3] = float("nan")
    Cz = eigen.mc_cov(12, K, 2520, seed=6, device=cuda)
    lib = _native.lib()
    out = {}
    try:
        for mode in (5, 14, 15, 16, 18, 20):  # 15 / 16: every reflector row stored; 18: skipped
            # no-op steps; 20: tau-only back-transform skips
            lib.mfa_eigen_set_bias_mode(mode)
            out[mode] = eigen.eigen_risk_adjust(F.to(cuda), Cz=Cz, return_bias=True)[1].cpu()
    finally:
        lib.mfa_eigen_set_bias_mode(5)
    for mode in (14, 15, 16, 18, 20):
        assert torch.equal(out[5].isnan(), out[mode].isnan())
        assert torch.equal(out[mode].nan_to_num(7.0), out[5].nan_to_num(7.0)), mode


@pytest.mark.gpu
@pytest.mark.parametrize("K", [42, 37])
def test_bias_mode19_newton_laguerre_matches_default(cuda, ab_lib, K):
    """A/B mode 19 (the default with Newton-refined reciprocal / square root in the Laguerre
    loop): the Sturm-guarded iteration lands within its stopping tolerance of the same roots, so
    the bias ratios agree with the default to rounding; NaN dates stay NaN."""
    import ctypes as C
    from llm_driven_multi_factor_model_amd import _native
    _native.register("mfa_eigen_set_bias_mode", [C.c_int])
    F = _spd(7, K, seed=K + 1, spread=2.5) * 1e-4
    F[2] = float("nan")
    Cz = eigen.mc_cov(12, K, 2520, seed=8, device=cuda)
    lib = _native.lib()
    out = {}
    try:
        for mode in (5, 19):
            lib.mfa_eigen_set_bias_mode(mode)
            out[mode] = eigen.eigen_risk_adjust(F.to(cuda), Cz=Cz, return_bias=True)[1].cpu()
    finally:
        lib.mfa_eigen_set_bias_mode(5)
    assert torch.equal(out[5].isnan(), out[19].isnan())
    torch.testing.assert_close(out[19], out[5], rtol=1e-12, atol=0, equal_nan=True)


@pytest.mark.gpu
@pytest.mark.parametrize("K,D,M", [(42, 7, 5), (30, 5, 4), (42, 1, 1)])
def test_hip_dense_bias_solver_tail_and_invalid_dates(cuda, ab_lib, K, D, M):
    """Lane-dense solver (3 problems per 2-wave workgroup): a last workgroup with empty slots
    (D * M not a multiple of 3), a NaN date in the middle of a workgroup, K < 42 (inactive
    rows in every slot) -- same bias ratios as the one-problem-per-wave mode-5 kernel."""
    F = _spd(D, K, seed=K + D, spread=2.5) * 1e-4
    if D > 2:
        F[2] = float("nan")
    Cz = eigen.mc_cov(M, K, 2520, seed=4, device=cuda)
    with eigen.using_bias_solver("tridiag"):
        Fa, va = eigen.eigen_risk_adjust(F.to(cuda), Cz=Cz, return_bias=True)
    with eigen.using_bias_solver("tridiag_dense"):
        Fb, vb = eigen.eigen_risk_adjust(F.to(cuda), Cz=Cz, return_bias=True)
    assert torch.equal(va.isnan(), vb.isnan())
    torch.testing.assert_close(vb.cpu(), va.cpu(), rtol=1e-11, atol=0, equal_nan=True)
    torch.testing.assert_close(Fb.cpu(), Fa.cpu(), rtol=1e-10, atol=1e-20, equal_nan=True)


def _philox_normals(m, T, K, seed):
    """numpy replica of mc_cov_kernel's draws: Philox4x32-10 keyed by (seed), counter
    (sim, time, factor // 2, 0x4D464131), two 53-bit uniforms, fp64 Box-Muller pair."""
    M32 = np.uint64(0xFFFFFFFF)
    t, k = np.meshgrid(np.arange(T, dtype=np.uint64), np.arange(K, dtype=np.uint64) // np.uint64(2), indexing="ij")
    x = np.full(t.shape, np.uint64(m)); y = t.copy(); z = k.copy(); w = np.full(t.shape, np.uint64(0x4D464131))
    k0, k1 = np.uint64(seed & 0xFFFFFFFF), np.uint64((seed >> 32) & 0xFFFFFFFF)
    for _ in range(10):
        p0 = np.uint64(0xD2511F53) * x
        p1 = np.uint64(0xCD9E8D57) * z
        x, y, z, w = ((p1 >> np.uint64(32)) ^ y ^ k0) & M32, p1 & M32, ((p0 >> np.uint64(32)) ^ w ^ k1) & M32, p0 & M32
        k0, k1 = (k0 + np.uint64(0x9E3779B9)) & M32, (k1 + np.uint64(0xBB67AE85)) & M32
    u = lambda hi, lo: (((hi >> np.uint64(5)) << np.uint64(26) | (lo >> np.uint64(6))).astype(np.float64) + 1.0) / 2.0 ** 53
    rr = np.sqrt(-2.0 * np.log(u(x, y)))
    ang = 2.0 * np.pi * u(z, w)
    odd = (np.arange(K) & 1)[None, :] == 1
    return np.where(odd, rr * np.sin(ang), rr * np.cos(ang))


@pytest.mark.gpu
def test_hip_mc_cov_is_fp64_cov_of_its_philox_draws(cuda):
    """Every entry of the fp64-MFMA draw covariance equals numpy's fp64 cov of the same Philox
    normals (checks the matrix-core tile layout and the centring)."""
    K, T, M, seed = 42, 300, 3, 7
    Cz = eigen.mc_cov(M, K, T, seed=seed, device=cuda).cpu().numpy()
    for m in range(M):
        Z = _philox_normals(m, T, K, seed)
        np.testing.assert_allclose(Cz[m], np.cov(Z.T), rtol=1e-11, atol=1e-13)


@pytest.mark.gpu
@pytest.mark.parametrize("T,splits", [(300, (5, 7)), (2520, (256, 16)), (2520, (1, 100, 171))])
def test_hip_mc_cov_range_is_a_slice(cuda, T, splits):
    """Any partition of the sims over launches (eigen_chunk, the short last chunk, world size)
    draws the covariances of one unsplit call bit for bit: the time-axis chunking depends on T
    only (at T = 2520 a 256-sim and a 16-sim launch used to sum in different orders)."""
    M = sum(splits)
    full = eigen.mc_cov(M, 42, T, seed=5, device=cuda)
    parts, m0 = [], 0
    for s in splits:
        parts.append(eigen.mc_cov(s, 42, T, seed=5, device=cuda, m0=m0))
        m0 += s
    assert torch.equal(full, torch.cat(parts))


@pytest.mark.gpu
@pytest.mark.parametrize("solver", sorted(eigen.BIAS_SOLVERS))
def test_hip_sharded_eigen_matches_one_shot(cuda, solver):
    """Chunked sum-accumulate + finalize kernels == the one-shot per-sim kernel (same Philox sims)."""
    _need_solver(solver)
    D, K, M = 10, 42, 20
    F = _spd(D, K, seed=4, spread=2.0) * 1e-4
    F[2] = float("nan")
    Fg = F.to(cuda)
    with eigen.using_bias_solver(solver):
        F1, v1 = eigen.eigen_risk_adjust(Fg, M=M, T_sim=400, seed=6, return_bias=True)
        F2, v2 = eigen.eigen_risk_adjust_sharded(Fg, M=M, T_sim=400, seed=6, chunk=7,
                                                 return_bias=True)
    torch.testing.assert_close(v2.cpu(), v1.cpu(), rtol=1e-12, atol=1e-14, equal_nan=True)
    torch.testing.assert_close(F2.cpu(), F1.cpu(), rtol=1e-11, atol=1e-18, equal_nan=True)


@pytest.mark.gpu
@pytest.mark.parametrize("mode", [21, 22, 23])
def test_bias_warm_date_chains_match_cold_solver(cuda, mode):
    from llm_driven_multi_factor_model_amd import _native as _n
    if mode != 21 and not _n.ab_build():
        pytest.skip("chains of 4 / 16 dates: A/B variants")
    """Bias modes 21 / 22 / 23: mode 5's kernel walking 8 / 4 / 16 consecutive dates of a sim
    per wave, each Laguerre iteration started from the previous date's eigenvalue of the same
    rank.  A slowly drifting spectrum (the Newey-West series), a NaN date inside a chain (the
    next date restarts cold) and a date count that is not a multiple of the chain: the same
    bias ratios as the cold-start mode 5 to the Laguerre stopping rounding."""
    import ctypes as C
    from llm_driven_multi_factor_model_amd import _native
    _native.register("mfa_eigen_set_bias_mode", [C.c_int])
    D, K, M = 45, 42, 12
    base = _spd(1, K, seed=21, spread=2.5)[0] * 1e-4
    g = torch.Generator().manual_seed(5)
    F = torch.empty(D, K, K, dtype=torch.float64)
    cur = base.clone()
    for d in range(D):  # a random walk of small symmetric perturbations
        E = torch.randn(K, K, generator=g, dtype=torch.float64) * 2e-10   # ||E|| ~ 3e-9 << 3e-7
        cur = cur + 0.5 * (E + E.T)
        F[d] = cur
    F[10] = float("nan")
    Cz = eigen.mc_cov(M, K, 2520, seed=9, device=cuda)
    lib = _native.lib()
    out = {}
    try:
        for md in (5, mode):
            assert lib.mfa_eigen_set_bias_mode(md) == 0
            out[md] = eigen.eigen_risk_adjust(F.to(cuda), Cz=Cz, return_bias=True)[1].cpu()
            # the sims-chunked accumulate path takes the same chains
            out[(md, "sh")] = eigen.eigen_risk_adjust_sharded(
                F.to(cuda), M=M, T_sim=2520, seed=9, chunk=5, return_bias=True)[1].cpu()
    finally:
        lib.mfa_eigen_set_bias_mode(5)
    assert torch.isnan(out[mode][10]).all() and torch.isfinite(out[mode][11:]).all()
    torch.testing.assert_close(out[mode], out[5], rtol=1e-12, atol=0, equal_nan=True)
    torch.testing.assert_close(out[(mode, "sh")], out[(5, "sh")], rtol=1e-12, atol=0, equal_nan=True)


@pytest.mark.gpu
@pytest.mark.parametrize("date0", [0, 8, 16])
def test_bias_date_chains_align_to_global_dates(cuda, date0):
    """The opt-in chained solver ("tridiag_chain"): a date block passed with its global offset
    (``date0``) that starts on a chain boundary (a multiple of 8) reproduces the one-process
    rows bit for bit -- chains start at global multiples of 8 -- and the sims-sharded
    accumulation path (all dates on every rank) takes the same chains."""
    D, K, M = 30, 42, 8
    base = _spd(1, K, seed=31, spread=2.5)[0] * 1e-4
    g = torch.Generator().manual_seed(8)
    F = torch.empty(D, K, K, dtype=torch.float64)
    cur = base.clone()
    for d in range(D):
        E = torch.randn(K, K, generator=g, dtype=torch.float64) * 2e-10
        cur = cur + 0.5 * (E + E.T)
        F[d] = cur
    Fg = F.to(cuda)
    Cz = eigen.mc_cov(M, K, 2520, seed=4, device=cuda)
    with eigen.using_bias_solver("tridiag_chain"):
        Fa, va = eigen.eigen_risk_adjust(Fg, Cz=Cz, return_bias=True)
        Fb, vb = eigen.eigen_risk_adjust(Fg[date0:], Cz=Cz, return_bias=True, date0=date0)
        Fs, vs = eigen.eigen_risk_adjust_sharded(Fg[date0:], M=M, T_sim=2520, seed=4, chunk=3,
                                                 return_bias=True, date0=date0)
        Ff, vf = eigen.eigen_risk_adjust_sharded(Fg, M=M, T_sim=2520, seed=4, chunk=3,
                                                 return_bias=True)
    assert torch.equal(vb, va[date0:]) and torch.equal(Fb, Fa[date0:])
    assert torch.equal(vs, vf[date0:])
