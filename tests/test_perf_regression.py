"""Perf regression guards on 1x MI355X, at fixed shapes.

Thresholds are ~2.5-3x the measured steady-state numbers in profiles/ (bench: 0.275 ms per 2520
dates at N = 5000; MC eigen adjust 37 ms per 2520 x 100; as-of search 0.10 ms at 6.7 M rows),
so clock ramp or a noisy neighbour does not fail them, while a fallback to a slow path (e.g. the
split K1/K2/K3 kernels, an eager PyTorch path or a per-date loop) does."""
import pytest
import torch

pytestmark = pytest.mark.gpu


def _time_ms(fn, reps=10, warm=5):
    for _ in range(warm):
        fn()
    torch.cuda.synchronize()
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    e0.record()
    for _ in range(reps):
        fn()
    e1.record()
    torch.cuda.synchronize()
    return e0.elapsed_time(e1) / reps


def test_xs_wls_headline_shape_throughput():
    from llm_driven_multi_factor_model_amd.models.panel import synthetic_panel
    from llm_driven_multi_factor_model_amd.ops.cross_section import xs_wls, xs_wls_workspace
    D, N, P, Q = 1000, 5000, 31, 10
    g = synthetic_panel(D, N, P, Q, seed=0, missing_frac=0.02).to("cuda:0")
    ws = xs_wls_workspace(D, P, Q, "cuda:0", N)
    out = xs_wls(g.styles, g.cap, g.ret, g.ind, P, workspace=ws, refine=False)
    ms = _time_ms(lambda: xs_wls(g.styles, g.cap, g.ret, g.ind, P, out=out, workspace=ws, refine=False))
    reg_per_s = D / (ms * 1e-3)
    print(f"xs_wls {D}x{N}: {ms:.3f} ms, {reg_per_s / 1e6:.2f} M reg/s")
    assert reg_per_s > 3.0e6, f"{reg_per_s:.3g} reg/s"


def test_mc_eigen_adjust_throughput():
    from llm_driven_multi_factor_model_amd.ops import eigen
    D, K, M = 252, 42, 100
    gen = torch.Generator().manual_seed(0)
    X = torch.randn(D, 300, K, generator=gen, dtype=torch.float64) * torch.logspace(-1, -3, K, dtype=torch.float64)
    F0 = (X.transpose(1, 2) @ X / 300).to("cuda:0")
    Cz = eigen.mc_cov(M, K, D, 1, "cuda:0")
    ms = _time_ms(lambda: eigen.eigen_risk_adjust(F0, M=M, Cz=Cz), reps=3, warm=1)
    print(f"eigen_risk_adjust {D}x{M}: {ms:.2f} ms")
    assert ms < 15.0, f"{ms:.2f} ms"


def test_asof_search_throughput():
    from llm_driven_multi_factor_model_amd.ops import asof
    ng, days, nst = 5600, 1200, 20
    d = "cuda:0"
    lg = torch.arange(ng, dtype=torch.int32, device=d).repeat_interleave(days)
    lk = torch.arange(days, dtype=torch.int64, device=d).repeat(ng)
    rg = torch.arange(ng, dtype=torch.int32, device=d).repeat_interleave(nst)
    rk = torch.sort(torch.randint(0, days, (ng, nst), device=d), dim=1).values.reshape(-1)
    ms = _time_ms(lambda: asof.asof_search(lg, lk, rg, rk, check_sorted=False))
    print(f"asof_search {lg.numel()} x {rg.numel()}: {ms:.3f} ms")
    assert ms < 0.5, f"{ms:.3f} ms"
