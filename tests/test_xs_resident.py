"""Resident fused CS-WLS kernel (mode 30, ``xs_resident_kernel``): one 4-wave workgroup per CU
keeps the residual-pass inputs of its first tiles in LDS and AGPRs, so only the rest of the date
is re-read from HBM.  Its moments follow the deterministic fused kernel's order, so its factor
returns equal the LDS-DMA kernel's (mode 31) to the solve's rounding, and both match the fp64
oracle (reference semantics: Barra-master/mfm/CrossSection.py:57-108)."""
import ctypes as C

import pytest
import torch

from llm_driven_multi_factor_model_amd.models.panel import synthetic_panel
from llm_driven_multi_factor_model_amd.ops import cross_section as X


def _run(lib, mode, p, P, **kw):
    lib.mfa_xs_set_mode(mode)
    try:
        out = X.xs_wls(p.styles, p.cap, p.ret, p.ind, P, **kw)
        torch.cuda.synchronize()
    finally:
        lib.mfa_xs_set_mode(0)
    return out


@pytest.fixture
def lib(ab_lib):
    """The resident kernel measured slower than the LDS-DMA fused kernel (530 vs 378 us; its
    stream ablations, profiles/r05/README.md): an A/B-library variant."""
    from llm_driven_multi_factor_model_amd import _native
    _native.register("mfa_xs_set_mode", [C.c_int])
    return ab_lib


# N: 3000 = every tile resident; 5000 = the headline (4-5 re-read tiles per wave); 12000 = many
# re-read tiles (several trips of the re-read loop); 72 = two tiles, partial last tile
@pytest.mark.gpu
@pytest.mark.parametrize("N", [72, 3000, 5000, 12000])
def test_resident_kernel_matches_oracle_and_dma_kernel(cuda, lib, N):
    P = 31
    p = synthetic_panel(23, N, P, 10, seed=N, missing_frac=0.03, empty_industries=1,
                        dtype=torch.float64)
    ref = X.xs_wls_reference(p.styles, p.cap, p.ret, p.ind, P)
    g = p.to(cuda)
    res = _run(lib, 30, g, P)
    dma = _run(lib, 31, g, P)
    torch.testing.assert_close(res.f.cpu(), ref.f, rtol=1e-9, atol=1e-12)
    torch.testing.assert_close(res.resid.cpu(), ref.resid, rtol=1e-9, atol=1e-13, equal_nan=True)
    torch.testing.assert_close(res.r2.cpu(), ref.r2, rtol=1e-9, atol=1e-12)
    torch.testing.assert_close(res.f, dma.f, rtol=1e-12, atol=1e-15)
    torch.testing.assert_close(res.resid, dma.resid, rtol=1e-12, atol=1e-15, equal_nan=True)
    torch.testing.assert_close(res.r2, dma.r2, rtol=1e-12, atol=1e-14)
    assert torch.equal(res.status, dma.status)
    # NaN exactly where the stock is invalid
    assert torch.equal(res.resid.isnan(), dma.resid.isnan())


@pytest.mark.gpu
def test_resident_kernel_is_bitwise_deterministic(cuda, lib):
    p = synthetic_panel(300, 5000, 31, 10, seed=9, missing_frac=0.02,
                        dtype=torch.float64).to(cuda)
    a = _run(lib, 30, p, 31)
    b = _run(lib, 30, p, 31)
    assert torch.equal(a.f, b.f) and torch.equal(a.r2, b.r2)
    assert torch.equal(a.resid.nan_to_num(7.0), b.resid.nan_to_num(7.0))


@pytest.mark.gpu
def test_resident_kernel_no_industries(cuda, lib):
    """P = 0: a single segment, no industry ids."""
    p = synthetic_panel(9, 5000, 0, 10, seed=4, missing_frac=0.01, dtype=torch.float64)
    ref = X.xs_wls_reference(p.styles, p.cap, p.ret, p.ind, 0)
    g = p.to(cuda)
    res = _run(lib, 30, g, 0)
    torch.testing.assert_close(res.f.cpu(), ref.f, rtol=1e-9, atol=1e-12)
    torch.testing.assert_close(res.resid.cpu(), ref.resid, rtol=1e-9, atol=1e-13, equal_nan=True)


@pytest.mark.gpu
def test_resident_kernel_feeds_the_device_refine(cuda, lib):
    """A near-singular date (two identical styles) is flagged by the solve and re-solved by the
    device pinv from the moments the resident kernel exports."""
    P = 31
    p = synthetic_panel(6, 5000, P, 10, seed=3, missing_frac=0.01, dtype=torch.float64)
    p.styles[2, 4] = 2.0 * p.styles[2, 1]
    ref = X.xs_wls_reference(p.styles, p.cap, p.ret, p.ind, P)
    g = p.to(cuda)
    out = _run(lib, 30, g, P, refine=True)
    assert int(out.status[2]) & 32, "date 2 should be refined on the device"
    torch.testing.assert_close(out.f.cpu(), ref.f, rtol=1e-8, atol=1e-11)
    torch.testing.assert_close(out.resid.cpu(), ref.resid, rtol=1e-8, atol=1e-12, equal_nan=True)
