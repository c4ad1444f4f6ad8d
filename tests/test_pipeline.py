"""Intra-GPU stage pipelining (parallel/pipeline.py): a host panel streamed through the GPU in
date chunks on h2d / compute / d2h streams equals one whole-panel xs_wls call."""
import pytest
import torch

from llm_driven_multi_factor_model_amd.models.panel import synthetic_panel
from llm_driven_multi_factor_model_amd.ops.cross_section import xs_wls, xs_wls_reference
from llm_driven_multi_factor_model_amd.parallel.pipeline import streamed_xs_wls


def test_cpu_device_is_reference_path():
    p = synthetic_panel(6, 64, 4, 3, seed=1, missing_frac=0.05)
    a = streamed_xs_wls(p.styles, p.cap, p.ret, p.ind, p.P, device="cpu", chunk=4)
    b = xs_wls_reference(p.styles, p.cap, p.ret, p.ind, p.P)
    torch.testing.assert_close(a.f, b.f, rtol=0, atol=0, equal_nan=True)


@pytest.mark.gpu
@pytest.mark.parametrize("chunk,depth,N", [(64, 3, 1000), (100, 2, 997), (1000, 3, 256)])
def test_streamed_equals_whole_panel(chunk, depth, N):
    p = synthetic_panel(333, N, 31, 10, seed=3, missing_frac=0.03, empty_industries=2)
    g = p.to("cuda:0")
    whole = xs_wls(g.styles, g.cap, g.ret, g.ind, p.P)
    s = streamed_xs_wls(p.styles, p.cap, p.ret, p.ind, p.P, device="cuda:0", chunk=chunk, depth=depth)
    torch.cuda.synchronize()
    assert s.f.device.type == "cpu" and s.f.is_pinned()
    torch.testing.assert_close(s.f, whole.f.cpu(), rtol=1e-12, atol=1e-14, equal_nan=True)
    torch.testing.assert_close(s.r2, whole.r2.cpu(), rtol=1e-12, atol=1e-14, equal_nan=True)
    torch.testing.assert_close(s.resid, whole.resid.cpu(), rtol=1e-5, atol=1e-7, equal_nan=True)
    assert torch.equal(s.status, whole.status.cpu())
