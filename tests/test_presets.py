"""Every RiskConfig preset builds and runs a RiskModel end to end (CPU here, GPU under -m gpu).

USE4-S runs a 5-lag Newey-West (MSCI USE4 Table 4.1); the reference's utils.Newey_West accepts
any q < T (Barra-master/mfm/utils.py:16-50), so no preset may be rejected by a lag limit.
"""
import pytest
import torch

from llm_driven_multi_factor_model_amd.models.panel import synthetic_panel
from llm_driven_multi_factor_model_amd.models.risk_model import RiskModel
from llm_driven_multi_factor_model_amd.ops import ew_scan
from llm_driven_multi_factor_model_amd.utils.config import PRESETS, preset


def _run(name, device):
    p = synthetic_panel(60, 96, P=5, Q=3, seed=4, missing_frac=0.01, device=device)
    over = {"eigen_sims": 8} if PRESETS[name].eigen_sims > 8 else {}
    cfg = preset(name, **over)
    m = RiskModel(p, cfg).run()
    return m, cfg


@pytest.mark.parametrize("name", sorted(PRESETS))
def test_preset_runs_cpu(name):
    m, cfg = _run(name, "cpu")
    assert m.nw_params == (cfg.nw_lags, cfg.nw_half_life)
    K = m.K
    # prefixes longer than q and K have finite covariances
    t0 = max(cfg.nw_lags, K) + 1
    assert torch.isfinite(m.nw_cov[t0:]).all()
    assert torch.isfinite(m.vra_cov[-1]).all()
    ref = ew_scan.newey_west_series_reference(m.factor_ret_global, cfg.nw_lags, cfg.nw_half_life)
    torch.testing.assert_close(m.nw_cov, ref, equal_nan=True)


@pytest.mark.gpu
@pytest.mark.parametrize("name", sorted(PRESETS))
def test_preset_runs_gpu(cuda, name):
    m, cfg = _run(name, cuda)
    t0 = max(cfg.nw_lags, m.K) + 1
    assert torch.isfinite(m.nw_cov[t0:]).all()
    assert torch.isfinite(m.vra_cov[-1]).all()
    ref = ew_scan.newey_west_series_reference(m.factor_ret_global.cpu(), cfg.nw_lags,
                                              cfg.nw_half_life)
    torch.testing.assert_close(m.nw_cov.cpu(), ref, rtol=1e-9, atol=1e-15, equal_nan=True)


def test_eigen_sims_mode_uses_newey_west_params():
    """eigen_shard='sims' rebuilds the NW series with the (q, tau) newey_west() used, not the
    config's."""
    p = synthetic_panel(50, 64, P=4, Q=3, seed=9)
    cfg = preset("bootstrap10k", eigen_sims=4)
    a = RiskModel(p, cfg)
    a.regress()
    a.newey_west(q=3, tau=40.0)
    a.eigen_adjust()
    b = RiskModel(p, preset("reference", eigen_sims=4, nw_lags=3, nw_half_life=40.0))
    b.regress()
    b.newey_west()
    b.eigen_adjust()
    torch.testing.assert_close(a.eigen_cov, b.eigen_cov, equal_nan=True)


def test_t_global_mismatch_rejected():
    p = synthetic_panel(20, 32, P=3, Q=2, seed=1)
    with pytest.raises(ValueError):
        RiskModel(p, T_global=25)
