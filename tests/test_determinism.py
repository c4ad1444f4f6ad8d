"""Run-twice bitwise determinism of the whole risk model.

With ``RiskConfig(deterministic=True)`` every stage is order-fixed: the CS-WLS kernel's wave-owned
LDS replicas, the blocked Newey-West / VRA scans (no atomics), per-(date, sim) Jacobi solves
with Philox draws keyed by the sim index, and in-order bias sums.  Two runs must agree bit for
bit, NaN positions included.
"""
import pytest
import torch

from llm_driven_multi_factor_model_amd.models.panel import synthetic_panel
from llm_driven_multi_factor_model_amd.models.risk_model import RiskModel
from llm_driven_multi_factor_model_amd.utils.config import preset


def _outputs(m):
    return dict(f=m.factor_ret, e=m.specific_ret, r2=m.r2, nw=m.nw_cov, er=m.eigen_cov,
                vr=m.vra_cov, lam=m.vra_lambda, bias=m.eigen_bias)


def _bitwise_equal(a, b):
    return a.shape == b.shape and torch.equal(torch.isnan(a), torch.isnan(b)) and \
        torch.equal(a.nan_to_num(0.0), b.nan_to_num(0.0))


def _check(device, D, N, sims):
    p = synthetic_panel(D, N, 31, 10, seed=11, device=device, missing_frac=0.02, empty_industries=1)
    cfg = preset("reference", eigen_sims=sims, deterministic=True)
    a = _outputs(RiskModel(p, cfg).run())
    b = _outputs(RiskModel(p, cfg).run())
    for k in a:
        assert _bitwise_equal(a[k], b[k]), k


def test_risk_model_bitwise_deterministic_cpu():
    _check("cpu", 40, 200, 3)


@pytest.mark.gpu
def test_risk_model_bitwise_deterministic_gpu(cuda):
    _check(cuda, 300, 2000, 20)
