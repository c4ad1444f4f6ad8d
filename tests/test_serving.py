"""Portfolio-risk serving: batched in-process queries equal the model's own attribution, and the
HTTP API (FastAPI TestClient, no network) returns the same numbers."""
import numpy as np
import pytest
import torch

from llm_driven_multi_factor_model_amd.models.panel import synthetic_panel
from llm_driven_multi_factor_model_amd.models.risk_model import RiskModel
from llm_driven_multi_factor_model_amd.serving import RiskService, make_app
from llm_driven_multi_factor_model_amd.utils.config import preset


def _model(device="cpu"):
    p = synthetic_panel(60, 120, 5, 4, seed=3, device=device, missing_frac=0.03)
    return RiskModel(p, preset("reference", eigen_sims=4)).run()


def _check_against_model(m):
    svc = RiskService(m)
    N, D = m.panel.N, m.panel.D
    g = torch.Generator().manual_seed(0)
    H = torch.rand(3, N, generator=g, dtype=torch.float64).to(m.panel.device)
    H = H / H.sum(1, keepdim=True)
    got = svc.query(H)
    spec = m.specific_risk_shrunk()
    held = svc.held_ok
    for b in range(3):
        h = torch.where(held, H[b], torch.zeros_like(H[b]))
        ref = m.risk_attribution(h, specific_vol=spec)
        torch.testing.assert_close(got.total_var[b], ref.total_var[-1], rtol=1e-10, atol=1e-14)
        torch.testing.assert_close(got.exposure[b], ref.exposure[-1], rtol=1e-10, atol=1e-12)
        torch.testing.assert_close(got.contrib[b], ref.contrib[-1], rtol=1e-9, atol=1e-12)
    return svc


def test_service_matches_model_attribution_cpu():
    m = _model()
    # the last date's valid rows are the regression's rows here (no ret-only holes)
    svc = _check_against_model(m)
    assert svc.info()["held_stocks"] > 100


def test_http_api_roundtrip():
    from fastapi.testclient import TestClient
    m = _model()
    svc = RiskService(m)
    client = TestClient(make_app(svc))
    h = client.get("/health").json()
    assert h["status"] == "ok" and h["factors"] == 1 + 5 + 4
    assert client.get("/factors").json()["factors"][0] == "country"
    names = svc.stocks[:10]
    pf = {n: 0.1 for n in names}
    pf["NOT_A_STOCK"] = 0.5
    r = client.post("/risk", json={"portfolios": [pf, {names[0]: 1.0}]}).json()["results"]
    assert len(r) == 2 and "NOT_A_STOCK" in r[0]["ignored"]
    H, _ = svc.weights([pf])
    ref = svc.query(H)
    assert np.isclose(r[0]["total_vol"], float(torch.sqrt(ref.total_var[0])), rtol=1e-12)
    shares = r[0]["variance_share"]
    assert np.isclose(sum(shares.values()), 1.0)
    assert client.post("/risk", json={}).status_code == 422
    one = client.post("/risk", json={"weights": {names[0]: 1.0}}).json()["results"][0]
    assert np.isclose(one["total_vol"], r[1]["total_vol"], rtol=1e-12)


@pytest.mark.gpu
def test_service_matches_model_attribution_gpu(cuda):
    _check_against_model(_model(cuda))
