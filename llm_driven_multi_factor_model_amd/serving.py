"""Portfolio-risk serving: a fitted risk model's latest forecast held on the GPU, answering
batched portfolio queries (HTTP via FastAPI, or in-process).

The reference ends at CSV files (``Barra-master/demo.py:56-96``); a production user of a Barra
model then asks "what is the risk of this portfolio today?" many times per day.
:class:`RiskService` snapshots one date of a :class:`models.risk_model.RiskModel`:

* the exposure matrix ``X_d`` [N, K]: country, one-hot industry and cap-weighted z-scored
  styles, with the regression's own style means / pooled sigma (``XsResult.stats``);
* the factor covariance ``F_d`` [K, K] (VRA-adjusted by default);
* specific volatilities ``s`` [N] (cap-decile Bayesian shrinkage, ``utils.bayes_shrink``).

A query of B portfolios is two fp64 GEMMs on the device, ``x = H X_d`` and ``x F_d``, plus
``sum_i h_i^2 s_i^2``: batched, no per-portfolio Python loop.  A stock counts as held only if
its exposures exist on that date (finite styles and capital, a known industry).  The next-day
return is not required, unlike the regression universe.
"""
import logging

import numpy as np
import torch

from .ops import attribution as attr

log = logging.getLogger("mfa.serving")


class RiskService:
    def __init__(self, model, date_index: int = -1, which: str = "vra",
                 specific_vol: torch.Tensor | None = None):
        p = model.panel
        cov = {"nw": model.nw_cov, "eigen": model.eigen_cov, "vra": model.vra_cov}[which]
        if cov is None or model.stats is None:
            raise RuntimeError("run the risk model before serving it")
        d = date_index % p.D
        self.date = str(np.datetime_as_string(np.asarray(p.dates)[d], unit="D"))
        self.which = which
        self.P, self.Q, self.N = p.P, p.Q, p.N
        self.K = 1 + p.P + p.Q
        self.factor_names = list(p.factor_names)
        self.stocks = [str(s) for s in p.stocks]
        self._pos = {s: i for i, s in enumerate(self.stocks)}
        self.device = p.device
        self.X = self._exposure_matrix(p, model.stats[d], d)           # [N, K] fp64
        self.held_ok = torch.isfinite(self.X).all(1)
        self.X = torch.nan_to_num(self.X, nan=0.0)
        self.F = cov[d].to(torch.float64).contiguous()                  # [K, K]
        if specific_vol is None:
            specific_vol = model.specific_risk_shrunk()[d]   # point in time: date d's own
        s = specific_vol.to(self.device, torch.float64)
        self.s2 = torch.nan_to_num(s * s, nan=0.0)                     # [N]
        self.F_ok = bool(torch.isfinite(self.F).all())

    @staticmethod
    def _exposure_matrix(p, stats_d, d) -> torch.Tensor:
        Q, P = p.Q, p.P
        X = p.styles[d].to(torch.float64)                              # [Q, N]
        cap = p.cap[d]
        ok = torch.isfinite(X).all(0) & torch.isfinite(cap) & (cap >= 0)
        cols = [torch.ones(p.N, 1, dtype=torch.float64, device=X.device)]
        if P > 0:
            ind = p.ind[d].long()
            ok &= (ind >= 0) & (ind < P)
            cols.append(torch.nn.functional.one_hot(ind.clamp(0, P - 1), P).to(torch.float64))
        mu, sig = stats_d[:Q].to(torch.float64), stats_d[Q].to(torch.float64)
        cols.append(((X - mu[:, None]) / sig).T)
        M = torch.cat(cols, 1)
        return torch.where(ok[:, None], M, torch.full_like(M, float("nan")))

    # ------------------------------------------------------------------ queries
    def weights(self, portfolios: list[dict]) -> tuple[torch.Tensor, list[list[str]]]:
        """Dense [B, N] holdings from ``{stock: weight}`` dicts; unknown / unheld names are
        returned per portfolio (and carry no weight)."""
        H = np.zeros((len(portfolios), self.N), dtype=np.float64)
        unknown = []
        ok = self.held_ok.cpu().numpy()
        for b, pf in enumerate(portfolios):
            miss = []
            for name, w in pf.items():
                i = self._pos.get(str(name))
                if i is None or not ok[i]:
                    miss.append(str(name))
                else:
                    H[b, i] += float(w)
            unknown.append(miss)
        return torch.from_numpy(H).to(self.device), unknown

    def query(self, H: torch.Tensor) -> attr.RiskAttribution:
        """Risk of B portfolios ``H`` [B, N] (or [N]) on the snapshot date."""
        H = H.to(self.device, torch.float64)
        if H.dim() == 1:
            H = H[None]
        H = torch.where(self.held_ok[None, :], H, torch.zeros((), dtype=torch.float64, device=H.device))
        x = H @ self.X                                                  # [B, K]
        svar = (H * H) @ self.s2                                        # [B]
        return attr.risk_attribution(x, self.F.expand(H.shape[0], -1, -1), svar)

    def query_json(self, portfolios: list[dict]) -> list[dict]:
        H, unknown = self.weights(portfolios)
        r = self.query(H)
        g = r.grouped(self.P)
        out = []
        tv, fv, sv = (torch.sqrt(t).cpu().numpy() for t in (r.total_var, r.factor_var, r.specific_var))
        ex, ctb = r.exposure.cpu().numpy(), r.contrib.cpu().numpy()
        gs = {k: v.cpu().numpy() for k, v in g.items()}
        for b in range(len(portfolios)):
            out.append({
                "date": self.date, "covariance": self.which,
                "total_vol": float(tv[b]), "factor_vol": float(fv[b]), "specific_vol": float(sv[b]),
                "variance_share": {k: float(v[b]) for k, v in gs.items()},
                "exposure": dict(zip(self.factor_names, map(float, ex[b]))),
                "risk_contribution": dict(zip(self.factor_names, map(float, ctb[b]))),
                "ignored": unknown[b],
            })
        return out

    def info(self) -> dict:
        return {"date": self.date, "covariance": self.which, "stocks": self.N, "factors": self.K,
                "held_stocks": int(self.held_ok.sum()), "covariance_finite": self.F_ok,
                "device": str(self.device)}


def make_app(service: RiskService):
    """FastAPI app: ``GET /health``, ``GET /factors``, ``POST /risk`` with
    ``{"portfolios": [{"000001.SZ": 0.5, ...}, ...]}`` (or a single ``{"weights": {...}}``)."""
    # (no `from __future__ import annotations` in this module: FastAPI resolves the request
    # model from the live annotation of the nested route function)
    from fastapi import FastAPI, HTTPException
    from pydantic import BaseModel

    class RiskRequest(BaseModel):
        portfolios: list[dict[str, float]] | None = None
        weights: dict[str, float] | None = None

    app = FastAPI(title="MI355X Barra risk service")

    @app.get("/health")
    def health():
        return {"status": "ok", **service.info()}

    @app.get("/factors")
    def factors():
        return {"factors": service.factor_names}

    @app.post("/risk")
    def risk(req: RiskRequest):
        pfs = req.portfolios if req.portfolios is not None else ([req.weights] if req.weights else None)
        if not pfs:
            raise HTTPException(status_code=422, detail="give 'portfolios' or 'weights'")
        if len(pfs) > 65536:
            raise HTTPException(status_code=413, detail="at most 65536 portfolios per request")
        return {"results": service.query_json(pfs)}

    return app
