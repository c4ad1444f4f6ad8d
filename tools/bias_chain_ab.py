"""A/B of the warm-started date chains of the bias solver (bias modes 21 / 22 / 23 = mode 5
walking 8 / 4 / 16 consecutive dates per wave) against the cold-start mode 5, on the
pipeline's own inputs: the Newey-West series of RiskModel on the bench panel (fp64, 2520 dates
x 5000 stocks, K = 42, M = 100 sims, T_sim = 2520).  Rounds interleaved; prints one JSON line
per round and a summary with the min ms per mode, the max relative bias difference to mode 5
and to the CPU LAPACK path on a few dates.

    python tools/bias_chain_ab.py [MODES=5,21,22,23] [ROUNDS=3]
"""
import json
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from llm_driven_multi_factor_model_amd import _native  # noqa: E402
from llm_driven_multi_factor_model_amd.models.panel import synthetic_panel  # noqa: E402
from llm_driven_multi_factor_model_amd.models.risk_model import RiskModel  # noqa: E402
from llm_driven_multi_factor_model_amd.ops import eigen  # noqa: E402
from llm_driven_multi_factor_model_amd.utils.config import preset  # noqa: E402

dev = torch.device("cuda:0")
modes = [int(m) for m in os.environ.get("MODES", "5,21,22,23").split(",")]
rounds = int(os.environ.get("ROUNDS", "3"))
D = int(os.environ.get("D", "2520"))
p = synthetic_panel(D, 5000, 31, 10, seed=3, missing_frac=0.01, dtype=torch.float64, device=dev)
cfg = preset("reference")
m = RiskModel(p, cfg)
m.regress()
m.newey_west()
F = m.nw_cov.contiguous()
M, T = cfg.eigen_sims, D
Cz = eigen.mc_cov(M, p.K, T, seed=cfg.eigen_seed, device=dev)
lib = _native.lib()
e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
ts, vs = {md: [] for md in modes}, {}
try:
    for md in modes:  # warm-up + outputs
        assert lib.mfa_eigen_set_bias_mode(md) == 0, md
        vs[md] = eigen.eigen_risk_adjust(F, Cz=Cz, scale_coef=cfg.eigen_scale, return_bias=True)[1]
    for r in range(rounds):
        rec = {"round": r}
        for md in modes:
            lib.mfa_eigen_set_bias_mode(md)
            torch.cuda.synchronize()
            e0.record()
            eigen.eigen_risk_adjust(F, Cz=Cz, scale_coef=cfg.eigen_scale, return_bias=True)
            e1.record()
            e1.synchronize()
            ts[md].append(e0.elapsed_time(e1))
            rec[f"mode{md}_ms"] = round(ts[md][-1], 3)
        print(json.dumps(rec), flush=True)
finally:
    lib.mfa_eigen_set_bias_mode(5)
base = vs[modes[0]]
fin = torch.isfinite(base)
sel = [d for d in (300, 1000, 1800, D - 1) if d < D and bool(fin[d].all())]
Fc, vc = eigen.eigen_risk_adjust(F[sel].cpu(), Cz=Cz.cpu(), scale_coef=cfg.eigen_scale, return_bias=True)
out = {"D": D, "K": p.K, "M": M, "valid_dates": int(fin.all(-1).sum())}
for md in modes:
    v = vs[md]
    out[f"mode{md}_min_ms"] = round(min(ts[md]), 3)
    out[f"mode{md}_max_rel_vs_mode{modes[0]}"] = float(((v - base).abs() / base.abs())[fin].max())
    out[f"mode{md}_max_rel_vs_lapack"] = float(((v[sel].cpu() - vc).abs() / vc.abs()).max())
print(json.dumps(out), flush=True)
