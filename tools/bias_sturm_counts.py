"""Where the bias solver's Laguerre phase spends its Sturm evaluations: A/B mode 68 (the
production mode-5 kernel writing each eigenvalue rank's Sturm-evaluation count instead of its
ratio; A/B library) on the pipeline's own inputs (bench panel, 2520 dates x 5000 stocks, K = 42,
M = 100).  Reports the mean count per rank, the wave's critical path (max over the 42 ranks of a
problem) and which rank sets it.

    MFA_HIP_LIB=.../_lib/ab/libmfa_hip.so python tools/bias_sturm_counts.py   # env D=2520
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
D = int(os.environ.get("D", "2520"))
p = synthetic_panel(D, 5000, 31, 10, seed=3, missing_frac=0.01, dtype=torch.float64, device=dev)
cfg = preset("reference")
m = RiskModel(p, cfg)
m.regress()
m.newey_west()
F = m.nw_cov.contiguous()
K, M = p.K, cfg.eigen_sims
w, _ = eigen.eigh(F)
valid = torch.isfinite(w).all(-1)
Cz = eigen.mc_cov(M, K, D, seed=cfg.eigen_seed, device=dev)
lib = _native.lib()
assert _native.ab_build(), "needs the A/B library (MFA_HIP_LIB)"
ws = torch.empty(D * M * K, dtype=torch.float64, device=dev)
S = torch.zeros(D, K, dtype=torch.float64, device=dev)
dv = valid.to(torch.int32).contiguous()
wc = w.contiguous()
try:
    assert lib.mfa_eigen_set_bias_mode(68) == 0
    _native.call("mfa_eigen_bias_accumulate", _native.ptr(wc), _native.ptr(dv), D, K, M,
                 _native.ptr(Cz), eigen.MAX_SWEEPS, eigen.TOL, _native.ptr(ws), _native.ptr(S),
                 _native.stream(dev))
    torch.cuda.synchronize()
finally:
    lib.mfa_eigen_set_bias_mode(5)
c = ws.view(D, M, K)[valid].reshape(-1, K)          # [problems, rank] Sturm evaluations
mx, arg = c.max(-1)
tnorm = w[valid].abs().amax(-1)
rel = (w[valid] / tnorm[:, None])                    # eigenvalue / ||T|| of F0 (not of S C S)
out = {"D": D, "K": K, "M": M, "problems": int(c.shape[0]),
       "mean_per_rank": [round(float(x), 2) for x in c.mean(0)],
       "mean_max_per_problem": round(float(mx.float().mean()), 2),
       "mean_over_ranks": round(float(c.mean()), 2),
       "max_p50_p90_p99": [float(mx.float().quantile(q)) for q in (0.5, 0.9, 0.99)],
       "argmax_rank_hist": torch.bincount(arg, minlength=K).tolist(),
       "F0_smallest_eig_over_norm_p50": float(rel[:, -1].median())}
print(json.dumps(out), flush=True)
