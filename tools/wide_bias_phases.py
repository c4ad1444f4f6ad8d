"""Phase ablations of the production K > 96 bias solver (mc_bias_wide2_kernel<144, 5>) on the
risk model's own inputs: the Newey-West covariances of a P = K - 17 / Q = 16 panel (252 dates x
5000 stocks), M = 100 draws.  abl bits (mfa_eigen_wide_set_ablation, timing only, outputs
meaningless): 1 = no Laguerre iterations, 2 = no eigenvectors / back-transform, 4 = no
tridiagonalisation.  Interleaved rounds; prints JSON lines and the min ms per setting.

    python tools/wide_bias_phases.py        # env: K=140 D=252
    LAYOUTS=mixed,pair K=80 python tools/wide_bias_phases.py   # full solver per kernel layout
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
K = int(os.environ.get("K", "140"))
D = int(os.environ.get("D", "252"))
p = synthetic_panel(D, 5000, K - 17, 16, seed=3, missing_frac=0.01, dtype=torch.float64, device=dev)
cfg = preset("reference")
m = RiskModel(p, cfg)
m.regress()
m.newey_west()
F = m.nw_cov.contiguous()
w, _ = eigen.eigh(F)
valid = torch.isfinite(w).all(-1)
w = torch.where(valid[:, None], w.clamp_min(0.0), w).contiguous()
Cz = eigen.mc_cov(cfg.eigen_sims, K, D, seed=cfg.eigen_seed, device=dev)
lib = _native.lib()
e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
if os.environ.get("LAYOUTS"):  # full solver per kernel layout, results compared to the first
    names = os.environ["LAYOUTS"].split(",")
    out, tl = {}, {n: [] for n in names}
    try:
        for rd in range(4):
            for n in names:
                eigen.set_wide_kernel_layout(n)
                torch.cuda.synchronize()
                e0.record()
                out[n] = eigen._bias_sum_wide(w, valid, Cz)
                e1.record()
                e1.synchronize()
                if rd:
                    tl[n].append(e0.elapsed_time(e1))
    finally:
        eigen.set_wide_kernel_layout("pair")
    ref = out[names[0]]
    for n in names:
        fin = torch.isfinite(ref)
        rel = float(((out[n] - ref).abs() / ref.abs().clamp_min(1e-300))[fin].max())
        print(json.dumps({"K": K, "D": D, "layout": n, "ms": sorted(round(t, 3) for t in tl[n]),
                          "max_rel_vs_" + names[0]: rel}), flush=True)
    sys.exit(0)
# SETTINGS=0,16,32: multisection rounds (bits 4-6) instead of the phase ablations
settings = [int(a) for a in os.environ.get("SETTINGS", "0,1,2,4").split(",")]
ts = {a: [] for a in settings}
try:
    for a in settings:
        lib.mfa_eigen_wide_set_ablation(a)
        eigen._bias_sum_wide(w, valid, Cz)
    for rd in range(3):
        rec = {"round": rd}
        for a in settings:
            lib.mfa_eigen_wide_set_ablation(a)
            torch.cuda.synchronize()
            e0.record()
            eigen._bias_sum_wide(w, valid, Cz)
            e1.record()
            e1.synchronize()
            ts[a].append(e0.elapsed_time(e1))
            rec[f"abl{a}_ms"] = round(ts[a][-1], 3)
        print(json.dumps(rec), flush=True)
finally:
    lib.mfa_eigen_wide_set_ablation(0)
print(json.dumps({"K": K, "D": D, "valid_dates": int(valid.sum()),
                  **{f"abl{a}_min_ms": round(min(ts[a]), 3) for a in settings}}), flush=True)
