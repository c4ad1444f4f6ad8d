"""Sweeps the Monte-Carlo bias Jacobi needs on REAL pipeline inputs (Newey-West covariances of a
2520 x 5000 synthetic panel) vs the eigen_bench matrices: time and result at max_sweeps = s.

The smallest s whose output equals the s = 30 output is the sweep count the kernel uses.
"""
import os
import sys
import time

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from llm_driven_multi_factor_model_amd.models.panel import synthetic_panel  # noqa: E402
from llm_driven_multi_factor_model_amd.models.risk_model import RiskModel  # noqa: E402
from llm_driven_multi_factor_model_amd.ops import eigen  # noqa: E402
from llm_driven_multi_factor_model_amd.utils.config import preset  # noqa: E402

dev = torch.device("cuda:0")
D, M = 2520, 100
p = synthetic_panel(D, 5000, 31, 10, seed=3, device=dev, missing_frac=0.01)
m = RiskModel(p, preset("reference"))
m.regress()
m.newey_west()
nw = m.nw_cov.contiguous()
K = nw.shape[-1]
g = torch.Generator().manual_seed(0)
X = torch.randn(D, 300, K, generator=g, dtype=torch.float64) * torch.logspace(-1, -3, K, dtype=torch.float64)
bench = (X.transpose(1, 2) @ X / 300).to(dev)
Cz = eigen.mc_cov(M, K, D, 1, dev)
w, _ = eigen.eigh(nw)
ok = torch.isfinite(w).all(-1)
wv = w[ok]
print(f"NW inputs: {int(ok.sum())} finite dates; eigenvalue spread (max/min) median "
      f"{(wv[:, -1] / wv[:, 0].clamp_min(1e-300)).median().item():.3e}", flush=True)
for name, F0 in (("pipeline NW", nw), ("eigen_bench", bench)):
    eigen.MAX_SWEEPS = 30
    ref = eigen.eigen_risk_adjust(F0, M=M, Cz=Cz, return_bias=True)[1]
    for s in (2, 3, 4, 5, 6, 8, 30):
        eigen.MAX_SWEEPS = s
        v = eigen.eigen_risk_adjust(F0, M=M, Cz=Cz, return_bias=True)[1]
        torch.cuda.synchronize()
        t0 = time.perf_counter()
        for _ in range(2):
            v = eigen.eigen_risk_adjust(F0, M=M, Cz=Cz, return_bias=True)[1]
        torch.cuda.synchronize()
        ms = (time.perf_counter() - t0) / 2 * 1e3
        fin = torch.isfinite(ref)
        d = ((v - ref).abs() / ref.abs())[fin].max().item()
        print(f"{name:12s} max_sweeps={s:2d}: {ms:7.2f} ms   max rel |v - v30| {d:.2e}", flush=True)
