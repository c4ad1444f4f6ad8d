"""Time the Monte-Carlo eigenfactor adjustment on D dates x M sims (K = 42)."""
import os
import sys
import time

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from llm_driven_multi_factor_model_amd.ops import eigen  # noqa: E402

D = int(sys.argv[1]) if len(sys.argv) > 1 else 2520
K, M = 42, 100
dev = torch.device("cuda:0")
g = torch.Generator().manual_seed(0)
X = torch.randn(D, 300, K, generator=g, dtype=torch.float64) * torch.logspace(-1, -3, K, dtype=torch.float64)
F0 = (X.transpose(1, 2) @ X / 300).to(dev)
Cz = eigen.mc_cov(M, K, D, 1, dev)
Fh, v = eigen.eigen_risk_adjust(F0, M=M, Cz=Cz, return_bias=True)
torch.cuda.synchronize()
t0 = time.perf_counter()
for _ in range(3):
    Fh, v = eigen.eigen_risk_adjust(F0, M=M, Cz=Cz, return_bias=True)
torch.cuda.synchronize()
el = (time.perf_counter() - t0) / 3
print(f"eigen_risk_adjust D={D} M={M} K={K}: {el*1e3:.2f} ms  ({D*M/el/1e6:.3f} M eigh/s)")
if len(sys.argv) > 2:
    Fr, vr = eigen.eigen_risk_adjust(F0[:4].cpu(), M=M, Cz=Cz.cpu(), T_sim=D, return_bias=True)
    print(f"max |v - v_cpu| = {(v[:4].cpu() - vr).abs().max():.3e}")
