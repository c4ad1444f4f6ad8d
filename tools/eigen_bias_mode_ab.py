"""A/B of the bias-Jacobi LDS layout (mfa_eigen_set_bias_mode): 0 = packed (A, M) double2,
1 = split fp64 A / fp64 M arrays, 2 = split with fp32 storage of M.  D dates x M sims, K = 42,
Newey-West-like clustered spectra (the pipeline's inputs need 6 sweeps)."""
import ctypes as C
import json
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from llm_driven_multi_factor_model_amd import _native  # noqa: E402
from llm_driven_multi_factor_model_amd.ops import eigen  # noqa: E402

D = int(sys.argv[1]) if len(sys.argv) > 1 else 2520
K, M = 42, 100
dev = torch.device("cuda:0")
g = torch.Generator().manual_seed(0)
X = torch.randn(D, 300, K, generator=g, dtype=torch.float64) * torch.logspace(-1, -3, K, dtype=torch.float64)
F0 = (X.transpose(1, 2) @ X / 300).to(dev)
Cz = eigen.mc_cov(M, K, D, 1, dev)
lib = _native.lib()
lib.mfa_eigen_set_bias_mode.argtypes = [C.c_int]
out, base = {"D": D, "M": M, "K": K}, None
for mode in (0, 1, 2, 0):
    lib.mfa_eigen_set_bias_mode(mode)
    Fh, v = eigen.eigen_risk_adjust(F0, M=M, Cz=Cz, return_bias=True)
    torch.cuda.synchronize()
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    e0.record()
    for _ in range(3):
        Fh, v = eigen.eigen_risk_adjust(F0, M=M, Cz=Cz, return_bias=True)
    e1.record()
    torch.cuda.synchronize()
    ms = e0.elapsed_time(e1) / 3
    if base is None:
        base = v.clone()
    rel = ((v - base).abs() / base.abs()).max().item()
    out[f"mode{mode}_ms"] = round(ms, 3)
    out[f"mode{mode}_max_rel_vs_mode0"] = rel
    print(json.dumps(out), flush=True)
lib.mfa_eigen_set_bias_mode(0)
