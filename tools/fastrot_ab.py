"""A/B of the Jacobi rotation parameters: IEEE fp64 div/sqrt (0) vs rcp/rsq + Newton (1), for
the Monte-Carlo bias kernel (D x M 42x42 eigensolves) and the batched F0 eigh."""
import ctypes as C
import os
import sys
import time

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from llm_driven_multi_factor_model_amd import _native  # noqa: E402
from llm_driven_multi_factor_model_amd.ops import eigen  # noqa: E402

_native.register("mfa_eigen_set_fast_rotation", [C.c_int])
dev = torch.device("cuda:0")
D, K, M = 2520, 42, 100
g = torch.Generator().manual_seed(0)
X = torch.randn(D, 300, K, generator=g, dtype=torch.float64) * torch.logspace(-1, -3, K, dtype=torch.float64)
F0 = (X.transpose(1, 2) @ X / 300).to(dev)
Cz = eigen.mc_cov(M, K, D, 1, dev)
out = {}
for fast in (0, 1, 0, 1):
    _native.lib().mfa_eigen_set_fast_rotation(fast)
    Fh, v = eigen.eigen_risk_adjust(F0, M=M, Cz=Cz, return_bias=True)
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    for _ in range(3):
        Fh, v = eigen.eigen_risk_adjust(F0, M=M, Cz=Cz, return_bias=True)
    torch.cuda.synchronize()
    el = (time.perf_counter() - t0) / 3 * 1e3
    t1 = time.perf_counter()
    for _ in range(5):
        w, U = eigen.eigh(F0)
    torch.cuda.synchronize()
    el2 = (time.perf_counter() - t1) / 5 * 1e3
    out[fast] = (v.clone(), w.clone())
    print(f"fast={fast}: eigen_risk_adjust {el:.2f} ms   eigh(F0) {el2:.3f} ms")
_native.lib().mfa_eigen_set_fast_rotation(0)
dv = ((out[1][0] - out[0][0]).abs() / out[0][0].abs()).nan_to_num(0).max().item()
dw = ((out[1][1] - out[0][1]).abs() / out[0][1].abs().max(-1, keepdim=True).values).max().item()
print(f"max rel |dv| {dv:.2e}   max rel |dw| {dw:.2e}")
