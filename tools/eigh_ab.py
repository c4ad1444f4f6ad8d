"""A/B of the batched F0 eigensolver: pair-block tournament Jacobi (mode 0) vs the row/column
cyclic Jacobi (mode 1), on Newey-West-like 42x42 covariances (D=2520) and odd K."""
import ctypes as C
import os
import sys
import time

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from llm_driven_multi_factor_model_amd import _native  # noqa: E402
from llm_driven_multi_factor_model_amd.ops import eigen  # noqa: E402

_native.register("mfa_eigh_set_mode", [C.c_int])
dev = torch.device("cuda:0")
g = torch.Generator(device=dev).manual_seed(0)
for K, D in ((42, 2520), (41, 512), (7, 512)):
    F = torch.randn(D, 300, K, device=dev, generator=g, dtype=torch.float64)
    F = F * torch.logspace(-3, 0, K, device=dev, dtype=torch.float64)  # spread spectrum
    A = F.transpose(1, 2) @ F / 300
    res = {}
    for mode in (1, 0):
        _native.lib().mfa_eigh_set_mode(mode)
        w, U = eigen.eigh(A)
        torch.cuda.synchronize()
        t0 = time.perf_counter()
        for _ in range(5):
            eigen.eigh(A)
        torch.cuda.synchronize()
        ms = (time.perf_counter() - t0) / 5 * 1e3
        rec = (U * w[:, None, :]) @ U.transpose(1, 2)
        err = ((rec - A).abs().max() / A.abs().max()).item()
        orth = (U.transpose(1, 2) @ U - torch.eye(K, device=dev, dtype=torch.float64)).abs().max().item()
        res[mode] = (ms, err, orth, w)
    _native.lib().mfa_eigh_set_mode(0)
    dw = ((res[0][3] - res[1][3]).abs().max() / res[1][3].abs().max()).item()
    print(f"K={K} D={D}: pairs {res[0][0]:.3f} ms (recon {res[0][1]:.1e}, orth {res[0][2]:.1e})  "
          f"rowcol {res[1][0]:.3f} ms (recon {res[1][1]:.1e})  max|dw|/|w| {dw:.1e}")
