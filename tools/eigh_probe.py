"""Batched 42x42 eigh: sweep counts and time of the Jacobi kernel vs torch.linalg.eigh (GPU)."""
import os
import sys
import time

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from llm_driven_multi_factor_model_amd import _native  # noqa: E402
from llm_driven_multi_factor_model_amd.ops import eigen  # noqa: E402

dev = torch.device("cuda:0")
K, M, D = 42, 100, int(sys.argv[1]) if len(sys.argv) > 1 else 64
g = torch.Generator().manual_seed(0)
d0 = torch.logspace(-2, -6, K, dtype=torch.float64)  # factor-variance-like spectrum
Cz = eigen.mc_cov(M, K, 2520, 1, dev)
S = d0.sqrt().to(dev)
Cb = (S[None, :, None] * Cz * S[None, None, :]).repeat(D, 1, 1, 1).reshape(-1, K, K).contiguous()
B = Cb.shape[0]
w = torch.empty(B, K, dtype=torch.float64, device=dev)
U = torch.empty(B, K, K, dtype=torch.float64, device=dev)
sw = torch.empty(B, dtype=torch.int32, device=dev)


def run(ms, tol):
    _native.call("mfa_eigh_batched", _native.ptr(Cb), B, K, ms, tol, _native.ptr(w), _native.ptr(U),
                 _native.ptr(sw), _native.stream(dev))


for ms, tol in [(30, 1e-15), (30, 1e-14), (30, 1e-13)]:
    run(ms, tol)
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    run(ms, tol)
    torch.cuda.synchronize()
    el = time.perf_counter() - t0
    h = torch.bincount(sw.cpu().long(), minlength=31)
    wr, Ur = torch.linalg.eigh(Cb[:64].cpu())
    err = (w[:64].cpu() - wr.flip(-1)).abs().max() / wr.abs().max()
    print(f"max_sweeps {ms} tol {tol:g}: {el*1e3:.2f} ms for {B} eighs ({el/B*1e6:.2f} us each); "
          f"sweeps hist {dict((i, int(c)) for i, c in enumerate(h) if c)}; rel eig err {err:.2e}")
torch.cuda.synchronize()
t0 = time.perf_counter()
wt, Ut = torch.linalg.eigh(Cb)
torch.cuda.synchronize()
print(f"torch.linalg.eigh (GPU): {(time.perf_counter()-t0)*1e3:.2f} ms for {B}")
