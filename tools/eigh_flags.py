"""Tridiagonal eigh of the pipeline's Newey-West covariances (1 GPU): how many matrices the
orthogonality check sends to the Jacobi fallback, and the time of each eigh mode."""
import ctypes as C
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

_native.register("mfa_eigh_set_mode", [C.c_int])
dev = torch.device("cuda:0")
p = synthetic_panel(2520, 5000, 31, 10, seed=3, device=dev, missing_frac=0.01, dtype=torch.float64)
rm = RiskModel(p, preset("reference"))
rm.regress()
rm.newey_west()
F0 = rm.nw_cov.contiguous()
B, K = F0.shape[0], F0.shape[-1]
ok = torch.isfinite(F0.reshape(B, -1)).all(-1)
w = torch.empty(B, K, dtype=torch.float64, device=dev)
U = torch.empty(B, K, K, dtype=torch.float64, device=dev)
flags = torch.zeros(B, dtype=torch.int32, device=dev)
lib = _native.lib()
out = {"matrices": B, "finite": int(ok.sum())}
for mode in (2, 0):
    lib.mfa_eigh_set_mode(mode)
    run = lambda: _native.call("mfa_eigh_batched", _native.ptr(F0), B, K, 30, 1e-15, _native.ptr(w),  # noqa: E731
                               _native.ptr(U), _native.ptr(flags), _native.stream(dev))
    run()
    torch.cuda.synchronize()
    if mode == 2:
        out["flagged"] = int(flags[ok].sum())
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    e0.record()
    for _ in range(5):
        run()
    e1.record()
    torch.cuda.synchronize()
    out[f"mode{mode}_ms"] = round(e0.elapsed_time(e1) / 5, 3)
# the same eigenvalues, near-diagonal matrices (the bias solver's regime): convergence from the
# diagonal guesses is immediate there
wv, V = torch.linalg.eigh(F0[ok].cpu())
Qs, _ = torch.linalg.qr(torch.eye(K, dtype=torch.float64) + 0.02 * torch.randn(K, K, dtype=torch.float64))
Fd = ((Qs * wv[:, None, :]) @ Qs.T).to(dev).contiguous()
Bd = Fd.shape[0]
wd = torch.empty(Bd, K, dtype=torch.float64, device=dev)
Ud = torch.empty(Bd, K, K, dtype=torch.float64, device=dev)
fd = torch.zeros(Bd, dtype=torch.int32, device=dev)
lib.mfa_eigh_set_mode(2)
run = lambda: _native.call("mfa_eigh_batched", _native.ptr(Fd), Bd, K, 30, 1e-15, _native.ptr(wd),  # noqa: E731
                           _native.ptr(Ud), _native.ptr(fd), _native.stream(dev))
run()
torch.cuda.synchronize()
e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
e0.record()
for _ in range(5):
    run()
e1.record()
torch.cuda.synchronize()
out["near_diag_mode2_ms"] = round(e0.elapsed_time(e1) / 5, 3)
Fv = F0[ok].contiguous()
for Bs in (1, 8, 64, 256, 1024):
    run = lambda: _native.call("mfa_eigh_batched", _native.ptr(Fv), Bs, K, 30, 1e-15, _native.ptr(wd),  # noqa: E731
                               _native.ptr(Ud), _native.ptr(fd), _native.stream(dev))
    run()
    torch.cuda.synchronize()
    e0.record()
    for _ in range(5):
        run()
    e1.record()
    torch.cuda.synchronize()
    out[f"B{Bs}_ms"] = round(e0.elapsed_time(e1) / 5, 3)
print(json.dumps(out))
