"""A/B of the wide-K (K = 140) bias statistic: rocSOLVER batched syevd (through torch) vs the
multi-wave HIP solver (csrc/eigen_wide.hip), D dates x M sims, plus the max relative difference
of the per-date sums and the HIP solver's phase ablations.  Prints JSON lines."""
import json
import os
import sys
import time

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from llm_driven_multi_factor_model_amd.ops import eigen  # noqa: E402

K = int(os.environ.get("K", 140))
D = int(os.environ.get("D", 60))
M = int(os.environ.get("M", 100))
dev = torch.device("cuda:0")
g = torch.Generator(device=dev).manual_seed(1)
X = torch.randn(D, 2 * K + 50, K, device=dev, generator=g, dtype=torch.float64)
F = X.transpose(1, 2) @ X / X.shape[1]
w, _ = eigen.eigh(F)
valid = torch.isfinite(w).all(-1)
w = w.clamp_min(0.0).contiguous()
Cz = eigen.mc_cov(M, K, 300, seed=2, device=dev)
out = {}
for name in ("hip", "hip_pair", "rocsolver"):
    eigen.set_wide_kernel_layout("pair" if name == "hip_pair" else "row")
    with eigen.using_wide_bias_solver("hip" if name.startswith("hip") else name):
        S = eigen._bias_sum_wide(w, valid, Cz)  # warm-up (kernel load, workspace)
        torch.cuda.synchronize()
        t0 = time.perf_counter()
        S = eigen._bias_sum_wide(w, valid, Cz)
        torch.cuda.synchronize()
        ms = (time.perf_counter() - t0) * 1e3
    out[name] = S
    print(json.dumps({"solver": name, "K": K, "D": D, "M": M, "ms": round(ms, 2),
                      "us_per_problem": round(ms * 1e3 / (D * M), 3)}), flush=True)
eigen.set_wide_kernel_layout("pair")
for name in ("hip", "hip_pair"):
    rel = ((out[name] - out["rocsolver"]).abs() / out["rocsolver"].abs()).max().item()
    print(json.dumps({f"max_rel_{name}_vs_rocsolver": rel}), flush=True)
# phase ablations of the HIP solver (timing only, outputs meaningless): 1 = no Laguerre,
# 2 = no eigenvectors / back-transform, 3 = tridiagonalisation + setup, 4 = no Householder
import ctypes  # noqa: E402
from llm_driven_multi_factor_model_amd import _native  # noqa: E402
_native.register("mfa_eigen_wide_set_ablation", [ctypes.c_int])
abl_ms = {}
try:
    with eigen.using_wide_bias_solver("hip"):
        for layout in ("row", "pair"):
            eigen.set_wide_kernel_layout(layout)
            for abl in (0, 1, 2, 3, 4, 6, 1 << 4, 2 << 4, 3 << 4, 5 << 4):  # + multisection rounds
                _native.lib().mfa_eigen_wide_set_ablation(abl)
                eigen._bias_sum_wide(w, valid, Cz)
                torch.cuda.synchronize()
                t0 = time.perf_counter()
                eigen._bias_sum_wide(w, valid, Cz)
                torch.cuda.synchronize()
                abl_ms[f"{layout}_{abl}"] = round((time.perf_counter() - t0) * 1e3, 2)
finally:
    _native.lib().mfa_eigen_wide_set_ablation(0)
    eigen.set_wide_kernel_layout("pair")
print(json.dumps({"hip_ablation_ms": abl_ms}), flush=True)
# multisection rounds must not change the results beyond rounding
with eigen.using_wide_bias_solver("hip"):
    try:
        _native.lib().mfa_eigen_wide_set_ablation(3 << 4)
        S3 = eigen._bias_sum_wide(w, valid, Cz)
    finally:
        _native.lib().mfa_eigen_wide_set_ablation(0)
rel3 = ((S3 - out["rocsolver"]).abs() / out["rocsolver"].abs()).max().item()
print(json.dumps({"max_rel_hip_pair_3rounds_vs_rocsolver": rel3}), flush=True)

# eigh of the F0 batch itself (D matrices, K x K): multi-wave HIP solver vs rocSOLVER
Fb = F.repeat((2520 + D - 1) // D, 1, 1)[:2520].contiguous()
for name in ("hip", "rocsolver"):
    with eigen.using_wide_bias_solver(name):
        eigen.eigh(Fb)
        torch.cuda.synchronize()
        t0 = time.perf_counter()
        wq, Uq = eigen.eigh(Fb)
        torch.cuda.synchronize()
        ms = (time.perf_counter() - t0) * 1e3
    print(json.dumps({"eigh": name, "B": Fb.shape[0], "K": K, "ms": round(ms, 2)}), flush=True)
