"""Phase ablation of the XL bias solver (A/B library: MFA_HIP_LIB=.../_lib/ab/libmfa_hip.so).

Times the K x K bias batch (252 dates x M sims) with each phase skipped in turn (results are
meaningless then; only the time is read): the difference to the full run is that phase's cost.
"""
import ctypes as C
import json
import os
import sys
import time

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from llm_driven_multi_factor_model_amd import _native  # noqa: E402
from llm_driven_multi_factor_model_amd.ops import eigen  # noqa: E402

_native.register("mfa_eigen_xl_set_ablation", [C.c_int])
dev = torch.device("cuda:0")
for K in [int(x) for x in os.environ.get("K", "150,200,256").split(",")]:
    D, M = 252, int(os.environ.get("M", "100"))
    g = torch.Generator(device=dev).manual_seed(K)
    X = torch.randn(D, K, 2 * K, generator=g, device=dev, dtype=torch.float64)
    w, _ = eigen.eigh(X @ X.transpose(1, 2) / (2 * K) * 1e-4)
    valid = torch.isfinite(w).all(-1)
    w = w.clamp_min(0.0).contiguous()
    Cz = eigen.mc_cov(M, K, 2 * K, seed=1, device=dev)
    rec = {"K": K, "D": D, "M": M}
    for name, bits in (("full", 0), ("no_householder_pass", 1), ("no_eigenvalues", 2),
                       ("no_vectors", 4), ("no_backtransform", 8), ("setup_only", 15)):
        assert _native.lib().mfa_eigen_xl_set_ablation(bits) == 0, "needs the A/B library"
        eigen._bias_sum_xl(w, valid, Cz)
        torch.cuda.synchronize()
        t0 = time.perf_counter()
        eigen._bias_sum_xl(w, valid, Cz)
        torch.cuda.synchronize()
        rec[name] = round((time.perf_counter() - t0) * 1e3, 2)
    _native.lib().mfa_eigen_xl_set_ablation(0)
    print(json.dumps(rec), flush=True)
