"""Time the Monte-Carlo eigenfactor bias stage (eigen_risk_adjust) at several factor counts K.

    python tools/bias_k_bench.py [D] [K ...]        # default D = 2520, K = 9 16 25 32 42 45 48 64

One JSON line per K: ms per call (median of 5), problems per second, and a hash of the bias
ratios (a variant that claims bitwise-identical output must print the same hash).  The inputs
are Newey-West-like matrices (random 300-row panels with a log-spaced factor scale, seed 0)."""
import hashlib
import json
import os
import sys
import time

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from llm_driven_multi_factor_model_amd.ops import eigen  # noqa: E402

D = int(sys.argv[1]) if len(sys.argv) > 1 else 2520
Ks = [int(k) for k in sys.argv[2:]] or [9, 16, 25, 32, 42, 45, 48, 64]
M = 100
dev = torch.device("cuda:0")
for K in Ks:
    g = torch.Generator().manual_seed(0)
    X = torch.randn(D, 300, K, generator=g, dtype=torch.float64) * torch.logspace(-1, -3, K, dtype=torch.float64)
    F0 = (X.transpose(1, 2) @ X / 300).to(dev)
    Cz = eigen.mc_cov(M, K, D, 1, dev)
    Fh, v = eigen.eigen_risk_adjust(F0, M=M, Cz=Cz, return_bias=True)
    ts = []
    for _ in range(5):
        torch.cuda.synchronize()
        t0 = time.perf_counter()
        eigen.eigen_risk_adjust(F0, M=M, Cz=Cz, return_bias=True)
        torch.cuda.synchronize()
        ts.append(time.perf_counter() - t0)
    ms = sorted(ts)[2] * 1e3
    h = hashlib.sha1(v.cpu().numpy().tobytes()).hexdigest()[:12]
    print(json.dumps({"K": K, "D": D, "M": M, "ms": round(ms, 3), "Mproblems_per_s": round(D * M / ms / 1e3, 2),
                      "v_hash": h, "lib": os.environ.get("MFA_HIP_LIB", "production")}), flush=True)
