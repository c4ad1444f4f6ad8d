"""Batched 140 x 140 symmetric eigensolvers on 1 GPU: torch.linalg.eigh vs rocSOLVER strided
batched syevd / syevj (ops/rocsolver.py).  Prints ms per batch and the max eigenvalue / bias
differences vs torch."""
import json
import os
import sys
import time

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from llm_driven_multi_factor_model_amd.ops import rocsolver  # noqa: E402

dev = torch.device("cuda:0")
K = int(os.environ.get("K", 140))
for B in [int(x) for x in os.environ.get("B", "100,1000,6800").split(",")]:
    g = torch.Generator(device=dev).manual_seed(0)
    X = torch.randn(B, K, 2 * K, generator=g, device=dev, dtype=torch.float64)
    A = X @ X.transpose(1, 2) / (2 * K)
    rec = {"B": B, "K": K}
    outs = {}
    for name in ("torch", "syevd", "syevj"):
        def run():
            if name == "torch":
                return torch.linalg.eigh(A)
            w, V, info = rocsolver.syev_batched(A, name)
            return w, V
        run()
        torch.cuda.synchronize()
        t0 = time.perf_counter()
        for _ in range(3):
            outs[name] = run()
        torch.cuda.synchronize()
        rec[f"{name}_ms"] = round((time.perf_counter() - t0) / 3 * 1e3, 2)
    for name in ("syevd", "syevj"):
        w, V = outs[name]
        rec[f"{name}_dw"] = float((w - outs["torch"][0]).abs().max() / outs["torch"][0].abs().max())
        rec[f"{name}_resid"] = float(((A @ V) - V * w[:, None, :]).abs().max())
    print(json.dumps(rec), flush=True)
