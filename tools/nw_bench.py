"""Newey-West expanding series at the bench shape (T = 2520, K = 42): event timing per lag count
(q = 2 reference preset, 5 = USE4-S) and a short loop for rocprofv3 kernel stats."""
import json
import os
import statistics
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from llm_driven_multi_factor_model_amd.ops import ew_scan  # noqa: E402

dev = torch.device("cuda:0")
g = torch.Generator(device=dev).manual_seed(0)
T, K = int(os.environ.get("T", 2520)), 42
F = torch.randn(T, K, device=dev, dtype=torch.float64, generator=g) * 0.01
ev0, ev1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
for q in (2, 5, 10):
    V = ew_scan.newey_west_series(F, q, 252.0)
    Vr = ew_scan.newey_west_series_reference(F[:400].cpu(), q, 252.0) if q == 2 else None
    ts = []
    for _ in range(5):
        ev0.record()
        for _ in range(10):
            ew_scan.newey_west_series(F, q, 252.0)
        ev1.record()
        ev1.synchronize()
        ts.append(ev0.elapsed_time(ev1) / 10)
    err = None
    if Vr is not None:
        a, b = V[:400].cpu(), Vr
        err = ((a - b).abs().nan_to_num(0).max() / b.abs().nan_to_num(0).max()).item()
    print(json.dumps({"T": T, "K": K, "q": q, "ms": round(statistics.median(ts), 4), "max_rel_err_vs_cpu": err}), flush=True)
