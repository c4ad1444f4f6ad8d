"""End-to-end factor pipeline (main.py equivalent) wall time by phase on synthetic prices.

    python tools/factor_e2e.py [N] [T]

Phases: host prep (sort / merge / factorize, pandas), descriptors (HIP rolling + per-date
kernels, incl. host<->device copies), post-processing (winsorize / composite / orthogonalize),
Barra export (pandas).
"""
import json
import os
import sys
import time

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from llm_driven_multi_factor_model_amd.models import factor_engine as FE  # noqa: E402

N = int(sys.argv[1]) if len(sys.argv) > 1 else 300
T = int(sys.argv[2]) if len(sys.argv) > 2 else 1250
dev = "cuda:0" if torch.cuda.is_available() else "cpu"
t0 = time.perf_counter()
prices, index, sw = FE.synthetic_prices(N=N, T=T, seed=0, suspend_frac=0.02)
gen_s = time.perf_counter() - t0
FE.factor_pipeline(prices.head(2000), index, sw, device=dev)  # warm-up (kernel load, allocator)
res = {}
for rep in range(2):
    t = {}
    t0 = time.perf_counter()
    eng = FE.FactorEngine(prices, index, device=dev)
    t["prep_s"] = time.perf_counter() - t0
    t0 = time.perf_counter()
    raw = eng.run(FE.FACTORS_TO_RUN)
    t["descriptors_s"] = time.perf_counter() - t0
    t["descriptor_kernel_ms"] = {k: round(v, 3) for k, v in eng.timings.items()}
    t0 = time.perf_counter()
    cols = [c for c in raw.columns if c not in ("ts_code", "trade_date")]
    grid = FE._Grid(raw, eng.device)  # as factor_pipeline: one grid index, in-place steps
    w = FE.winsorize_frame(raw, cols, 2.5, device=dev, grid=grid, copy=False)
    c = FE.composite_frame(w, eng.cfg.composite, device=dev, copy=False)
    o = FE.orthogonalize_frame(c, eng.cfg.ortho, device=dev, grid=grid, copy=False)
    t["postprocess_s"] = time.perf_counter() - t0
    t0 = time.perf_counter()
    final, info = FE.barra_export(o, sw)
    t["export_s"] = time.perf_counter() - t0
    t["total_s"] = t["prep_s"] + t["descriptors_s"] + t["postprocess_s"] + t["export_s"]
    res = t
print(json.dumps({"N": N, "T": T, "rows": len(prices), "device": dev, "synth_s": round(gen_s, 2),
                  **{k: (round(v, 3) if isinstance(v, float) else v) for k, v in res.items()}}))
