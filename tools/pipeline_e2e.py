"""In-HBM end-to-end job (cli pipeline = main.py + demo.py without the CSV round trip) by phase,
on synthetic loader frames held in memory (non-I/O time only).

    python tools/pipeline_e2e.py [N] [T]      # default 5000 x 2520

The descriptors are the rank-invariant segment-anchored kernels (the only GPU path).  Prints one JSON line per timed run: descriptors (device factor engine incl. its host prep),
exposures -> RiskPanel scatter, RiskModel.run (all four stages), their sum (non_io_s).
"""
import json
import os
import sys
import time

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from llm_driven_multi_factor_model_amd.models import e2e  # noqa: E402
from llm_driven_multi_factor_model_amd.models import factor_engine as FE  # noqa: E402

N = int(sys.argv[1]) if len(sys.argv) > 1 else 5000
T = int(sys.argv[2]) if len(sys.argv) > 2 else 2520
dev = "cuda:0" if torch.cuda.is_available() else "cpu"
t0 = time.perf_counter()
prices, index, sw = FE.synthetic_prices_fast(N=N, T=T, seed=0, n_ind=31, suspend_frac=0.01)
# the stored loader panel's order, (ts_code, trade_date) -- the order FactorCalculator's
# _prepare_data sorts the master into -- so the reader's row-group index applies; the generator
# groups rows by stock in first-listed order
prices = prices.sort_values(["ts_code", "trade_date"], kind="stable").reset_index(drop=True)
gen_s = time.perf_counter() - t0
print(json.dumps({"rows": len(prices), "gen_s": round(gen_s, 2)}), flush=True)
cols = e2e._columns_from_frames(prices, index)
t0 = time.perf_counter()
cols = (e2e.stage_host_columns(cols[0]), cols[1])   # the native reader's output layout (I/O)
print(json.dumps({"stage_host_s": round(time.perf_counter() - t0, 3)}), flush=True)
small_p, small_i, small_sw = FE.synthetic_prices(N=60, T=300, seed=1, n_ind=31)
e2e.run_pipeline(small_p, small_i, small_sw, device=dev)  # warm-up: kernel load, allocator
from llm_driven_multi_factor_model_amd.utils import native_io  # noqa: E402
# reps 3 / 4: the same columns without the reader's row-group index (the key-based build:
# S16 codes uploaded, device unique of codes and dates)
for rep, ixd in ((0, True), (1, True), (2, True), (3, False), (4, False)):
    pc = dict(cols[0]) if ixd else {k: v for k, v in cols[0].items() if k != native_io.ROW_INDEX}
    t0 = time.perf_counter()
    model, info, _, t = e2e.run_pipeline(pc, dict(cols[1]), sw, device=dev)
    wall = time.perf_counter() - t0
    rec = {"N": N, "T": T, "D": model.panel.D, "K": model.K, "rep": rep,
           "row_index": ixd and native_io.ROW_INDEX in cols[0],
           **{k: round(v, 4) for k, v in t.items() if k.endswith("_s")}, "wall_s": round(wall, 4)}
    rec["non_io_s"] = round(sum(v for k, v in t.items() if k.endswith("_s")), 4)
    rec["kernel_ms"] = {k: round(v, 3) for k, v in t.get("kernel_ms", {}).items()}
    print(json.dumps(rec), flush=True)
