"""Sub-step times of the date-sharded exposures path on ONE process (no collectives):
full device engine, date_shard(lo, hi), descriptors on the shard, owned rows, post-processing.

    python tools/shard_prof.py [N] [T] [world] [rank]
"""
import json
import os
import sys
import time

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from llm_driven_multi_factor_model_amd.models import e2e  # noqa: E402
from llm_driven_multi_factor_model_amd.models import factor_engine as FE  # noqa: E402
from llm_driven_multi_factor_model_amd.parallel.dist import shard_range  # noqa: E402

N = int(sys.argv[1]) if len(sys.argv) > 1 else 5000
T = int(sys.argv[2]) if len(sys.argv) > 2 else 2520
world = int(sys.argv[3]) if len(sys.argv) > 3 else 4
rank = int(sys.argv[4]) if len(sys.argv) > 4 else 1
dev = torch.device("cuda:0")
prices, index, sw = FE.synthetic_prices_fast(N=N, T=T, seed=0, n_ind=31, suspend_frac=0.01)
p, i = e2e._columns_from_frames(prices, index)
p = e2e.stage_host_columns(p)
small = FE.synthetic_prices(N=60, T=300, seed=1, n_ind=31)
e2e.run_pipeline(*small, device=dev)
rec = {}


def tick(name, t0):
    torch.cuda.synchronize()
    rec[name] = round(time.perf_counter() - t0, 4)
    print(json.dumps({name: rec[name]}), flush=True)
    return time.perf_counter()


for rep in range(2):
    t = time.perf_counter()
    full = e2e.DeviceFactorEngine(dict(p), dict(i), device=dev)
    t = tick("full_engine", t)
    lo, hi = shard_range(full.D, rank, world)
    full.cashflow_ttm()
    t = tick("ttm_full", t)
    sh = full.date_shard(lo, hi)
    t = tick("date_shard", t)
    res = sh.compute(FE.FACTORS_TO_RUN)
    t = tick("compute_shard", t)
    rec["kernel_ms"] = sh.timings
    own = torch.nonzero(sh.own).flatten()
    res = {k: v[own] for k, v in res.items()}
    eng = sh.owned()
    t = tick("owned", t)
    col = FE.postprocess_columns(eng, res, eng.cfg)
    t = tick("postprocess", t)
    print(json.dumps({"rep": rep, "rows_full": full.R, "rows_shard": sh.R, "rows_own": eng.R,
                      **rec}), flush=True)
