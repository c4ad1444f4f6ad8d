"""K12 as-of join timing at the full-A panel size (get_data.ipynb#c4: 6,687,296 daily rows;
~5,600 stocks x 20 quarterly statements): host threaded join vs the HIP search + gather."""
import json
import sys
import time
from pathlib import Path

import numpy as np
import torch

sys.path.insert(0, str(Path(__file__).resolve().parents[1]))
from llm_driven_multi_factor_model_amd.ops import asof  # noqa: E402
from llm_driven_multi_factor_model_amd.utils import pit  # noqa: E402

rng = np.random.default_rng(0)
ng, days, nst = 5600, 1200, 20
lg = np.repeat(np.arange(ng, dtype=np.int32), days)
lk = np.tile(np.arange(days, dtype=np.int64), ng)
rg = np.repeat(np.arange(ng, dtype=np.int32), nst)
rk = np.sort(rng.integers(0, days, (ng, nst)), axis=1).reshape(-1).astype(np.int64)
vals = rng.standard_normal((len(rg), 8)).astype(np.float32)

t0 = time.perf_counter()
want = pit.asof_indices(lg, lk, rg, rk)
host_ms = (time.perf_counter() - t0) * 1e3

d = "cuda:0"
tl = [torch.from_numpy(a).to(d) for a in (lg, lk, rg, rk)]
tv = torch.from_numpy(vals).to(d)
for _ in range(3):
    idx = asof.asof_search(*tl, check_sorted=False)
    out = asof.asof_gather(tv, idx)
torch.cuda.synchronize()
n = 20
e0, e1, e2 = (torch.cuda.Event(enable_timing=True) for _ in range(3))
e0.record()
for _ in range(n):
    idx = asof.asof_search(*tl, check_sorted=False)
e1.record()
for _ in range(n):
    out = asof.asof_gather(tv, idx)
e2.record()
torch.cuda.synchronize()
ok = bool(np.array_equal(idx.cpu().numpy(), want))
res = {"rows_left": int(len(lg)), "rows_right": int(len(rg)), "host_join_ms": round(host_ms, 2),
       "gpu_search_ms": round(e0.elapsed_time(e1) / n, 4), "gpu_gather8_ms": round(e1.elapsed_time(e2) / n, 4),
       "exact_match": ok}
print(json.dumps(res))
assert ok
