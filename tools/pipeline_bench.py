"""Host-resident panel (2520 dates x 5000 stocks, pinned) regressed on 1x MI355X:
serial (copy whole panel -> xs_wls -> copy results back) vs parallel/pipeline.streamed_xs_wls
(h2d / compute / d2h streams over date chunks)."""
import json
import sys
import time
from pathlib import Path

import torch

sys.path.insert(0, str(Path(__file__).resolve().parents[1]))
from llm_driven_multi_factor_model_amd.models.panel import synthetic_panel  # noqa: E402
from llm_driven_multi_factor_model_amd.ops.cross_section import xs_wls  # noqa: E402
from llm_driven_multi_factor_model_amd.parallel.pipeline import streamed_xs_wls  # noqa: E402

D, N = 2520, 5000
p = synthetic_panel(D, N, 31, 10, seed=0, missing_frac=0.02)
X, cap, ret, ind = (t.contiguous().pin_memory() for t in (p.styles, p.cap, p.ret, p.ind))
dev = torch.device("cuda:0")
in_bytes = sum(t.numel() * t.element_size() for t in (X, cap, ret, ind))


def serial():
    g = [t.to(dev, non_blocking=True) for t in (X, cap, ret, ind)]
    o = xs_wls(*g[:3], g[3], 31, refine=False)
    f = torch.empty(o.f.shape, dtype=o.f.dtype, pin_memory=True)
    r = torch.empty(o.resid.shape, dtype=o.resid.dtype, pin_memory=True)
    f.copy_(o.f, non_blocking=True)
    r.copy_(o.resid, non_blocking=True)
    torch.cuda.synchronize()
    return f


def timed(fn, reps=5):
    fn()
    torch.cuda.synchronize()
    ts = []
    for _ in range(reps):
        t0 = time.perf_counter()
        fn()
        torch.cuda.synchronize()
        ts.append((time.perf_counter() - t0) * 1e3)
    return min(ts)


res = {"dates": D, "stocks": N, "panel_MB": round(in_bytes / 1e6, 1), "serial_ms": round(timed(serial), 2)}
for chunk in (128, 256, 512):
    ms = timed(lambda: streamed_xs_wls(X, cap, ret, ind, 31, device=dev, chunk=chunk, depth=3, refine=False))
    res[f"streamed_chunk{chunk}_ms"] = round(ms, 2)
ref = serial()
s = streamed_xs_wls(X, cap, ret, ind, 31, device=dev, chunk=256, depth=3, refine=False)
res["max_abs_diff_f"] = float((s.f - ref).abs().nan_to_num().max())
res["h2d_GBps_serial"] = round(in_bytes / res["serial_ms"] / 1e6, 1)
print(json.dumps(res))
