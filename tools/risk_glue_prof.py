"""Which torch (at::native) operators run inside ``RiskModel.run`` and what they cost.

torch.profiler over one warm ``RiskModel.run`` (2520 dates x 5000 stocks by default): prints
the operators by self device time with their Python call sites, plus the total device time of
the HIP kernels of this library vs everything else ("glue").
"""
import argparse
import os
import sys

import torch
from torch.profiler import ProfilerActivity, profile

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from llm_driven_multi_factor_model_amd.models.panel import synthetic_panel  # noqa: E402
from llm_driven_multi_factor_model_amd.models.risk_model import RiskModel  # noqa: E402
from llm_driven_multi_factor_model_amd.utils.config import preset  # noqa: E402

ap = argparse.ArgumentParser()
ap.add_argument("--dates", type=int, default=2520)
ap.add_argument("--stocks", type=int, default=5000)
ap.add_argument("--storage", default="fp64")
a = ap.parse_args()
dev = torch.device("cuda:0")
dt = torch.float64 if a.storage == "fp64" else torch.float32
p = synthetic_panel(a.dates, a.stocks, 31, 10, seed=3, device=dev, missing_frac=0.01, dtype=dt)
cfg = preset("reference")
RiskModel(p, cfg, sync_stages=False).run()  # warm (library load, workspaces, clocks)
torch.cuda.synchronize()
with profile(activities=[ProfilerActivity.CPU, ProfilerActivity.CUDA], with_stack=True) as prof:
    m = RiskModel(p, cfg, sync_stages=False).run()
    torch.cuda.synchronize()
ev = prof.key_averages(group_by_stack_n=4)
rows = sorted(ev, key=lambda e: -e.self_device_time_total)
print(f"{'self dev us':>12} {'calls':>6}  op / stack")
for e in rows[:40]:
    if e.self_device_time_total <= 0:
        continue
    st = " <- ".join(s.split("/")[-1] for s in (e.stack or [])[:4])
    print(f"{e.self_device_time_total:12.1f} {e.count:6d}  {e.key[:60]}  [{st[:150]}]")
kern = [e for e in prof.events() if e.device_type == torch.autograd.DeviceType.CUDA]
ours = sum(e.self_device_time_total for e in kern if "anonymous namespace" in e.name or "mfa" in e.name)
tot = sum(e.self_device_time_total for e in kern)
print(f"device time: total {tot / 1e3:.2f} ms, library kernels {ours / 1e3:.2f} ms, "
      f"glue {(tot - ours) / 1e3:.3f} ms")
