"""cProfile of the factor pipeline's host phases (prep / post-processing / export) on the GPU
path, 1000 x 2520 synthetic prices by default: where the non-kernel time goes.

    python tools/factor_host_prof.py [N] [T]
"""
import contextlib
import cProfile
import io
import os
import pstats
import sys
import time

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from llm_driven_multi_factor_model_amd.models import factor_engine as FE  # noqa: E402

N = int(sys.argv[1]) if len(sys.argv) > 1 else 1000
T = int(sys.argv[2]) if len(sys.argv) > 2 else 2520
dev = "cuda:0"
prices, index, sw = FE.synthetic_prices(N=N, T=T, seed=0, suspend_frac=0.02)
with contextlib.redirect_stdout(io.StringIO()):
    FE.factor_pipeline(prices.head(2000), index, sw, device=dev)
profs, times = {}, {}


def phase(name, fn):
    torch.cuda.synchronize()
    p = cProfile.Profile()
    t0 = time.perf_counter()
    p.enable()
    with contextlib.redirect_stdout(io.StringIO()):
        out = fn()
    torch.cuda.synchronize()
    p.disable()
    times[name] = time.perf_counter() - t0
    profs[name] = p
    return out


for rep in range(2):
    eng = phase("prep", lambda: FE.FactorEngine(prices, index, device=dev))
    raw = phase("descriptors", lambda: eng.run(FE.FACTORS_TO_RUN))
    cols = [c for c in raw.columns if c not in ("ts_code", "trade_date")]

    def post():
        grid = FE._Grid(raw, eng.device)
        w = FE.winsorize_frame(raw, cols, 2.5, device=dev, grid=grid, copy=False)
        c = FE.composite_frame(w, eng.cfg.composite, device=dev, copy=False)
        return FE.orthogonalize_frame(c, eng.cfg.ortho, device=dev, grid=grid, copy=False)
    o = phase("post", post)
    phase("export", lambda: FE.barra_export(o, sw))
print({k: round(v, 3) for k, v in times.items()}, "total", round(sum(times.values()), 3))
for name, p in profs.items():
    s = io.StringIO()
    pstats.Stats(p, stream=s).sort_stats("tottime").print_stats(14)
    print(f"==== {name} ({times[name]:.3f} s)")
    print("\n".join(line[:170] for line in s.getvalue().splitlines()[6:24]))

# the pipeline entry point (single process: columnar fast path) end to end
for rep in range(2):
    torch.cuda.synchronize()
    p = cProfile.Profile()
    t0 = time.perf_counter()
    p.enable()
    with contextlib.redirect_stdout(io.StringIO()):
        final, info, tt = FE.factor_pipeline(prices, index, sw, device=dev)
    p.disable()
    wall = time.perf_counter() - t0
print("factor_pipeline (columnar)", {k: (round(v, 3) if isinstance(v, float) else v) for k, v in tt.items() if k != "kernel_ms"},
      "wall", round(wall, 3), "rows", len(final))
s = io.StringIO()
pstats.Stats(p, stream=s).sort_stats("tottime").print_stats(20)
print("\n".join(line[:170] for line in s.getvalue().splitlines()[6:30]))
