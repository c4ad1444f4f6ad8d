"""Time the rolling-descriptor kernels on a flat stock-sorted panel (N stocks x T days).

BASELINE.md: the reference's rolling BETA/HSIGMA runs at ~1.2k stock-days/s (a lower bound),
RSTR / DASTD / CMRA at 8.6 / 9.1 / 2.7 s per 30k stock-days.
"""
import json
import os
import sys
import time

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from llm_driven_multi_factor_model_amd.ops import rolling as RL  # noqa: E402

N = int(sys.argv[1]) if len(sys.argv) > 1 else 5000
T = int(sys.argv[2]) if len(sys.argv) > 2 else 3780
dev = torch.device("cuda:0")
g = torch.Generator(device=dev).manual_seed(0)
R = N * T
mkt = torch.randn(T, device=dev, generator=g) * 0.012
ret = (mkt[None, :] * 1.1 + torch.randn(N, T, device=dev, generator=g) * 0.02).reshape(-1).float()
ret[torch.rand(R, device=dev, generator=g) < 0.02] = float("nan")  # suspensions
mret = mkt[None, :].expand(N, T).reshape(-1).contiguous().float()
lr = torch.log1p(ret)
turn = torch.rand(R, device=dev, generator=g) * 5
stock = torch.arange(N, device=dev, dtype=torch.int32).repeat_interleave(T)
seg_lo = RL.seg_lo_from_codes(stock)

lay = RL.SegLayout(seg_lo)   # built once per engine (the segment layout + virtual inputs)
cases = {
    "beta_hsigma": lambda: RL.beta_hsigma(ret, mret, seg_lo, 252, 63.0, 42, row_ord=lay),
    "rstr": lambda: RL.rstr(lr, seg_lo, 504, 21, 126.0, 42, row_ord=lay),
    "dastd": lambda: RL.dastd(ret, mret, seg_lo, 252, 42.0, 42, row_ord=lay),
    "cmra": lambda: RL.cmra(lr, seg_lo, 252, row_ord=lay),
    "cmra_partial": lambda: RL.cmra(lr, seg_lo, 252, partial=True),
    "liquidity_3sums": lambda: RL.window_sums(turn, seg_lo, [(21, 15), (63, 42), (252, 126)], 0.01,
                                              log=True, row_ord=lay),
    "stom": lambda: RL.rolling_sum(turn, seg_lo, 21, 15, 0.01, log=True, row_ord=lay),
    "stoa": lambda: RL.rolling_sum(turn, seg_lo, 252, 126, 0.01, log=True, row_ord=lay),
}


def run(direct):
    res, outs = {}, {}
    with RL.direct_kernels(direct):
        for name, fn in cases.items():
            outs[name] = fn()
            torch.cuda.synchronize()
            t0 = time.perf_counter()
            for _ in range(5):
                fn()
            torch.cuda.synchronize()
            el = (time.perf_counter() - t0) / 5
            res[name] = {"ms": round(el * 1e3, 3), "Mstock_days_per_s": round(R / el / 1e6, 1)}
    return res, outs


torch.cuda.synchronize()
t0 = time.perf_counter()
for _ in range(3):
    RL.SegLayout(seg_lo).virt(ret)
torch.cuda.synchronize()
layout_ms = (time.perf_counter() - t0) / 3 * 1e3
direct, od = run(True)
scan, os_ = run(False)
agree = {}
for name in cases:
    a, b = od[name], os_[name]
    a = tuple(a) if isinstance(a, (tuple, list)) else (a,)
    b = tuple(b) if isinstance(b, (tuple, list)) else (b,)
    worst = 0.0
    for x, y in zip(a, b):
        same_nan = bool((torch.isnan(x) == torch.isnan(y)).all())
        m = torch.isfinite(x) & torch.isfinite(y)
        rel = ((x[m].double() - y[m].double()).abs() / y[m].double().abs().clamp_min(1e-6)).max().item()
        worst = max(worst, rel if same_nan else float("inf"))
    agree[name] = worst
print(json.dumps({"N": N, "T": T, "stock_days": R, "Rv": lay.Rv, "layout_plus_one_series_ms": round(layout_ms, 3),
                  "kernels": scan, "direct_kernels": direct, "seg_vs_direct_max_rel": agree}))
