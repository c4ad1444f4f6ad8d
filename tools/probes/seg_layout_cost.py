"""Cost of a standalone rolling-beta recompute on the segment layout (BASELINE config 4 shape,
5000 stocks x 3780 days): the layout build with its two input series, the kernel on a built
layout, and the whole call.  Wall-clock per call (synchronised), median of 20.

    python tools/probes/seg_layout_cost.py
    rocprofv3 --kernel-trace --stats -d gpurun_out/x -- python3 tools/probes/seg_layout_cost.py
"""
import json
import os
import statistics
import sys
import time

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__)))))
from llm_driven_multi_factor_model_amd.ops import rolling as RL  # noqa: E402

dev = torch.device("cuda:0")
N, T = 5000, 3780
g = torch.Generator(device=dev).manual_seed(0)
mkt = torch.randn(T, device=dev, generator=g) * 0.012
ret = (mkt[None, :] * 1.1 + torch.randn(N, T, device=dev, generator=g) * 0.02).reshape(-1).float()
mret = mkt[None, :].expand(N, T).reshape(-1).contiguous().float()
seg = RL.seg_lo_from_codes(torch.arange(N, device=dev, dtype=torch.int32).repeat_interleave(T))


def wall(fn, reps=20):
    fn()
    torch.cuda.synchronize()
    ts = []
    for _ in range(reps):
        t0 = time.perf_counter()
        fn()
        torch.cuda.synchronize()
        ts.append(time.perf_counter() - t0)
    return round(statistics.median(ts) * 1e3, 4)


lay = RL.SegLayout(seg, None, (ret, mret))
print(json.dumps({
    "rows": N * T,
    "layout_build_with_2_series_ms": wall(lambda: RL.SegLayout(seg, None, (ret, mret))),
    "layout_build_no_series_ms": wall(lambda: RL.SegLayout(seg, None)),
    "kernel_on_built_layout_ms": wall(lambda: RL.beta_hsigma(ret, mret, seg, 252, 63.0, 42, row_ord=lay)),
    "whole_call_ms": wall(lambda: RL.beta_hsigma(ret, mret, seg, 252, 63.0, 42)),
}), flush=True)
