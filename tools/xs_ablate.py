"""Interleaved A/B timing of xs_wls kernel variants (one process, rounds interleaved).

variant bits: 1 = skip segment LDS atomics, 2 = skip the style Gram FMAs, 4 = skip the residual
pass (timing only; results are garbage for variants != 0).
Env: VARIANTS (default 0,1,4,5), D, N.
"""
import os
import statistics
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from llm_driven_multi_factor_model_amd import _native  # noqa: E402
from llm_driven_multi_factor_model_amd.models.panel import synthetic_panel  # noqa: E402


def main():
    D, N, P, Q = int(os.environ.get("D", 2520)), int(os.environ.get("N", 5000)), 31, 10
    dev = torch.device("cuda:0")
    p = synthetic_panel(D, N, P, Q, seed=1, device=dev, missing_frac=0.01)
    K = 1 + P + Q
    f = torch.empty(D, K, dtype=torch.float64, device=dev)
    e = torch.empty(D, N, dtype=torch.float32, device=dev)
    r2 = torch.empty(D, dtype=torch.float64, device=dev)
    st = torch.empty(D, Q + 2, dtype=torch.float64, device=dev)
    s = torch.empty(D, dtype=torch.int32, device=dev)
    variants = [int(v) for v in os.environ.get("VARIANTS", "0,1,4,5").split(",")]
    ws = torch.empty(_native.query("mfa_xs_wls_workspace", D, N, P, Q), dtype=torch.uint8, device=dev)
    times = {v: [] for v in variants}
    ev0, ev1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    for rnd in range(12):
        for v in variants:
            ev0.record()
            for _ in range(5):
                _native.call("mfa_xs_wls_variant", _native.ptr(p.styles), _native.ptr(p.cap),
                             _native.ptr(p.ret), _native.ptr(p.ind), D, N, P, v,
                             _native.ptr(f), _native.ptr(e), _native.ptr(r2), _native.ptr(st),
                             _native.ptr(s), _native.ptr(ws), _native.stream(dev))
            ev1.record()
            ev1.synchronize()
            if rnd >= 2:
                times[v].append(ev0.elapsed_time(ev1) / 5)
    for v, t in times.items():
        print(f"variant {v}: median {statistics.median(t)*1e3:.1f} us  min {min(t)*1e3:.1f} us")


if __name__ == "__main__":
    main()
