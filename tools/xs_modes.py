"""Interleaved A/B timing of the CS-WLS execution modes (one process, rounds interleaved).

mode 0 = fused single kernel (moments -> solve -> residuals per workgroup), mode 1 = the three
separate kernels.  Both must give the same factor returns; the script checks that first.
Env: D, N, SORT=1 orders the panel's stocks by industry (models.panel.order_by_industry).
"""
import ctypes as C
import os
import statistics
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from llm_driven_multi_factor_model_amd import _native  # noqa: E402
from llm_driven_multi_factor_model_amd.models import panel as pn  # noqa: E402
from llm_driven_multi_factor_model_amd.ops.cross_section import xs_wls, xs_wls_workspace  # noqa: E402

_native.register("mfa_xs_set_mode", [C.c_int])


def main():
    D, N, P, Q = int(os.environ.get("D", 2520)), int(os.environ.get("N", 5000)), 31, 10
    dev = torch.device("cuda:0")
    p = pn.synthetic_panel(D, N, P, Q, seed=1, device=dev, missing_frac=0.01)
    if os.environ.get("SORT", "0") == "1" and hasattr(pn, "order_by_industry"):
        p = pn.order_by_industry(p)
    ws = xs_wls_workspace(D, P, Q, dev, N)
    modes = [int(m) for m in os.environ.get("MODES", "0,1").split(",")]
    outs = {}
    for m in modes:
        _native.lib().mfa_xs_set_mode(m)
        outs[m] = xs_wls(p.styles, p.cap, p.ret, p.ind, P, refine=False, workspace=ws)
        torch.cuda.synchronize()
    m0 = modes[0]
    for m in modes[1:]:
        df = (outs[m].f - outs[m0].f).abs().nan_to_num(0).max().item()
        de = (outs[m].resid - outs[m0].resid).abs().nan_to_num(0).max().item()
        dr = (outs[m].r2 - outs[m0].r2).abs().nan_to_num(0).max().item()
        print(f"mode {m} vs {m0}: max|df| {df:.2e}  max|de| {de:.2e}  max|dr2| {dr:.2e}")
    times = {m: [] for m in modes}
    ev0, ev1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    for rnd in range(12):
        for m in modes:
            _native.lib().mfa_xs_set_mode(m)
            out = outs[m]
            ev0.record()
            for _ in range(5):
                xs_wls(p.styles, p.cap, p.ret, p.ind, P, refine=False, out=out, workspace=ws)
            ev1.record()
            ev1.synchronize()
            if rnd >= 2:
                times[m].append(ev0.elapsed_time(ev1) / 5)
    _native.lib().mfa_xs_set_mode(0)
    for m, t in times.items():
        print(f"mode {m}: median {statistics.median(t)*1e3:.1f} us  min {min(t)*1e3:.1f} us")


if __name__ == "__main__":
    main()
