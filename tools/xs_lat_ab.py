"""Interleaved timing of the production CS-WLS call (``xs_wls``, refine on, deterministic) under
kernel execution modes (``mfa_xs_set_mode``) at several shard sizes D, fp64 and fp32 panels.

mode 0 = default fused kernel (2 workgroups / CU, 2-slot fp64 / 4-slot fp32 rings), 7 = fused
without the fp32 residual prefetch, 1 = three separate kernels.  The round-2 latency-mode
variants (modes 30..33: one workgroup per CU with deep LDS-DMA rings) were measured with this
tool and removed (profiles/r02_xs_latency_mode_ab.md).  Checks bitwise agreement with the first
mode first.

    MODES=0,7 DS=64,256,315,2520 python tools/xs_lat_ab.py
"""
import json
import os
import statistics
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from llm_driven_multi_factor_model_amd import _native  # noqa: E402
from llm_driven_multi_factor_model_amd.models.panel import synthetic_panel  # noqa: E402
from llm_driven_multi_factor_model_amd.ops.cross_section import xs_wls, xs_wls_workspace  # noqa: E402


def main():
    dev = torch.device("cuda:0")
    N, P, Q = 5000, 31, int(os.environ.get("Q", 10))
    modes = [int(m) for m in os.environ.get("MODES", "0,30").split(",")]
    Ds = [int(d) for d in os.environ.get("DS", "64,256,315,2520").split(",")]
    reps = int(os.environ.get("REPS", "20"))
    lib = _native.lib()
    ev0, ev1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    for dts in os.environ.get("DTYPES", "fp64,fp32").split(","):
        dt = torch.float64 if dts == "fp64" else torch.float32
        for D in Ds:
            p = synthetic_panel(D, N, P, Q, seed=1, device=dev, missing_frac=0.01, dtype=dt)
            ws = xs_wls_workspace(D, P, Q, dev, N)
            outs = {}

            def call(m):
                lib.mfa_xs_set_mode(m)
                outs[m] = xs_wls(p.styles, p.cap, p.ret, p.ind, P, want_resid=True, refine=True,
                                 out=outs.get(m), workspace=ws)

            for m in modes:
                call(m)
            torch.cuda.synchronize()
            o0 = outs[modes[0]]
            for m in modes[1:]:
                o = outs[m]
                same = bool(torch.equal(o.f.nan_to_num(0), o0.f.nan_to_num(0)) and
                            torch.equal(o.resid.nan_to_num(0), o0.resid.nan_to_num(0)) and
                            torch.equal(o.r2.nan_to_num(0), o0.r2.nan_to_num(0)))
                print(json.dumps({"storage": dts, "D": D, "mode": m, "bitwise_equal_mode0": same,
                                  "max_df": (o.f - o0.f).abs().nan_to_num(0).max().item()}), flush=True)
            # each mode's call captured into its own HIP graph (the mode is read at launch time):
            # replays measure the kernels, not Python launch overhead
            graphs = {}
            torch.cuda.synchronize()
            for m in modes:
                graphs[m] = torch.cuda.CUDAGraph()
                with torch.cuda.graph(graphs[m]):
                    call(m)
            lib.mfa_xs_set_mode(0)
            for _ in range(20):
                graphs[modes[0]].replay()
            res = {m: [] for m in modes}
            for _ in range(6):
                for m in modes:
                    graphs[m].replay()
                    ev0.record()
                    for _ in range(reps):
                        graphs[m].replay()
                    ev1.record()
                    ev1.synchronize()
                    res[m].append(ev0.elapsed_time(ev1) / reps * 1e3)
            print(json.dumps({"storage": dts, "D": D, "Q": Q, "us": {f"mode{m}": round(statistics.median(res[m]), 1)
                                                             for m in modes}}), flush=True)
            lib.mfa_xs_set_mode(0)


if __name__ == "__main__":
    main()
