"""Strong-scaling shard sizes (315 / 630 dates = 2520 over 8 / 4 GPUs): fused kernel (one
workgroup per date) vs the chunked path (S stock chunks per date: moments, solve, residual
kernels) vs the pipelined team kernel (C chunks per date), fp64 panel, refine + deterministic
(the production call).  One JSON line per D: median us per variant, max |df| vs fused.

    python tools/xs_chunk_ab.py        # env: DATES=315,630,2520
"""
import ctypes as C
import json
import os
import statistics
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from llm_driven_multi_factor_model_amd import _native  # noqa: E402
from llm_driven_multi_factor_model_amd.models.panel import synthetic_panel  # noqa: E402
from llm_driven_multi_factor_model_amd.ops import cross_section as X  # noqa: E402

_native.register("mfa_xs_set_chunks", [C.c_int])
_native.register("mfa_xs_set_coop", [C.c_int])
VARIANTS = {"fused": (0, 0), "chunk2": (2, 0), "chunk3": (3, 0), "chunk4": (4, 0),
            "team_auto": (0, -1), "team2": (0, 2), "team4": (0, 4)}


def main():
    dev = torch.device("cuda:0")
    N, P, Q = 5000, 31, 10
    lib = _native.lib()
    dates = [int(x) for x in os.environ.get("DATES", "315,630,2520").split(",")]
    base = synthetic_panel(max(dates), N, P, Q, seed=1, device=dev, missing_frac=0.01,
                           dtype=torch.float64)
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    for D in dates:
        p = base.slice_dates(0, D)
        st, cp, rt, ind = (t.contiguous() for t in (p.styles, p.cap, p.ret, p.ind))
        outs, ts, wss = {}, {v: [] for v in VARIANTS}, {}
        for v, (s, c) in VARIANTS.items():
            lib.mfa_xs_set_chunks(s)
            lib.mfa_xs_set_coop(c)
            wss[v] = X.xs_wls_workspace(D, P, Q, dev, N)
            outs[v] = X.xs_wls(st, cp, rt, ind, P, workspace=wss[v])
            for _ in range(20):
                X.xs_wls(st, cp, rt, ind, P, out=outs[v], workspace=wss[v])
        torch.cuda.synchronize()
        for _ in range(7):
            for v, (s, c) in VARIANTS.items():
                lib.mfa_xs_set_chunks(s)
                lib.mfa_xs_set_coop(c)
                e0.record()
                for _ in range(20):
                    X.xs_wls(st, cp, rt, ind, P, out=outs[v], workspace=wss[v])
                e1.record()
                torch.cuda.synchronize()
                ts[v].append(e0.elapsed_time(e1) * 1e3 / 20)
        lib.mfa_xs_set_chunks(0)
        lib.mfa_xs_set_coop(0)
        ref = outs["fused"].f
        print(json.dumps({"D": D, "us": {v: round(statistics.median(t), 1) for v, t in ts.items()},
                          "max_df": {v: float((o.f - ref).abs().max()) for v, o in outs.items()}}),
              flush=True)


if __name__ == "__main__":
    main()
