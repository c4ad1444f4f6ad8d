"""Strong-scaling remainder split A/B: a D-date shard with D between #CU and 2 #CU runs the first
C dates fused (one workgroup per date, one per CU) and the remaining D - C dates through the
chunked path (S stock chunks per date) on a second stream at the same time, so the leftover
work spreads over idle CU slots instead of doubling up whole dates on D - C CUs.

    python tools/xs_split_ab.py        # env: DATES=315,400,630 C=256 S=2,3,4
"""
import ctypes as C_
import json
import os
import statistics
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from llm_driven_multi_factor_model_amd import _native  # noqa: E402
from llm_driven_multi_factor_model_amd.models.panel import synthetic_panel  # noqa: E402
from llm_driven_multi_factor_model_amd.ops import cross_section as X  # noqa: E402

_native.register("mfa_xs_set_chunks", [C_.c_int])


def main():
    dev = torch.device("cuda:0")
    N, P, Q = 5000, 31, 10
    lib = _native.lib()
    cus = torch.cuda.get_device_properties(dev).multi_processor_count
    Cfix = int(os.environ.get("C", cus))
    Ss = [int(x) for x in os.environ.get("S", "2,3,4").split(",")]
    dates = [int(x) for x in os.environ.get("DATES", "315,400,630").split(",")]
    base = synthetic_panel(max(dates), N, P, Q, seed=1, device=dev, missing_frac=0.01,
                           dtype=torch.float64)
    side = torch.cuda.Stream(dev)
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    for D in dates:
        p = base.slice_dates(0, D)
        st, cp, rt, ind = (t.contiguous() for t in (p.styles, p.cap, p.ret, p.ind))
        lib.mfa_xs_set_chunks(0)
        ws_all = X.xs_wls_workspace(D, P, Q, dev, N)
        ref = X.xs_wls(st, cp, rt, ind, P, workspace=ws_all)
        C = min(Cfix, D)
        wsA = X.xs_wls_workspace(C, P, Q, dev, N)
        outA = X.xs_wls(st[:C], cp[:C], rt[:C], ind[:C], P, workspace=wsA)
        variants = {"fused": None}
        for S in Ss:
            lib.mfa_xs_set_chunks(S)
            wsB = X.xs_wls_workspace(D - C, P, Q, dev, N)
            outB = X.xs_wls(st[C:], cp[C:], rt[C:], ind[C:], P, workspace=wsB)
            variants[f"split_c{C}_s{S}"] = (S, wsB, outB)
        lib.mfa_xs_set_chunks(0)
        ts = {v: [] for v in variants}
        done = torch.cuda.Event()

        def run(v):
            if variants[v] is None:
                X.xs_wls(st, cp, rt, ind, P, out=ref, workspace=ws_all)
                return
            S, wsB, outB = variants[v]
            fork = torch.cuda.Event()
            fork.record()
            side.wait_event(fork)
            lib.mfa_xs_set_chunks(S)
            with torch.cuda.stream(side):
                X.xs_wls(st[C:], cp[C:], rt[C:], ind[C:], P, out=outB, workspace=wsB)
            lib.mfa_xs_set_chunks(0)
            X.xs_wls(st[:C], cp[:C], rt[:C], ind[:C], P, out=outA, workspace=wsA)
            done.record(side)
            torch.cuda.current_stream().wait_event(done)

        for v in variants:
            for _ in range(10):
                run(v)
        torch.cuda.synchronize()
        for _ in range(7):
            for v in variants:
                e0.record()
                for _ in range(20):
                    run(v)
                e1.record()
                torch.cuda.synchronize()
                ts[v].append(e0.elapsed_time(e1) * 1e3 / 20)
        err = {}
        for v, val in variants.items():
            if val is None:
                continue
            f = torch.cat([outA.f, val[2].f])
            err[v] = float((f - ref.f).abs().max())
        print(json.dumps({"D": D, "cus": cus, "us": {v: round(statistics.median(t), 1)
                                                     for v, t in ts.items()},
                          "max_df_vs_fused": err}), flush=True)


if __name__ == "__main__":
    main()
