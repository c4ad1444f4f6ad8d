"""Per-date phase times of the resident fused CS-WLS kernel (mode 30 and its A/B geometries):
every workgroup stamps the wall clock (100 MHz) at start / end of the moments stream / end of
the reduction / end of the solve / end, plus its hardware id.  Prints one JSON line per mode:
median and mean us per phase, the span of all dates, the event-timed call, and the busy
fraction of the CUs (sum of workgroup lifetimes / (CUs x span)).

    python tools/xs_resident_phases.py      # env: MODES=30,32 D=2520 N=5000
"""
import ctypes as C
import json
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from llm_driven_multi_factor_model_amd import _native  # noqa: E402
from llm_driven_multi_factor_model_amd.models.panel import synthetic_panel  # noqa: E402
from llm_driven_multi_factor_model_amd.ops import cross_section as X  # noqa: E402

_native.register("mfa_xs_set_mode", [C.c_int])
_native.register("mfa_xs_set_prof", [C.c_void_p])
TICK_US = 0.01  # wall_clock64: 100 MHz


def main():
    dev = torch.device("cuda:0")
    D, N, P, Q = int(os.environ.get("D", 2520)), int(os.environ.get("N", 5000)), 31, 10
    lib = _native.lib()
    p = synthetic_panel(D, N, P, Q, seed=1, device=dev, missing_frac=0.01, dtype=torch.float64)
    st, cp, rt, ind = (t.contiguous() for t in (p.styles, p.cap, p.ret, p.ind))
    ws = X.xs_wls_workspace(D, P, Q, dev, N)
    prof = torch.zeros(D * 6, dtype=torch.int64, device=dev)
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    ncu = torch.cuda.get_device_properties(dev).multi_processor_count
    for m in [int(x) for x in os.environ.get("MODES", "30").split(",")]:
        lib.mfa_xs_set_mode(m)
        try:
            out = X.xs_wls(st, cp, rt, ind, P, workspace=ws)
            for _ in range(10):
                X.xs_wls(st, cp, rt, ind, P, out=out, workspace=ws)
            torch.cuda.synchronize()
            lib.mfa_xs_set_prof(prof.data_ptr())
            e0.record()
            X.xs_wls(st, cp, rt, ind, P, out=out, workspace=ws)
            e1.record()
            e1.synchronize()
        finally:
            lib.mfa_xs_set_prof(None)
            lib.mfa_xs_set_mode(0)
        t = prof.view(D, 6).cpu().double()
        ph = (t[:, 1:5] - t[:, 0:4]) * TICK_US            # moments, reduction, solve, residual
        life = (t[:, 4] - t[:, 0]) * TICK_US
        span = float((t[:, 4].max() - t[:, 0].min()) * TICK_US)
        rec = {"mode": m, "D": D, "N": N, "call_us": round(e0.elapsed_time(e1) * 1e3, 1),
               "span_us": round(span, 1),
               "busy_frac": round(float(life.sum()) / (ncu * span), 3),
               "first_start_to_last_start_us": round(float((t[:, 0].max() - t[:, 0].min()) * TICK_US), 1)}
        for k, name in enumerate(("moments", "reduce", "solve", "resid")):
            rec[f"{name}_med_us"] = round(float(ph[:, k].median()), 2)
            rec[f"{name}_mean_us"] = round(float(ph[:, k].mean()), 2)
        rec["life_med_us"] = round(float(life.median()), 2)
        print(json.dumps(rec), flush=True)


if __name__ == "__main__":
    main()
