"""A/B of CS-WLS kernel modes on the production call (xs_wls, refine on, deterministic
default), rounds interleaved, for fp64 / fp32 panels and several date counts (1 GPU).

    python tools/xs_mode_time.py        # env: MODES=0,20 DATES=64,315,2520 DTYPES=fp64,fp32

mode 0 = fused kernel (LDS-DMA ring), 20 = fused kernel with plain-load moments.
Prints one JSON line per (dtype, D): median us per mode and max |df| / |de| vs the first mode.
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

_native.register("mfa_xs_set_mode", [C.c_int])


def main():
    dev = torch.device("cuda:0")
    N, P, Q = 5000, 31, 10
    modes = [int(m) for m in os.environ.get("MODES", "0,20").split(",")]
    dates = [int(x) for x in os.environ.get("DATES", "64,315,2520").split(",")]
    lib = _native.lib()
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    for dt in os.environ.get("DTYPES", "fp64,fp32").split(","):
        base = synthetic_panel(max(dates), N, P, Q, seed=1, device=dev, missing_frac=0.01,
                               dtype=torch.float64 if dt == "fp64" else torch.float32)
        for D in dates:
            p = base.slice_dates(0, D)
            st, cp, rt, ind = (t.contiguous() for t in (p.styles, p.cap, p.ret, p.ind))
            ws = X.xs_wls_workspace(D, P, Q, dev, N)
            outs, ts = {}, {m: [] for m in modes}
            for m in modes:
                lib.mfa_xs_set_mode(m)
                outs[m] = X.xs_wls(st, cp, rt, ind, P, workspace=ws)
                for _ in range(30):
                    X.xs_wls(st, cp, rt, ind, P, out=outs[m], workspace=ws)
            torch.cuda.synchronize()
            for _ in range(7):
                for m in modes:
                    lib.mfa_xs_set_mode(m)
                    e0.record()
                    for _ in range(20):
                        X.xs_wls(st, cp, rt, ind, P, out=outs[m], workspace=ws)
                    e1.record()
                    e1.synchronize()
                    ts[m].append(e0.elapsed_time(e1) / 20 * 1e3)
            lib.mfa_xs_set_mode(0)
            rec = {"storage": dt, "D": D}
            for m in modes:
                rec[f"mode{m}_us"] = round(statistics.median(ts[m]), 1)
                if m != modes[0]:
                    rec[f"mode{m}_df"] = float((outs[m].f - outs[modes[0]].f).abs().max())
                    rec[f"mode{m}_de"] = float((outs[m].resid - outs[modes[0]].resid).nan_to_num(0).abs().max())
            print(json.dumps(rec), flush=True)


if __name__ == "__main__":
    main()
