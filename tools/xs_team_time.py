"""Event timing of the team (cooperative) CS-WLS kernel against the fused kernel (1 GPU).

For every storage dtype and D in ``DATES`` it times ``xs_wls`` (refine on, deterministic: the
bench.py production call) with the team kernel off (fused, one workgroup per date) and with
C = ``CHUNKS`` workgroups per date, checks f / R^2 / e against the fused result and prints one
JSON line per configuration.

    python tools/xs_team_time.py      # env: DATES=315,2520 CHUNKS=2,3,4,6,8 DTYPES=fp64,fp32
"""
import json
import os
import statistics
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from llm_driven_multi_factor_model_amd import _native  # noqa: E402
from llm_driven_multi_factor_model_amd.models.panel import synthetic_panel  # noqa: E402
from llm_driven_multi_factor_model_amd.ops import cross_section as X  # noqa: E402


def timeit(fn, reps=20, rounds=5):
    ev0, ev1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    for _ in range(3):
        fn()
    ts = []
    for _ in range(rounds):
        ev0.record()
        for _ in range(reps):
            fn()
        ev1.record()
        ev1.synchronize()
        ts.append(ev0.elapsed_time(ev1) / reps * 1e3)
    return statistics.median(ts), min(ts)


def main():
    dev = torch.device("cuda:0")
    N, P, Q = int(os.environ.get("N", 5000)), 31, 10
    dates = [int(x) for x in os.environ.get("DATES", "315,2520").split(",")]
    chunks = [int(x) for x in os.environ.get("CHUNKS", "2,3,4,6,8").split(",") if x]
    dtypes = os.environ.get("DTYPES", "fp64,fp32").split(",")
    lags = [int(x) for x in os.environ.get("LAGS", "1").split(",")]
    lib = _native.lib()
    for dt in dtypes:
        base = synthetic_panel(max(dates), N, P, Q, seed=1, device=dev, missing_frac=0.01,
                               dtype=torch.float64 if dt == "fp64" else torch.float32)
        for _ in range(50):
            X.xs_wls(base.styles, base.cap, base.ret, base.ind, P)
        torch.cuda.synchronize()
        for D in dates:
            p = base.slice_dates(0, D)
            st, cp, rt, ind = (t.contiguous() for t in (p.styles, p.cap, p.ret, p.ind))
            ref = None
            for C, lag in [(0, 0)] + [(c, l) for c in chunks for l in lags]:
                lib.mfa_xs_set_coop(C)
                lib.mfa_xs_set_pipe(max(lag, 1), 0)
                try:
                    ws = X.xs_wls_workspace(D, P, Q, dev, N)
                    out = X.xs_wls(st, cp, rt, ind, P, workspace=ws)
                    torch.cuda.synchronize()
                    med, mn = timeit(lambda: X.xs_wls(st, cp, rt, ind, P, out=out, workspace=ws))
                    cc = _native.query("mfa_xs_coop_chunks", D, N)
                finally:
                    lib.mfa_xs_set_coop(0)
                    lib.mfa_xs_set_pipe(1, 0)
                rec = {"storage": dt, "D": D, "coop": C, "lag": lag, "chunks": cc, "us_med": round(med, 1),
                       "us_min": round(mn, 1), "Mreg_s": round(D / med, 3),
                       "timeouts": int((out.status & 64).ne(0).sum())}
                if ref is None:
                    ref = out
                    ref = type(out)(**{k: (v.clone() if v is not None else None)
                                       for k, v in out.__dict__.items()})
                else:
                    rec["f_maxdiff"] = float((out.f - ref.f).abs().max())
                    rec["r2_maxdiff"] = float((out.r2 - ref.r2).abs().max())
                    rec["e_maxdiff"] = float((out.resid - ref.resid).nan_to_num(0).abs().max())
                    rec["e_nan_eq"] = bool(torch.equal(out.resid.isnan(), ref.resid.isnan()))
                print(json.dumps(rec), flush=True)


if __name__ == "__main__":
    main()
