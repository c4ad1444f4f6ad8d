"""Event timing of the CS-WLS regression per path / storage / dates-per-launch (1 GPU).

For every storage dtype and every D in ``DATES`` it times ``xs_wls`` (refine on, as
``RiskModel.regress`` and bench.py run it) with the automatic path, with one workgroup per
date forced (``S=-1``) and with forced chunk counts; prints one JSON line per configuration.
Optional ``OLD_LIB`` = a round-1 build of ``csrc/xs_wls.hip`` (fp32 fused kernel only, raw
ctypes) timed at D = 2520 for an interleaved A/B of the fp32 kernel.

    python tools/xs_time.py            # env: DATES=315,630,1260,2520 CHUNKS=2,4,8 N=5000
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
    dates = [int(x) for x in os.environ.get("DATES", "315,630,1260,2520").split(",")]
    chunks = [int(x) for x in os.environ.get("CHUNKS", "2,4,8").split(",") if x]
    dtypes = os.environ.get("DTYPES", "fp64,fp32").split(",")
    lib = _native.lib()
    base = {dt: synthetic_panel(max(dates), N, P, Q, seed=1, device=dev, missing_frac=0.01,
                                dtype=torch.float64 if dt == "fp64" else torch.float32)
            for dt in dtypes}
    # warm the clocks
    p = base[dtypes[0]]
    for _ in range(100):
        X.xs_wls(p.styles, p.cap, p.ret, p.ind, P)
    torch.cuda.synchronize()
    for dt in dtypes:
        for D in dates:
            p = base[dt].slice_dates(0, D)
            st, cp, rt, ind = (t.contiguous() for t in (p.styles, p.cap, p.ret, p.ind))
            ref = None
            for S in [0, -1] + chunks:
                lib.mfa_xs_set_chunks(S)
                used = _native.query("mfa_xs_chunks", D, N)
                ws = X.xs_wls_workspace(D, P, Q, dev, N)
                out = X.xs_wls(st, cp, rt, ind, P, workspace=ws)
                med, mn = timeit(lambda: X.xs_wls(st, cp, rt, ind, P, out=out, workspace=ws))
                if ref is None:
                    ref = out.f.clone()
                err = (out.f - ref).abs().nan_to_num(0).max().item()
                print(json.dumps({"storage": dt, "D": D, "N": N, "chunks_req": S, "chunks": used,
                                  "us_median": round(med, 1), "us_min": round(mn, 1),
                                  "reg_per_s_M": round(D / med, 3), "max_df_vs_auto": err}),
                      flush=True)
            lib.mfa_xs_set_chunks(0)
    old = os.environ.get("OLD_LIB")
    if old and "fp32" in base:
        D = 2520
        olib = C.CDLL(old)
        olib.mfa_xs_wls.argtypes = [C.c_void_p] * 4 + [C.c_int] * 5 + [C.c_double] + [C.c_void_p] * 7
        olib.mfa_xs_wls_workspace.argtypes = [C.c_int] * 3
        olib.mfa_xs_wls_workspace.restype = C.c_size_t
        p = base["fp32"].slice_dates(0, D)
        K = 1 + P + Q
        f = torch.empty(D, K, dtype=torch.float64, device=dev)
        e = torch.empty(D, N, dtype=torch.float32, device=dev)
        r2 = torch.empty(D, dtype=torch.float64, device=dev)
        sts = torch.empty(D, Q + 2, dtype=torch.float64, device=dev)
        s = torch.empty(D, dtype=torch.int32, device=dev)
        ows = torch.empty(olib.mfa_xs_wls_workspace(D, P, Q), dtype=torch.uint8, device=dev)
        nws = X.xs_wls_workspace(D, P, Q, dev, N)
        ptr = _native.ptr

        def run_old():
            rc = olib.mfa_xs_wls(ptr(p.styles), ptr(p.cap), ptr(p.ret), ptr(p.ind), D, N, P, Q, 0,
                                 1e-14, ptr(f), ptr(e), ptr(r2), ptr(sts), ptr(s), ptr(ows),
                                 _native.stream(dev))
            assert rc == 0

        def run_new(flags):
            _native.call("mfa_xs_wls", ptr(p.styles), ptr(p.cap), ptr(p.ret), ptr(p.ind), D, N, P,
                         Q, flags, 1e-14, ptr(f), ptr(e), ptr(r2), ptr(sts), ptr(s), ptr(nws),
                         _native.stream(dev))
        res = {"old_r01": [], "new_norefine": [], "new_refine": []}
        for _ in range(4):
            res["old_r01"].append(timeit(run_old)[0])
            res["new_norefine"].append(timeit(lambda: run_new(0))[0])
            res["new_refine"].append(timeit(lambda: run_new(X.XS_REFINE))[0])
        print(json.dumps({"ab_fp32_D2520_us": {k: round(statistics.median(v), 1)
                                               for k, v in res.items()}}), flush=True)


if __name__ == "__main__":
    main()
