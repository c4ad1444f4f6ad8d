"""Interleaved A/B of the fp32 fused CS-WLS kernel's timing-only ablation variants between the
current library and other builds (``OLD_LIB`` or ``LIBS=name=path,...``): localises a timing difference to a phase.

variant 0 = full, 4 = no residual pass, 8 = no solve, 12 = moments only, 1 = no segment
atomics, 2 = no style-Gram FMAs (``mfa_xs_wls_variant``).
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


def main():
    dev = torch.device("cuda:0")
    D, N, P, Q = int(os.environ.get("D", 2520)), 5000, 31, 10
    variants = [int(v) for v in os.environ.get("VARIANTS", "0,4,8,12,1,2").split(",")]
    f64 = os.environ.get("DTYPE", "fp32") == "fp64"
    dt = torch.float64 if f64 else torch.float32
    p = synthetic_panel(D, N, P, Q, seed=1, device=dev, missing_frac=0.01, dtype=dt)
    K = 1 + P + Q
    f = torch.empty(D, K, dtype=torch.float64, device=dev)
    e = torch.empty(D, N, dtype=dt, device=dev)
    r2 = torch.empty(D, dtype=torch.float64, device=dev)
    sts = torch.empty(D, Q + 2, dtype=torch.float64, device=dev)
    s = torch.empty(D, dtype=torch.int32, device=dev)
    ws = torch.empty(64 << 20, dtype=torch.uint8, device=dev)
    libs = {"new": _native.lib()}
    for item in os.environ.get("LIBS", "").split(","):  # name=path,...
        if item:
            name, path = item.split("=")
            libs[name] = C.CDLL(path)
    if os.environ.get("OLD_LIB"):
        libs["old"] = C.CDLL(os.environ["OLD_LIB"])
    sym = "mfa_xs_wls_variant_f64" if f64 else "mfa_xs_wls_variant"
    for lib in libs.values():
        getattr(lib, sym).argtypes = [C.c_void_p] * 4 + [C.c_int] * 4 + [C.c_void_p] * 7
    ptr = _native.ptr
    ev0, ev1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)

    def t(lib, v, reps=10):
        fn = lambda: getattr(lib, sym)(ptr(p.styles), ptr(p.cap), ptr(p.ret), ptr(p.ind), D, N,
                                            P, v, ptr(f), ptr(e), ptr(r2), ptr(sts), ptr(s), ptr(ws),
                                            _native.stream(dev))
        assert fn() == 0
        ev0.record()
        for _ in range(reps):
            fn()
        ev1.record()
        ev1.synchronize()
        return ev0.elapsed_time(ev1) / reps * 1e3

    for _ in range(50):
        t(next(iter(libs.values())), 0, 2)
    res = {(n, v): [] for n in libs for v in variants}
    for _ in range(6):
        for v in variants:
            for n, lib in libs.items():
                res[(n, v)].append(t(lib, v))
    for v in variants:
        print(json.dumps({"variant": v, **{n: round(statistics.median(res[(n, v)]), 1)
                                           for n in libs}}), flush=True)


if __name__ == "__main__":
    main()
