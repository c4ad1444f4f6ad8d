"""Interleaved timing of CS-WLS kernel execution modes of ONE build (``LIB``, default: the
in-tree library) for fp32 and fp64 panels, with the timing-only ablation variants.

mode 0 = fused VALU-moments kernel (2 workgroups / CU); 10 / 11 / 12 = fused MFMA-moments
kernel with 3 / 4 / 2 workgroups per CU (segment replicas 4 / 2 / 8).  Checks that every mode
gives the same factor returns as mode 0 first.

    MODES=0,10,12 VARIANTS=0,12 python tools/xs_ab_modes.py
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
    modes = [int(m) for m in os.environ.get("MODES", "0,10,12").split(",")]
    variants = [int(v) for v in os.environ.get("VARIANTS", "0,12").split(",")]
    lib = C.CDLL(os.environ["LIB"]) if os.environ.get("LIB") else _native.lib()
    lib.mfa_xs_set_mode.argtypes = [C.c_int]
    ptr = _native.ptr
    ev0, ev1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    for dts in os.environ.get("DTYPES", "fp32,fp64").split(","):
        dt = torch.float64 if dts == "fp64" else torch.float32
        sym = getattr(lib, "mfa_xs_wls_variant_f64" if dts == "fp64" else "mfa_xs_wls_variant")
        sym.argtypes = [C.c_void_p] * 4 + [C.c_int] * 4 + [C.c_void_p] * 7
        p = synthetic_panel(D, N, P, Q, seed=1, device=dev, missing_frac=0.01, dtype=dt)
        K = 1 + P + Q
        bufs = {m: (torch.empty(D, K, dtype=torch.float64, device=dev),
                    torch.empty(D, N, dtype=dt, device=dev),
                    torch.empty(D, dtype=torch.float64, device=dev),
                    torch.empty(D, Q + 2, dtype=torch.float64, device=dev),
                    torch.empty(D, dtype=torch.int32, device=dev)) for m in modes}
        ws = torch.empty(64 << 20, dtype=torch.uint8, device=dev)

        def call(m, v):
            f, e, r2, st, s = bufs[m]
            lib.mfa_xs_set_mode(m)
            rc = sym(ptr(p.styles), ptr(p.cap), ptr(p.ret), ptr(p.ind), D, N, P, v, ptr(f), ptr(e),
                     ptr(r2), ptr(st), ptr(s), ptr(ws), _native.stream(dev))
            assert rc == 0, (m, v, rc)

        for m in modes:
            call(m, 0)
        torch.cuda.synchronize()
        f0, e0, r20 = bufs[modes[0]][:3]
        for m in modes[1:]:
            f, e, r2 = bufs[m][:3]
            print(json.dumps({"storage": dts, "mode": m, "max_df": (f - f0).abs().nan_to_num(0).max().item(),
                              "max_de": (e - e0).abs().nan_to_num(0).max().item(),
                              "max_dr2": (r2 - r20).abs().nan_to_num(0).max().item()}), flush=True)
        for _ in range(30):
            call(modes[0], 0)
        res = {(m, v): [] for m in modes for v in variants}
        for _ in range(6):
            for v in variants:
                for m in modes:
                    call(m, v)
                    ev0.record()
                    for _ in range(10):
                        call(m, v)
                    ev1.record()
                    ev1.synchronize()
                    res[(m, v)].append(ev0.elapsed_time(ev1) / 10 * 1e3)
        for v in variants:
            print(json.dumps({"storage": dts, "D": D, "variant": v,
                              **{f"mode{m}": round(statistics.median(res[(m, v)]), 1) for m in modes}}),
                  flush=True)
        lib.mfa_xs_set_mode(0)


if __name__ == "__main__":
    main()
