"""K > 144 eigen stage on 1 GPU: the XL kernels (csrc/eigen_xl.hip, mc_cov_xl_kernel) against the
round-5 path (rocSOLVER batched syevd + rocBLAS GEMM, ``set_wide_bias_solver("rocsolver")``).

One JSON line per measurement:
  * ``eigh``: B Newey-West-like SPD matrices, ms per batch, max relative eigenvalue difference and
    max |A U - U diag(w)| / |A| of each path;
  * ``bias``: the bias sums of D dates x M sims (``_bias_sum_wide``), ms and max relative
    difference between the paths;
  * ``mc_cov``: M draw covariances at T rows;
  * ``risk``: RiskModel.run at P + Q + 1 = K, canonical timing (tools/risk_timing.py), both paths.

    python tools/xl_bench.py --K 180,256 --B 252 --D 252 --M 100
"""
from __future__ import annotations

import argparse
import json
import os
import sys
import time

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from llm_driven_multi_factor_model_amd.ops import eigen  # noqa: E402


def timed(fn, reps=3):
    fn()
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    for _ in range(reps):
        out = fn()
    torch.cuda.synchronize()
    return out, (time.perf_counter() - t0) / reps * 1e3


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--K", default="180,256")
    ap.add_argument("--B", type=int, default=252)
    ap.add_argument("--D", type=int, default=252)
    ap.add_argument("--M", type=int, default=100)
    ap.add_argument("--T", type=int, default=600)
    ap.add_argument("--risk", action="store_true", help="also time RiskModel.run (252 dates)")
    ap.add_argument("--no-rocsolver", action="store_true")
    ap.add_argument("--wpe", default="2", help="XL solver waves per SIMD to time, e.g. 2,4")
    a = ap.parse_args()
    dev = torch.device("cuda:0")
    paths = [f"hip{w}" for w in a.wpe.split(",")] + ([] if a.no_rocsolver else ["rocsolver"])

    def use(path):
        if path.startswith("hip"):
            eigen.set_xl_waves_per_simd(int(path[3:]))
            return eigen.using_wide_bias_solver("hip")
        return eigen.using_wide_bias_solver(path)
    for K in [int(x) for x in a.K.split(",")]:
        g = torch.Generator(device=dev).manual_seed(K)
        X = torch.randn(a.B, K, 2 * K, generator=g, device=dev, dtype=torch.float64)
        A = X @ X.transpose(1, 2) / (2 * K) * 1e-4
        ref = torch.linalg.eigvalsh(A).flip(-1)
        for path in paths:
            with use(path):
                (w, U), ms = timed(lambda: eigen.eigh(A))
            res = float(((A @ U - U * w[:, None, :]).abs().amax((-1, -2)) / A.abs().amax((-1, -2))).max())
            print(json.dumps({"what": "eigh", "path": path, "K": K, "B": a.B, "ms": round(ms, 3),
                              "dw_rel": float(((w - ref).abs() / ref.abs().amax(-1, keepdim=True)).max()),
                              "resid": res,
                              "flagged": int(eigen.LAST_EIGH_FLAGS.sum()) if path.startswith("hip") and K > eigen.WIDE_HIP_MAX_K else None}),
                  flush=True)
        with use(paths[0]):
            Cz, ms = timed(lambda: eigen.mc_cov(a.M, K, a.T, seed=1, device=dev))
        print(json.dumps({"what": "mc_cov", "path": "hip", "K": K, "M": a.M, "T": a.T,
                          "ms": round(ms, 3)}), flush=True)
        w, _ = eigen.eigh(A[:a.D] if a.D <= a.B else A)
        D = w.shape[0]
        valid = torch.isfinite(w).all(-1)
        w = w.clamp_min(0.0).contiguous()
        S = {}
        for path in paths:
            with use(path):
                S[path], ms = timed(lambda: eigen._bias_sum_wide(w, valid, Cz), reps=1)
            rec = {"what": "bias", "path": path, "K": K, "D": D, "M": a.M, "ms": round(ms, 2)}
            if path != paths[0]:
                rec["rel_diff_vs_first"] = float(((S[path] - S[paths[0]]).abs() / S[paths[0]].abs()).max())
            print(json.dumps(rec), flush=True)
        if a.risk:
            from tools.risk_timing import risk_model_timing
            from llm_driven_multi_factor_model_amd.utils.config import preset
            P, Q = K - 17, 16
            cfg = preset("reference", eigen_sims=a.M, nw_half_life=1000.0, vra_half_life=10.0,
                         eigen_sim_length=2 * K)
            for path in paths:
                with use(path):
                    r = risk_model_timing(252 + K, 5000, P, Q, cfg, dev, seeds=(3,), reps=3)
                print(json.dumps({"what": "risk", "path": path, "K": K, "D": 252 + K,
                                  "median_ms": r["median_ms"]}), flush=True)


if __name__ == "__main__":
    main()
