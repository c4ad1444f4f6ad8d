"""Run every BASELINE.json configuration once on this machine and print one JSON summary.

  1  50-stock x 100-day synthetic panel, 3 style factors, CPU demo.py path (plumbing, no GPU)
  2  CSI300 (300 stocks) x 5y daily, 10 style + 31 SW-industry factors, 1 GPU (full risk model)
  3  All-A ~5000 stocks x 10y daily, full factor set (full risk model on this GPU; the 8-GPU
     date-sharded run is bench.py / risk_stages.py under torchrun)
  4  252-day rolling beta recompute, 5000 stocks x 15y
  5  Newey-West factor cov + 10k-simulation eigen "bootstrap" + risk attribution

Reference costs are BASELINE.md's measured / extrapolated survey-host numbers.
"""
import contextlib
import io
import json
import os
import sys
import time

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from llm_driven_multi_factor_model_amd.ops import rolling as RL  # noqa: E402
from llm_driven_multi_factor_model_amd.utils.config import preset  # noqa: E402
from tools.risk_timing import risk_model_timing  # noqa: E402


def timed(fn, reps=2):
    fn()  # warm-up (kernel loading, allocator)
    if torch.cuda.is_available():
        torch.cuda.synchronize()
    t0 = time.perf_counter()
    for _ in range(reps):
        out = fn()
    if torch.cuda.is_available():
        torch.cuda.synchronize()
    return (time.perf_counter() - t0) / reps, out


def risk_run(D, N, P, Q, cfg, device, attribution=False, reps=5):
    """The canonical timing (tools/risk_timing.py): median over seeds 3 / 7 / 11 x ``reps``."""
    r = risk_model_timing(D, N, P, Q, cfg, device, reps=reps, attribution=attribution)
    return r["median_ms"] / 1e3, r


def main():
    res = {}
    # 1: toy config through the drop-in mfm API on the CPU (demo.py path)
    os.environ["MFA_DEVICE"] = "cpu"
    import mfm
    from tests.test_mfm_compat import toy_frame
    df = toy_frame(T=100, N=50, P=3, Q=3)

    def demo():
        with contextlib.redirect_stdout(io.StringIO()):
            m = mfm.MFM(df, 3, 3)
            m.reg_by_time()
            m.Newey_West_by_time(q=2, tao=252)
            m.eigen_risk_adj_by_time(M=100, scale_coef=1.4)
            m.vol_regime_adj_by_time(tao=42)
    t, _ = timed(demo, reps=1)
    res["1_toy_cpu_demo"] = {"seconds": round(t, 3), "reference_seconds": 3.5}
    dev = torch.device("cuda:0")
    # 2: CSI300 x 5y, K = 42, full risk model (M = 100)
    t, r = risk_run(1250, 300, 31, 10, preset("reference"), dev)
    res["2_csi300_5y_risk_model"] = {"seconds": round(t, 4), "timing": r,
                                     "reference_seconds": 6.9 + 28 + 11.5 * 60}
    # 3: All-A 5000 x 10y, full risk model on one GPU
    t, r = risk_run(2520, 5000, 31, 10, preset("reference"), dev)
    res["3_alla_10y_risk_model_1gpu"] = {"seconds": round(t, 4), "timing": r,
                                         "reference_seconds": 4.4 * 60 + 1.9 * 60 + 45 * 60}
    # 4: 252-day rolling beta / hsigma, 5000 x 15y
    N, T = 5000, 3780
    g = torch.Generator(device=dev).manual_seed(0)
    mkt = torch.randn(T, device=dev, generator=g) * 0.012
    ret = (mkt[None, :] * 1.1 + torch.randn(N, T, device=dev, generator=g) * 0.02).reshape(-1).float()
    mret = mkt[None, :].expand(N, T).reshape(-1).contiguous().float()
    seg = RL.seg_lo_from_codes(torch.arange(N, device=dev, dtype=torch.int32).repeat_interleave(T))
    # the whole recompute: segment layout (+ host read of its size) and inputs placed, kernel;
    # and the kernel alone on a layout the engine already holds (shared by every descriptor)
    t, _ = timed(lambda: RL.beta_hsigma(ret, mret, seg, 252, 63.0, 42), reps=5)
    lay = RL.SegLayout(seg, None, (ret, mret))
    tk, _ = timed(lambda: RL.beta_hsigma(ret, mret, seg, 252, 63.0, 42, row_ord=lay), reps=20)
    res["4_rolling_beta_5000x15y"] = {"seconds": round(t, 5), "stock_days": N * T,
                                      "kernel_on_built_layout_seconds": round(tk, 5),
                                      "reference_seconds": 4.3 * 3600}
    # 5: NW + 10k-sim eigen bootstrap + attribution (CSI300 x 5y shape; sims-sharded mode)
    t, r = risk_run(1250, 300, 31, 10, preset("bootstrap10k"), dev, attribution=True, reps=3)
    res["5_nw_bootstrap10k_attribution"] = {"seconds": round(t, 3), "timing": r,
                                            "reference_seconds": 57.0 * 1250}
    for v in res.values():
        v["speedup_vs_reference"] = round(v["reference_seconds"] / v["seconds"], 1)
    print(json.dumps(res))


if __name__ == "__main__":
    main()
