"""Date-sharded in-HBM end-to-end job (cli pipeline under torchrun) at benchmark size.

Every rank generates the same synthetic loader frames (stand-in for reading the loader CSVs),
runs ``e2e.run_pipeline(..., ctx)`` on its date block + halo, and the risk model over the ranks'
blocks.  Prints one JSON line per timed repetition with the slowest rank's phase times; rank 0
then reruns the whole panel in one process with the DEFAULT config and prints the max differences of the gathered outputs and
whether each is bitwise equal.  Sorted loader rows: every rank selects and uploads only its rows
(DeviceFactorEngine.from_host_shard).

    torchrun --nproc-per-node 8 --master-addr 127.0.0.1 tools/pipeline_dist.py [N] [T]
    MFA_DIST_BACKEND=gloo torchrun --nproc-per-node 4 ... (rehearsal: ranks share one GPU)
"""
import json
import os
import sys
import time

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from llm_driven_multi_factor_model_amd.models import e2e  # noqa: E402
from llm_driven_multi_factor_model_amd.models import factor_engine as FE  # noqa: E402
from llm_driven_multi_factor_model_amd.parallel import dist as pdist  # noqa: E402
from llm_driven_multi_factor_model_amd.utils.config import preset  # noqa: E402

KEYS = ("factor_ret", "r2", "nw_cov", "eigen_cov", "vra_cov", "vra_lambda")


def main():
    N = int(sys.argv[1]) if len(sys.argv) > 1 else 5000
    T = int(sys.argv[2]) if len(sys.argv) > 2 else 2520
    ctx = pdist.init_distributed()
    t0 = time.perf_counter()

    def note(msg):  # progress on stderr (a long silent phase looks hung to the GPU harness)
        print(f"[rank {ctx.rank} +{time.perf_counter() - t0:.1f}s] {msg}", file=sys.stderr,
              flush=True)
    prices, index, sw = FE.synthetic_prices_fast(N=N, T=T, seed=0, n_ind=31, suspend_frac=0.01)
    if os.environ.get("MFA_SORTED", "1") != "0":  # the stored panel's (ts_code, trade_date) order
        prices = prices.sort_values(["ts_code", "trade_date"], kind="stable").reset_index(drop=True)
    note("synthetic loader frames ready")
    cols = e2e._columns_from_frames(prices, index)
    cols = (e2e.stage_host_columns(cols[0]), cols[1])   # the native reader's layout (I/O)
    del prices
    note("columns staged")
    cfg = preset("reference")
    small = FE.synthetic_prices(N=60, T=300, seed=1, n_ind=31)
    e2e.run_pipeline(*small, risk_cfg=cfg, ctx=ctx)  # warm-up: kernel load, allocator, comms
    note("warm-up done")
    for rep in range(2):
        pdist.barrier(ctx)
        t0 = time.perf_counter()
        model, info, _, t = e2e.run_pipeline(dict(cols[0]), dict(cols[1]), sw, risk_cfg=cfg,
                                             ctx=ctx)
        wall = time.perf_counter() - t0
        rec = {k: pdist.all_reduce_max(v, ctx) for k, v in t.items() if k.endswith("_s")}
        rec["wall_s"] = pdist.all_reduce_max(wall, ctx)
        rec["non_io_s"] = sum(v for k, v in rec.items() if k.endswith("_s") and k != "wall_s")
        note(f"rep {rep} done")
        if ctx.rank == 0:
            print(json.dumps({"world": ctx.world, "backend": ctx.backend, "N": N, "T": T,
                              "D_panel": sum(model.sizes), "K": model.K, "rep": rep,
                              "host_shard": t.get("host_shard"),
                              **{k: round(v, 4) for k, v in rec.items()},
                              "kernel_ms_rank0": {k: round(v, 3) for k, v in
                                                  t.get("kernel_ms", {}).items()}}), flush=True)
    got = {k: pdist.gather_to_root(getattr(model, k).contiguous(), ctx) for k in KEYS}
    note("gathered")
    if ctx.rank == 0:
        one, _, _, t1 = e2e.run_pipeline(dict(cols[0]), dict(cols[1]), sw, risk_cfg=cfg,
                                         device=ctx.device)
        diff = {}
        for k in KEYS:
            a, b = got[k], getattr(one, k)
            ok = torch.isfinite(a) & torch.isfinite(b)
            diff[k] = {"max_abs": float((a - b)[ok].abs().max()) if ok.any() else None,
                       "max_rel": float(((a - b).abs() / b.abs().clamp_min(1e-30))[ok].max())
                       if ok.any() else None,
                       "nan_mismatch": int((torch.isfinite(a) != torch.isfinite(b)).sum()),
                       "bitwise": bool(torch.equal(a.nan_to_num(7.0), b.nan_to_num(7.0)))}
        print(json.dumps({"vs_one_process": diff,
                          "one_process_non_io_s": round(sum(v for k, v in t1.items()
                                                            if k.endswith("_s")), 4)}), flush=True)
    pdist.barrier(ctx)


if __name__ == "__main__":
    main()
