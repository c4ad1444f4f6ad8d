"""Multi-rank RiskModel on GPU tensors vs a single-process run of the same panel.

Launch under torchrun.  On a one-GPU box, set MFA_DIST_BACKEND=gloo: several ranks then share
the device (RCCL refuses that).  Every rank regresses and adjusts its date shard.  Rank 0 gathers
the outputs, reruns the whole panel in one process, and prints the max abs differences for each
(time_scan, eigen_shard) mode.  Synthetic fp64 panel.

    MFA_DIST_BACKEND=gloo torchrun --nproc-per-node 4 --master-addr 127.0.0.1 tools/dist_rehearsal.py
"""
import json
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from llm_driven_multi_factor_model_amd.models.panel import synthetic_panel  # noqa: E402
from llm_driven_multi_factor_model_amd.models.risk_model import RiskModel  # noqa: E402
from llm_driven_multi_factor_model_amd.parallel import dist as pdist  # noqa: E402
from llm_driven_multi_factor_model_amd.utils.config import preset  # noqa: E402


def main():
    ctx = pdist.init_distributed()
    dev = ctx.device
    D, N = int(os.environ.get("D", 504)), int(os.environ.get("N", 1000))
    full = synthetic_panel(D, N, 31, 10, seed=5, device=dev, missing_frac=0.01, dtype=torch.float64)
    a, b = pdist.shard_range(D, ctx.rank, ctx.world)
    keys = ("f", "r2", "nw", "er", "vr", "lam")
    res = {}
    for scan in ("gather", "carry"):
        for shard in ("dates", "sims"):
            cfg = preset("reference", eigen_sims=20, eigen_shard=shard, time_scan=scan)
            m = RiskModel(full.slice_dates(a, b), cfg, T_global=D, ctx=ctx).run()
            got = dict(zip(keys, (pdist.gather_to_root(v, ctx) for v in (
                m.factor_ret, m.r2, m.nw_cov, m.eigen_cov, m.vra_cov, m.vra_lambda))))
            if ctx.rank == 0:
                one = RiskModel(full, preset("reference", eigen_sims=20, time_scan=scan),
                                ctx=pdist.DistContext(device=dev)).run()  # one process
                ref = dict(zip(keys, (one.factor_ret, one.r2, one.nw_cov, one.eigen_cov,
                                      one.vra_cov, one.vra_lambda)))
                res[f"{scan}/{shard}"] = {k: float((got[k] - ref[k]).abs().nan_to_num(0).max())
                                          for k in keys}
            pdist.barrier(ctx)
    if ctx.rank == 0:
        print(json.dumps({"world": ctx.world, "backend": ctx.backend, "device": str(dev), "D": D,
                          "N": N, "max_abs_diff_vs_one_process": res}), flush=True)
    pdist.barrier(ctx)
    torch.distributed.destroy_process_group()


if __name__ == "__main__":
    main()
