"""Time every risk-model stage (bench config by default); 1 GPU or torchrun.

BASELINE.json config 5 ("Newey-West factor-cov + 10k-bootstrap risk attribution, RCCL
all-reduce across 8 GPU"):

    torchrun --nproc-per-node 8 --master-addr 127.0.0.1 tools/risk_stages.py \
        --preset bootstrap10k --attribution

Under torchrun the dates are sharded over ranks (regression, NW, VRA); with ``--preset
bootstrap10k`` the 10k Monte-Carlo sims of the eigen adjustment are sharded over ranks and
combined with one all_reduce.  Rank 0 prints one JSON line: the canonical timing of
tools/risk_timing.py (median over panel seeds x reps of the max over ranks, per-seed stage
medians and Jacobi re-solve counts).
"""
import argparse
import json
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from llm_driven_multi_factor_model_amd.parallel import dist as pdist  # noqa: E402
from llm_driven_multi_factor_model_amd.utils.config import preset  # noqa: E402
from tools.risk_timing import risk_model_timing  # noqa: E402

ap = argparse.ArgumentParser()
ap.add_argument("--dates", type=int, default=2520, help="total dates (sharded under torchrun)")
ap.add_argument("--stocks", type=int, default=5000)
ap.add_argument("--P", type=int, default=31)
ap.add_argument("--Q", type=int, default=10)
ap.add_argument("--sims", type=int, default=None, help="override the preset's eigen sims")
ap.add_argument("--preset", default="reference")
ap.add_argument("--storage", choices=["fp64", "fp32"], default="fp64",
                help="panel storage dtype (fp64 = the reference's input precision)")
ap.add_argument("--reps", type=int, default=5)
ap.add_argument("--seeds", default="3,7,11", help="panel seeds (the median is over seeds x reps)")
ap.add_argument("--attribution", action="store_true", help="also time an equal-weight attribution")
a = ap.parse_args()
ctx = pdist.init_distributed()
over = {"eigen_sims": a.sims} if a.sims else {}
cfg = preset(a.preset, **over)
res = risk_model_timing(a.dates, a.stocks, a.P, a.Q, cfg, ctx.device,
                        seeds=[int(x) for x in a.seeds.split(",")], reps=a.reps, ctx=ctx,
                        attribution=a.attribution,
                        dtype=torch.float64 if a.storage == "fp64" else torch.float32)
if ctx.rank == 0:
    print(json.dumps({"shape": vars(a), "eigen_sims": cfg.eigen_sims,
                      "eigen_shard": cfg.eigen_shard, **res}))
if ctx.enabled:
    torch.distributed.destroy_process_group()
