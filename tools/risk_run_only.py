"""RiskModel.run alone, for a kernel trace that holds only the model's kernels.

    python tools/risk_run_only.py --make gpurun_out/panel.pt     # generate + save (not traced)
    rocprofv3 --kernel-trace --stats -d OUT -- python tools/risk_run_only.py --load gpurun_out/panel.pt

The traced process loads the saved fp64 panel from host memory (host -> device copies only, no
generator kernels), runs one warm-up ``RiskModel.run`` and ``--reps`` timed ones, and prints the
per-stage milliseconds of the last one.  Divide the kernel counts of the trace by reps + 1.
"""
import argparse
import json
import os
import sys
import time

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from llm_driven_multi_factor_model_amd.models.panel import RiskPanel, synthetic_panel  # noqa: E402
from llm_driven_multi_factor_model_amd.models.risk_model import RiskModel  # noqa: E402
from llm_driven_multi_factor_model_amd.utils.config import preset  # noqa: E402

ap = argparse.ArgumentParser()
ap.add_argument("--make", default=None)
ap.add_argument("--load", default=None)
ap.add_argument("--dates", type=int, default=2520)
ap.add_argument("--stocks", type=int, default=5000)
ap.add_argument("--reps", type=int, default=2)
ap.add_argument("--P", type=int, default=31)
ap.add_argument("--Q", type=int, default=10)
ap.add_argument("--bias-mode", type=int, default=None, help="mfa_eigen_set_bias_mode (A/B)")
ap.add_argument("--nw-half-life", type=float, default=None,
                help="wide K: a long half-life keeps the Newey-West covariances positive definite")
a = ap.parse_args()
if a.make:
    p = synthetic_panel(a.dates, a.stocks, a.P, a.Q, seed=3, missing_frac=0.01, dtype=torch.float64)
    torch.save({"styles": p.styles, "cap": p.cap, "ret": p.ret, "ind": p.ind,
                "dates": torch.from_numpy(p.dates.astype("int64"))}, a.make)
    sys.exit(0)
d = torch.load(a.load, weights_only=True)
import numpy as np  # noqa: E402
P = int(d["ind"].max()) + 1 if d["ind"].numel() else 0
p = RiskPanel(styles=d["styles"], cap=d["cap"], ret=d["ret"], ind=d["ind"], P=max(P, a.P),
              dates=d["dates"].numpy().astype("datetime64[ns]"),
              stocks=np.array([f"{i:06d}.SZ" for i in range(d["cap"].shape[1])], dtype=object)
              ).to("cuda:0")
cfg = preset("reference") if a.nw_half_life is None else \
    preset("reference", nw_half_life=a.nw_half_life, eigen_sim_length=2 * (1 + p.P + p.Q))
if a.bias_mode is not None:
    from llm_driven_multi_factor_model_amd import _native
    assert _native.lib().mfa_eigen_set_bias_mode(a.bias_mode) == 0, "bias mode not in this library"
for rep in range(a.reps + 1):
    m = RiskModel(p, cfg)
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    m.run()
    torch.cuda.synchronize()
    tot = (time.perf_counter() - t0) * 1e3
from llm_driven_multi_factor_model_amd.ops import eigen  # noqa: E402
fl = eigen.LAST_EIGH_FLAGS
print(json.dumps({"K": 1 + p.P + p.Q, "dates": p.D, "bias_mode": a.bias_mode,
                  "eigh_flags": {int(v): int((fl == v).sum()) for v in fl.unique()} if fl is not None else None,
                  "total_ms": round(tot, 3),
                  "stage_ms": {k: round(v, 3) for k, v in m.times.ms.items()}}))
