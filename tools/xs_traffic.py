"""One production CS-WLS call pattern for PMC traffic counting (2520 x 5000 fp64, 1 GPU):
argv[1] = fused (default kernel) | team<C> (pipelined team kernel, C chunks per date)."""
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from llm_driven_multi_factor_model_amd import _native  # noqa: E402
from llm_driven_multi_factor_model_amd.models.panel import synthetic_panel  # noqa: E402
from llm_driven_multi_factor_model_amd.ops import cross_section as X  # noqa: E402

which = sys.argv[1] if len(sys.argv) > 1 else "fused"
dev = torch.device("cuda:0")
if which == "sum":  # calibration: one known 1 GiB fp64 read per call
    x = torch.ones(128 * 1024 * 1024, dtype=torch.float64, device=dev)
    for _ in range(5):
        x.sum()
    torch.cuda.synchronize()
    sys.exit(0)
D, N, P, Q = 2520, 5000, 31, 10
p = synthetic_panel(D, N, P, Q, seed=1, device=dev, missing_frac=0.01, dtype=torch.float64)
lib = _native.lib()
if which.startswith("team"):
    lib.mfa_xs_set_coop(int(which[4:]))
ws = X.xs_wls_workspace(D, P, Q, dev, N)
out = X.xs_wls(p.styles, p.cap, p.ret, p.ind, P, workspace=ws)
for _ in range(4):
    X.xs_wls(p.styles, p.cap, p.ret, p.ind, P, out=out, workspace=ws)
torch.cuda.synchronize()
lib.mfa_xs_set_coop(0)
