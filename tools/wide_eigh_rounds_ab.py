"""A/B of multisection rounds before the Laguerre loop of the wide F0 eigh (mfa_eigh_wide_fix at
K = 80 / 140) on the pipeline's own inputs: the Newey-West covariances of RiskModel on a
P = K - 17 industries / Q = 16 styles panel.  Interleaved rounds; per setting the min ms and the
max relative eigenvalue difference to LAPACK (CPU) on the finite dates.

    python tools/wide_eigh_rounds_ab.py        # env: K=140 D=504 ROUNDS_LIST=0,1,2,3,4
    ABSTOL=1 ROUNDS_LIST=0 ...                  # settings = abstol on/off (rounds fixed)

With ABSTOL=1 the settings are mfa_eigen_wide_set_eig_abstol(0 / 1) (LAPACK-style absolute
eigenvalue accuracy eps ||T||) and the report adds the max error relative to ||F||.
"""
import json
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from llm_driven_multi_factor_model_amd import _native  # noqa: E402
from llm_driven_multi_factor_model_amd.models.panel import synthetic_panel  # noqa: E402
from llm_driven_multi_factor_model_amd.models.risk_model import RiskModel  # noqa: E402
from llm_driven_multi_factor_model_amd.ops import eigen  # noqa: E402
from llm_driven_multi_factor_model_amd.utils.config import preset  # noqa: E402

dev = torch.device("cuda:0")
K = int(os.environ.get("K", "140"))
D = int(os.environ.get("D", "504"))
ABS = os.environ.get("ABSTOL") == "1"
settings = [0, 1] if ABS else [int(r) for r in os.environ.get("ROUNDS_LIST", "0,1,2,3,4").split(",")]


def knob(lib, r):
    return lib.mfa_eigen_wide_set_eig_abstol(r) if ABS else lib.mfa_eigen_wide_set_eig_rounds(r)
p = synthetic_panel(D, 5000, K - 17, 16, seed=3, missing_frac=0.01, dtype=torch.float64, device=dev)
m = RiskModel(p, preset("reference"))
m.regress()
m.newey_west()
F = m.nw_cov.contiguous()
fin = torch.isfinite(F.reshape(D, -1)).all(-1)
Fv = F[fin].contiguous()
lib = _native.lib()
e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
ts, ws = {r: [] for r in settings}, {}
try:
    for r in settings:
        assert knob(lib, r) == 0
        ws[r] = eigen.eigh(Fv)[0]
    for rd in range(3):
        rec = {"round": rd}
        for r in settings:
            knob(lib, r)
            torch.cuda.synchronize()
            e0.record()
            eigen.eigh(Fv)
            e1.record()
            e1.synchronize()
            ts[r].append(e0.elapsed_time(e1))
            rec[f"rounds{r}_ms"] = round(ts[r][-1], 3)
        print(json.dumps(rec), flush=True)
finally:
    lib.mfa_eigen_wide_set_eig_rounds(0)
    lib.mfa_eigen_wide_set_eig_abstol(0)
ref = torch.linalg.eigvalsh(Fv.cpu()).flip(-1)
out = {"K": K, "matrices": int(Fv.shape[0]), "knob": "abstol" if ABS else "rounds"}
nrm = ref.abs().amax(-1, keepdim=True)
for r in settings:
    out[f"rounds{r}_min_ms"] = round(min(ts[r]), 3)
    out[f"rounds{r}_max_rel_vs_lapack"] = float(((ws[r].cpu() - ref).abs() / ref.abs().clamp_min(1e-300)).max())
    out[f"rounds{r}_max_err_over_norm"] = float(((ws[r].cpu() - ref).abs() / nrm).max())
print(json.dumps(out), flush=True)
