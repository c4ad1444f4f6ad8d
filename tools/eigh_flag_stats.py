"""How many of the risk model's F0 matrices (Newey-West covariances, bench panel shape) the
K <= 64 tridiagonal eigh flags for the Jacobi re-solve (eigenvectors not orthogonal to 1e-12),
their orthogonality errors before the re-solve, and the eigh time.

    python tools/eigh_flag_stats.py        # env: D=2520 SEED=3
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
D = int(os.environ.get("D", "2520"))
seed = int(os.environ.get("SEED", "3"))
p = synthetic_panel(D, 5000, 31, 10, seed=seed, missing_frac=0.01, dtype=torch.float64, device=dev)
m = RiskModel(p, preset("reference"))
m.regress()
m.newey_west()
F = m.nw_cov.contiguous()
fin = torch.isfinite(F.reshape(D, -1)).all(-1)
A = F[fin].contiguous()
B, K = A.shape[0], A.shape[-1]
lib = _native.lib()
w = torch.empty(B, K, dtype=torch.float64, device=dev)
U = torch.empty(B, K, K, dtype=torch.float64, device=dev)
flags = torch.empty(B, dtype=torch.int32, device=dev)
# the tridiagonal EIG kernel alone: flags + its raw eigenvectors
assert lib.mfa_eigh_set_mode(2) == 0
e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
tw = {0: [], 1: []}
for rd in range(4):
  for warm in (0, 1):
    lib.mfa_eigh_set_warm(warm)
    e0.record()
    _native.call("mfa_eigh_batched", _native.ptr(A), B, K, eigen.MAX_SWEEPS, eigen.TOL, _native.ptr(w),
                 _native.ptr(U), _native.ptr(flags), _native.stream(dev))
    e1.record()
    e1.synchronize()
    tw[warm].append(e0.elapsed_time(e1))
nfl = int(flags.sum())
err = (U.transpose(1, 2) @ U - torch.eye(K, dtype=torch.float64, device=dev)).abs().amax((1, 2))
print(json.dumps({"D": D, "seed": seed, "matrices": B, "flagged": nfl, "eigh_ms_min_cold_resolve": round(min(tw[0]), 3),
                  "eigh_ms_min_warm_resolve": round(min(tw[1]), 3),
                  "final_orth_err_max": float(err.max())}), flush=True)
