"""Where the flagged-matrix Jacobi re-solve of the K <= 64 F0 eigh spends its time: the eigh
(tridiagonal kernel + re-solve of the flagged matrices) timed with max_sweeps = 0 / 1 / 2 / 3 /
MAX_SWEEPS, warm (orthonormalised tridiagonal eigenvectors, B = Q^T A Q) and cold (V = I).
max_sweeps = 0 leaves the re-solve's setup alone (outputs meaningless), so
T(warm, 0) - T(cold, 0) is the warm setup and T(x, n) - T(x, 0) the cost of n sweeps.

    python tools/eigh_resolve_split.py        # env: D=2520 SEED=3
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
assert lib.mfa_eigh_set_mode(2) == 0
e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
cfgs = [(wm, ns) for wm in (0, 1) for ns in (0, 1, 2, 3, eigen.MAX_SWEEPS)]
t = {c: [] for c in cfgs}
err = {}
for rd in range(5):
    for wm, ns in cfgs:
        lib.mfa_eigh_set_warm(wm)
        e0.record()
        _native.call("mfa_eigh_batched", _native.ptr(A), B, K, ns, eigen.TOL, _native.ptr(w),
                     _native.ptr(U), _native.ptr(flags), _native.stream(dev))
        e1.record()
        e1.synchronize()
        t[(wm, ns)].append(e0.elapsed_time(e1))
        if rd == 0:
            fl = flags.bool()
            Uf = U[fl]
            E = (Uf.transpose(1, 2) @ Uf - torch.eye(K, dtype=torch.float64, device=dev)).abs().amax()
            R = (A[fl] @ Uf - Uf * w[fl][:, None, :]).abs().amax() / A[fl].abs().amax()
            err[(wm, ns)] = (float(E) if fl.any() else 0.0, float(R) if fl.any() else 0.0)
lib.mfa_eigh_set_warm(1)
print(json.dumps({"D": D, "seed": seed, "matrices": B, "flagged": int(flags.sum()),
                  "ms_min": {f"{'warm' if wm else 'cold'}_sweeps{ns}": round(min(v), 4)
                             for (wm, ns), v in t.items()},
                  "orth_err_resid": {f"{'warm' if wm else 'cold'}_sweeps{ns}": e
                                     for (wm, ns), e in err.items()}}), flush=True)
