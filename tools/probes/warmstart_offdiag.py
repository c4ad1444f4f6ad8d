"""Probe for a warm-started Monte-Carlo Jacobi (next-step idea, README): per sim m, how far from
diagonal is C_b(d) = S_d C_z,m S_d in the eigenbasis of C_b(d-1)?  Jacobi converges
quadratically, so the starting relative off-diagonal norm sets the sweep count
(cold start from the identity basis needs ~6 sweeps on these inputs)."""
import json
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__)))))
from llm_driven_multi_factor_model_amd.models.panel import synthetic_panel  # noqa: E402
from llm_driven_multi_factor_model_amd.ops.cross_section import xs_wls_reference  # noqa: E402
from llm_driven_multi_factor_model_amd.ops.ew_scan import newey_west_series  # noqa: E402

torch.manual_seed(0)
D, N, P, Q, M = 400, 300, 31, 10, 8
p = synthetic_panel(D, N, P, Q, seed=3)
f = xs_wls_reference(p.styles, p.cap, p.ret, p.ind, P, want_resid=False).f
V = newey_west_series(f, q=2, tau=252.0)
K = V.shape[-1]
z = torch.randn(M, K, 2 * D, dtype=torch.float64)
Cz = z @ z.transpose(1, 2) / (2 * D)


def rel_off(A):
    d = torch.diagonal(A, dim1=-2, dim2=-1)
    off = (A * A).sum((-2, -1)) - (d * d).sum(-1)
    return (off / (d * d).sum(-1)).sqrt()


res = {}
for lo in (100, 250, 399):
    out = []
    for d in (lo - 1, lo):
        w0, U0 = torch.linalg.eigh(V[d])
        s = w0.clamp(min=0).sqrt()
        out.append(s[None, :, None] * Cz * s[None, None, :])     # C_b(d) in F0(d)'s eigenbasis
    # eigen bases of F0 differ between d-1 and d: rotate C_b(d-1)'s eigvecs into d's F0 basis
    w_prev, U_prev = torch.linalg.eigh(V[lo - 1])
    w_cur, U_cur = torch.linalg.eigh(V[lo])
    R = U_cur.transpose(-1, -2) @ U_prev                          # prev F0 basis -> cur F0 basis
    _, Wprev = torch.linalg.eigh(out[0])                          # eigvecs of C_b(d-1)
    Wstart = R @ Wprev
    A = Wstart.transpose(-1, -2) @ out[1] @ Wstart
    res[f"date{lo}"] = {"cold_rel_off": float(rel_off(out[1]).mean()),
                        "warm_rel_off": float(rel_off(A).mean())}
print(json.dumps(res))
