"""Convergence tolerance / sweep cap of the MC bias Jacobi vs time and accuracy (1 GPU).

Inputs are the pipeline's own: Newey-West covariances of the factor returns regressed from a
synthetic 2520 x 5000 fp64 panel, M = 100 draw covariances.  For every (tol, max_sweeps) it
times ``mfa_eigen_adjust`` and compares the bias multipliers with (a) the default setting and
(b) a float64 LAPACK ``eigh`` oracle (CPU) on a subset of dates.

    python tools/eigen_tol.py          # env: SETTINGS="1e-15:30,1e-12:30,..." SUB=24 MODES=0,3

``MODES`` are bias-solver modes (``mfa_eigen_set_bias_mode``: 0 = pair-block Jacobi, 3 =
Householder tridiagonal + Laguerre; mode 3 ignores tol / max_sweeps).
"""
import json
import os
import statistics
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from llm_driven_multi_factor_model_amd import _native  # noqa: E402
from llm_driven_multi_factor_model_amd.models.panel import synthetic_panel  # noqa: E402
from llm_driven_multi_factor_model_amd.models.risk_model import RiskModel  # noqa: E402
from llm_driven_multi_factor_model_amd.ops import eigen  # noqa: E402
from llm_driven_multi_factor_model_amd.utils.config import preset  # noqa: E402


def main():
    dev = torch.device("cuda:0")
    D = int(os.environ.get("D", 2520))
    M = int(os.environ.get("M", 100))
    p = synthetic_panel(D, 5000, 31, 10, seed=3, device=dev, missing_frac=0.01, dtype=torch.float64)
    rm = RiskModel(p, preset("reference"))
    rm.regress()
    rm.newey_west()
    F0 = rm.nw_cov.contiguous()
    K = F0.shape[-1]
    w, U = eigen.eigh(F0)
    valid = torch.isfinite(w).all(-1) & (w.min(-1).values >= 0)
    w = torch.where(valid[:, None], w.clamp_min(0.0), w).contiguous()
    U = U.contiguous()
    dv = valid.to(torch.int32).contiguous()
    Cz = eigen.mc_cov(M, K, D, 1, dev)
    Fh = torch.empty(D, K, K, dtype=torch.float64, device=dev)
    ws = torch.empty(D * M * K, dtype=torch.float64, device=dev)
    ev0, ev1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)

    def run(tol, ms):
        vb = torch.empty(D, K, dtype=torch.float64, device=dev)
        _native.call("mfa_eigen_adjust", _native.ptr(w), _native.ptr(U), _native.ptr(dv), D, K, M,
                     _native.ptr(Cz), 1.4, ms, tol, _native.ptr(ws), _native.ptr(Fh),
                     _native.ptr(vb), _native.stream(dev))
        return vb

    # CPU oracle on a subset of valid dates
    sub = torch.nonzero(valid).flatten()[:: max(1, int(valid.sum()) // int(os.environ.get("SUB", 24)))]
    wc, Czc = w[sub].cpu(), Cz.cpu()
    vm_ref = []
    for i in range(len(sub)):
        s = torch.sqrt(wc[i])
        lam, V = torch.linalg.eigh(s[None, :, None] * Czc * s[None, None, :])
        lam, V = lam.flip(-1), V.flip(-1)
        vm_ref.append((((V * V) * wc[i][None, :, None]).sum(1) / lam).mean(0))
    vm_ref = torch.stack(vm_ref)
    v_ref = 1.4 * (torch.sqrt(vm_ref) - 1.0) + 1.0
    settings = [s.split(":") for s in os.environ.get(
        "SETTINGS", "1e-15:30,1e-14:30,1e-13:30,1e-12:30,1e-11:30,1e-10:30,1e-15:8,1e-15:7,1e-15:6,1e-15:5").split(",")]
    lib = _native.lib()
    lib.mfa_eigen_set_bias_mode(0)
    base = run(eigen.TOL, eigen.MAX_SWEEPS)
    for mode in [int(x) for x in os.environ.get("MODES", "0").split(",")]:
        lib.mfa_eigen_set_bias_mode(mode)
        for tol, ms in settings:
            tol, ms = float(tol), int(ms)
            vb = run(tol, ms)
            ts = []
            for _ in range(3):
                ev0.record()
                run(tol, ms)
                ev1.record()
                ev1.synchronize()
                ts.append(ev0.elapsed_time(ev1))
            rel_base = ((vb - base).abs() / base.abs()).nan_to_num(0).max().item()
            rel_ref = ((vb[sub].cpu() - v_ref).abs() / v_ref.abs()).max().item()
            print(json.dumps({"mode": mode, "tol": tol, "max_sweeps": ms,
                              "ms": round(statistics.median(ts), 2),
                              "max_rel_dv_vs_default": rel_base, "max_rel_dv_vs_lapack": rel_ref,
                              "nan_mismatch": int((vb.isnan() != base.isnan()).sum())}), flush=True)
    lib.mfa_eigen_set_bias_mode(0)


if __name__ == "__main__":
    main()
