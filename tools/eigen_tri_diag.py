"""Where do the two bias solvers disagree?  Per-(date, sim) bias ratios of the Jacobi (mode 0)
and tridiagonal (mode 3) solvers on the pipeline's inputs, the worst entries checked against
LAPACK on the CPU (eigenvalue gaps printed)."""
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


def main():
    dev = torch.device("cuda:0")
    D, M = int(os.environ.get("D", 2520)), int(os.environ.get("M", 100))
    p = synthetic_panel(D, 5000, 31, 10, seed=3, device=dev, missing_frac=0.01, dtype=torch.float64)
    rm = RiskModel(p, preset("reference"))
    rm.regress()
    rm.newey_west()
    F0 = rm.nw_cov.contiguous()
    K = F0.shape[-1]
    w, U = eigen.eigh(F0)
    valid = torch.isfinite(w).all(-1) & (w.min(-1).values >= 0)
    w = torch.where(valid[:, None], w.clamp_min(0.0), w).contiguous()
    dv = valid.to(torch.int32).contiguous()
    Cz = eigen.mc_cov(M, K, D, 1, dev)
    lib = _native.lib()
    per = {}
    for mode in (0, 3):
        lib.mfa_eigen_set_bias_mode(mode)
        ws = torch.empty(D * M * K, dtype=torch.float64, device=dev)
        Fh = torch.empty(D, K, K, dtype=torch.float64, device=dev)
        vb = torch.empty(D, K, dtype=torch.float64, device=dev)
        _native.call("mfa_eigen_adjust", _native.ptr(w), _native.ptr(U.contiguous()), _native.ptr(dv),
                     D, K, M, _native.ptr(Cz), 1.4, eigen.MAX_SWEEPS, eigen.TOL, _native.ptr(ws),
                     _native.ptr(Fh), _native.ptr(vb), _native.stream(dev))
        per[mode] = ws.view(D, M, K).cpu()
    lib.mfa_eigen_set_bias_mode(0)
    a, b = per[0], per[3]
    rel = ((a - b).abs() / a.abs()).nan_to_num(0)
    print(json.dumps({"max_rel": rel.max().item(), "n_rel_gt_1e-8": int((rel > 1e-8).sum()),
                      "n_rel_gt_1e-10": int((rel > 1e-10).sum()), "n": rel.numel()}), flush=True)
    flat = torch.topk(rel.flatten(), 6).indices
    wc, Czc = w.cpu(), Cz.cpu()
    bad = []
    for idx in flat.tolist():
        d, m, k = idx // (M * K), (idx // K) % M, idx % K
        s = torch.sqrt(wc[d])
        A = s[:, None] * Czc[m] * s[None, :]
        lam, V = torch.linalg.eigh(A)
        lam, V = lam.flip(-1), V.flip(-1)
        vr = ((V * V) * wc[d][:, None]).sum(0) / lam
        bad.append({"A": A, "D0": wc[d], "k": k, "jacobi": a[d, m].clone(), "tridiag": b[d, m].clone()})
        gaps = (lam[:-1] - lam[1:]) / lam[:-1].abs()
        print(json.dumps({"d": d, "m": m, "k": k, "jacobi": a[d, m, k].item(), "tridiag": b[d, m, k].item(),
                          "lapack": vr[k].item(), "lam_k": lam[k].item(),
                          "relgap_prev": gaps[k - 1].item() if k > 0 else None,
                          "relgap_next": gaps[k].item() if k < K - 1 else None,
                          "lam_min": lam[-1].item(), "lam_max": lam[0].item()}), flush=True)
    os.makedirs("gpurun_out", exist_ok=True)
    torch.save(bad, "gpurun_out/eigen_tri_bad.pt")


if __name__ == "__main__":
    main()
