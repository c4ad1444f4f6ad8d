"""Per-phase instruction budget of the production bias solver (K = 42 instantiation, VERDICT r05
item 3): runs the production kernel (bias mode 5) and its phase ablations (A/B library modes
71 = no Laguerre iterations, 72 = no eigenvectors / back-transform, 74 = no tridiagonalisation)
on the same inputs, one eigen_risk_adjust call each.  Run under rocprofv3 --pmc with the A/B
library; the summary (tools/bias_phase_budget.py --summarize DIR) turns the per-kernel counters
into per-problem (per-wave) counts and the per-phase differences.

    MFA_HIP_LIB=.../_lib/ab/libmfa_hip.so rocprofv3 --kernel-trace --pmc SQ_WAVES SQ_INSTS_VALU \
        SQ_INSTS_SALU SQ_INSTS_LDS SQ_INSTS_VALU_FMA_F64 SQ_INSTS_VALU_MUL_F64 SQ_INSTS_VALU_ADD_F64 \
        SQ_INSTS_VALU_TRANS_F64 -d DIR -o run --output-format csv -- python3 tools/bias_phase_budget.py
    python3 tools/bias_phase_budget.py --summarize DIR
"""
import collections
import csv
import ctypes as C
import glob
import json
import os
import re
import sys

MODES = {5: "production", 71: "no Laguerre", 72: "no eigenvectors / back-transform",
         73: "setup + tridiagonalisation", 77: "setup only"}
ABL_OF_MODE = {5: 0, 71: 1, 72: 2, 73: 3, 77: 7}


def run(D=252, M=100):
    """The pipeline's own inputs: the Newey-West matrices of a 252-date x 5000-stock synthetic
    panel (K = 42), M = 100 draws of length D."""
    import torch
    sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
    from llm_driven_multi_factor_model_amd import _native
    from llm_driven_multi_factor_model_amd.models.panel import synthetic_panel
    from llm_driven_multi_factor_model_amd.models.risk_model import RiskModel
    from llm_driven_multi_factor_model_amd.ops import eigen
    from llm_driven_multi_factor_model_amd.utils.config import preset
    p = synthetic_panel(D, 5000, 31, 10, seed=3, missing_frac=0.01, dtype=torch.float64, device="cuda:0")
    m = RiskModel(p, preset("reference"))
    m.regress()
    m.newey_west()
    F0 = m.nw_cov.contiguous()
    F0 = F0[torch.isfinite(F0.reshape(D, -1)).all(-1)].contiguous()
    Cz = eigen.mc_cov(M, F0.shape[-1], D, 1, "cuda:0")
    lib = _native.lib()
    lib.mfa_eigen_set_bias_mode.argtypes = [C.c_int]
    for mode in MODES:
        assert lib.mfa_eigen_set_bias_mode(mode) == 0, mode
        eigen.eigen_risk_adjust(F0, M=M, Cz=Cz, return_bias=True)
        torch.cuda.synchronize()
    lib.mfa_eigen_set_bias_mode(5)


def abl_of(name):
    """ABL template argument of a mc_bias_tri2_kernel<42, true, ABL, ...> instantiation."""
    m = re.search(r"mc_bias_tri2_kernel<42, true, (\d+), 4, false,", name) or \
        re.search(r"mc_bias_tri2_kernelILi42ELb1ELi(\d+)E", name)   # demangled or mangled
    return int(m.group(1)) if m else None


def summarize(d):
    agg = collections.defaultdict(lambda: collections.defaultdict(float))
    for f in glob.glob(os.path.join(d, "**", "*counter_collection.csv"), recursive=True):
        for r in csv.DictReader(open(f)):
            a = abl_of(r["Kernel_Name"])
            if a is not None:
                agg[a][r["Counter_Name"]] += float(r["Counter_Value"])
    per = {}
    for a, c in sorted(agg.items()):
        w = c.get("SQ_WAVES", 0.0)
        per[a] = {k: round(v / w) for k, v in c.items() if k != "SQ_WAVES"} if w else {}
    full = per.get(0, {})
    name = {abl: MODES[mode] for mode, abl in ABL_OF_MODE.items()}
    out = {"per_problem": {name.get(a, str(a)): v for a, v in per.items()}, "phase": {}}
    if all(a in per for a in (0, 1, 2, 3, 7)):
        # setup = ABL 7 alone; tridiagonalisation = ABL 3 - ABL 7 (both skip the data-dependent
        # phases); Laguerre = full - ABL 1; eigenvectors + back-transform = full - ABL 2
        keys = list(full)
        ph = {"setup (C_z S scaling, diagonal ranks, guesses)": per[7],
              "Householder tridiagonalisation": {k: per[3][k] - per[7][k] for k in keys},
              "Laguerre eigenvalues": {k: full[k] - per[1][k] for k in keys},
              "twisted eigenvectors + back-transform + ratio": {k: full[k] - per[2][k] for k in keys}}
        ph["sum of phases"] = {k: sum(v[k] for v in list(ph.values())) for k in keys}
        ph["production (measured)"] = full
        out["phase"] = ph
    print(json.dumps(out, indent=1))


if __name__ == "__main__":
    if len(sys.argv) > 2 and sys.argv[1] == "--summarize":
        summarize(sys.argv[2])
    else:
        run()
