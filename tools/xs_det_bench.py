"""CS-WLS at the bench shape (2520 x 5000, P=31, Q=10): default vs bitwise-deterministic kernel,
fp64 and fp32 panel storage (refine on, as the bench and RiskModel.regress run it)."""
import os
import sys
import time

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from llm_driven_multi_factor_model_amd.models.panel import synthetic_panel  # noqa: E402
from llm_driven_multi_factor_model_amd.ops import cross_section as X  # noqa: E402

from llm_driven_multi_factor_model_amd import _native  # noqa: E402

lib = _native.lib()
for dt in (torch.float64, torch.float32):
    p = synthetic_panel(2520, 5000, 31, 10, seed=3, device="cuda:0", missing_frac=0.01, dtype=dt)
    ws = X.xs_wls_workspace(2520, 31, 10, p.styles.device, 5000)
    for det, mode in ((False, 0), (True, 0), (True, 20), (False, 0), (True, 0), (True, 20)):
        lib.mfa_xs_set_mode(mode)  # 20 = deterministic kernel without lane-quarter atomics (A/B)
        out = X.xs_wls(p.styles, p.cap, p.ret, p.ind, 31, deterministic=det, refine=True,
                       workspace=ws)
        torch.cuda.synchronize()
        t0 = time.perf_counter()
        for _ in range(50):
            X.xs_wls(p.styles, p.cap, p.ret, p.ind, 31, deterministic=det, refine=True, out=out,
                     workspace=ws)
        torch.cuda.synchronize()
        print(f"{dt} deterministic={det} mode={mode}: {(time.perf_counter() - t0) / 50 * 1e6:.1f} "
              "us / 2520 dates", flush=True)
lib.mfa_xs_set_mode(0)
