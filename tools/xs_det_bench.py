"""CS-WLS at the bench shape (2520 x 5000, P=31, Q=10): default vs bitwise-deterministic kernel."""
import os
import sys
import time

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from llm_driven_multi_factor_model_amd.models.panel import synthetic_panel  # noqa: E402
from llm_driven_multi_factor_model_amd.ops import cross_section as X  # noqa: E402

p = synthetic_panel(2520, 5000, 31, 10, seed=3, device="cuda:0", missing_frac=0.01)
for det in (False, True, False, True):
    out = X.xs_wls(p.styles, p.cap, p.ret, p.ind, 31, deterministic=det, refine=False)
    ws = X.xs_wls_workspace(2520, 31, 10, p.styles.device, 5000)
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    for _ in range(50):
        X.xs_wls(p.styles, p.cap, p.ret, p.ind, 31, deterministic=det, refine=False, out=out, workspace=ws)
    torch.cuda.synchronize()
    print(f"deterministic={det}: {(time.perf_counter() - t0) / 50 * 1e6:.1f} us / 2520 dates", flush=True)
