"""Latency attribution of the CS-WLS solve kernel (K2) from in-kernel s_memtime stamps."""
import ctypes as C
import os
import sys

import numpy as np
import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from llm_driven_multi_factor_model_amd import _native  # noqa: E402
from llm_driven_multi_factor_model_amd.models.panel import synthetic_panel  # noqa: E402
from llm_driven_multi_factor_model_amd.ops.cross_section import xs_wls  # noqa: E402

D = int(sys.argv[1]) if len(sys.argv) > 1 else 2520
N, P, Q = 5000, 31, 10
dev = torch.device("cuda:0")
p = synthetic_panel(D, N, P, Q, seed=1, device=dev, missing_frac=0.01)
out = xs_wls(p.styles, p.cap, p.ret, p.ind, P, refine=False)
buf = torch.zeros(D, 8, dtype=torch.int64, device=dev)
_native.register("mfa_xs_set_stamps", [C.c_void_p])
_native.lib().mfa_xs_set_stamps(_native.ptr(buf))
torch.cuda.synchronize()
xs_wls(p.styles, p.cap, p.ret, p.ind, P, refine=False, out=out)
torch.cuda.synchronize()
_native.lib().mfa_xs_set_stamps(None)
s = buf.cpu().numpy().astype(np.float64)
names = ["load", "totals+MID+at", "Y+MFMA", "cholesky+solve", "industries+store"]
print(f"D={D}  span(first start -> last end) = {s[:, 5].max() - s[:, 0].min():.0f} clk; "
      f"per-date total median {np.median(s[:, 5] - s[:, 0]):.0f} clk")
for i, n in enumerate(names):
    dt = s[:, i + 1] - s[:, i]
    print(f"  {n:18s} median {np.median(dt):8.0f}  p90 {np.percentile(dt, 90):8.0f}  max {dt.max():8.0f}")
st = s[:, 0] - s[:, 0].min()
print(f"  start spread: median {np.median(st):.0f}  max {st.max():.0f} clk")
