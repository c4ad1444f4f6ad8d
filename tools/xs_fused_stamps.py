"""Phase attribution of the fused CS-WLS kernel from in-kernel s_memtime stamps.

Per date: moments / solve / residual phase lengths (core clocks), and how many workgroups were
co-resident on a CU while each phase ran (HW_ID + XCC_ID recorded by the kernel).
"""
import ctypes as C
import os
import sys
from collections import defaultdict

import numpy as np
import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from llm_driven_multi_factor_model_amd import _native  # noqa: E402
from llm_driven_multi_factor_model_amd.models import panel as pn  # noqa: E402
from llm_driven_multi_factor_model_amd.ops.cross_section import xs_wls  # noqa: E402

D = int(os.environ.get("D", 2520))
N, P, Q = 5000, 31, 10
dev = torch.device("cuda:0")
p = pn.synthetic_panel(D, N, P, Q, seed=1, device=dev, missing_frac=0.01)
if os.environ.get("SORT", "0") == "1":
    p = pn.order_by_industry(p)
out = xs_wls(p.styles, p.cap, p.ret, p.ind, P, refine=False)
buf = torch.zeros(2 * D, 8, dtype=torch.int64, device=dev)
_native.register("mfa_xs_set_stamps", [C.c_void_p])
_native.register("mfa_xs_set_mode", [C.c_int])
_native.lib().mfa_xs_set_stamps(_native.ptr(buf))
_native.lib().mfa_xs_set_mode(int(os.environ.get("MODE", "2")))
torch.cuda.synchronize()
for _ in range(3):
    xs_wls(p.styles, p.cap, p.ret, p.ind, P, refine=False, out=out)
torch.cuda.synchronize()
_native.lib().mfa_xs_set_stamps(None)
_native.lib().mfa_xs_set_mode(0)
s = buf.cpu().numpy().astype(np.int64)
ss = s[D:].astype(np.float64)
s = s[:D]
t = s[:, :4].astype(np.float64)
t0 = t[:, 0].min()
print(f"D={D} span {t[:, 3].max() - t0:.0f} clk")
for i, n in enumerate(["moments", "solve", "resid"]):
    dt = t[:, i + 1] - t[:, i]
    print(f"  {n:8s} median {np.median(dt):8.0f}  p10 {np.percentile(dt, 10):8.0f}  p90 {np.percentile(dt, 90):8.0f}")
hw, xcc = s[:, 4], s[:, 5]
cu = ((hw >> 8) & 0xF) | (((hw >> 13) & 0x7) << 4) | (((hw >> 12) & 1) << 7) | ((xcc & 0xF) << 8)
by = defaultdict(list)
for d in range(D):
    by[int(cu[d])].append(d)
print(f"  distinct CU ids {len(by)}; dates per CU median {np.median([len(v) for v in by.values()]):.0f}")
# co-residency: for each date's moments phase, how many other dates on the same CU overlap it
ov = []
for v in by.values():
    for d in v:
        a, b = t[d, 0], t[d, 1]
        ov.append(sum(1 for e in v if e != d and t[e, 0] < b and t[e, 3] > a))
print(f"  overlapping WGs during a date's moments phase: mean {np.mean(ov):.2f}  max {max(ov)}")
starts = np.sort(t[:, 0] - t0)
print(f"  start times: 256th {starts[255]:.0f}  512th {starts[min(511, D - 1)]:.0f}  last {starts[-1]:.0f}")
names = ["load", "totals+MID+at", "Y+MFMA", "cholesky+solve", "industries+store"]
for i, n in enumerate(names):
    dt = ss[:, i + 1] - ss[:, i]
    print(f"  solve/{n:18s} median {np.median(dt):8.0f}  p90 {np.percentile(dt, 90):8.0f}")
