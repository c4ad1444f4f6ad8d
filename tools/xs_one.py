"""Run one CS-WLS kernel variant a few times (for rocprofv3 PMC collection)."""
import ctypes as C
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from llm_driven_multi_factor_model_amd import _native  # noqa: E402
from llm_driven_multi_factor_model_amd.models.panel import synthetic_panel  # noqa: E402

v = int(sys.argv[1]) if len(sys.argv) > 1 else 0
D = int(sys.argv[2]) if len(sys.argv) > 2 else 2520
N = int(sys.argv[3]) if len(sys.argv) > 3 else 5000
P, Q = 31, 10
dev = torch.device("cuda:0")
p = synthetic_panel(D, N, P, Q, seed=1, device=dev, missing_frac=0.01)
K = 1 + P + Q
f = torch.empty(D, K, dtype=torch.float64, device=dev)
e = torch.empty(D, N, dtype=torch.float32, device=dev)
r2 = torch.empty(D, dtype=torch.float64, device=dev)
st = torch.empty(D, Q + 2, dtype=torch.float64, device=dev)
s = torch.empty(D, dtype=torch.int32, device=dev)
ws = torch.empty(_native.query("mfa_xs_wls_workspace", D, N, P, Q), dtype=torch.uint8, device=dev)
for _ in range(3):
    _native.call("mfa_xs_wls_variant", _native.ptr(p.styles), _native.ptr(p.cap), _native.ptr(p.ret),
                 _native.ptr(p.ind), D, N, P, v, _native.ptr(f), _native.ptr(e), _native.ptr(r2),
                 _native.ptr(st), _native.ptr(s), _native.ptr(ws), _native.stream(dev))
torch.cuda.synchronize()
