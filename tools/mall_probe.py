"""Read bandwidth vs working-set size (1 GPU): repeated reductions over buffers that fit the
256 MB Infinity Cache (MALL) or not.  Tells whether a re-read served by the MALL is cheaper for
the CUs than one served by HBM."""
import json
import torch

dev = torch.device("cuda:0")
out = {}
for mb in (16, 64, 128, 192, 256, 512, 2048):
    n = mb * 1024 * 1024 // 8
    x = torch.ones(n, dtype=torch.float64, device=dev)
    for _ in range(5):
        x.sum()
    torch.cuda.synchronize()
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    reps = max(5, 4096 // mb)
    e0.record()
    for _ in range(reps):
        x.sum()
    e1.record()
    torch.cuda.synchronize()
    ms = e0.elapsed_time(e1) / reps
    out[f"{mb}MB"] = round(n * 8 / ms / 1e9, 2)
    del x
print(json.dumps({"read_TB_s_by_working_set": out}))
