"""HBM read-bandwidth probe: torch reduction over a large fp32 buffer."""
import torch
x = torch.empty(256 * 1024 * 1024, dtype=torch.float32, device="cuda").fill_(1.0)  # 1 GiB
for _ in range(3):
    x.sum()
torch.cuda.synchronize()
e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
e0.record()
for _ in range(20):
    x.sum()
e1.record()
torch.cuda.synchronize()
ms = e0.elapsed_time(e1) / 20
print(f"sum 1GiB: {ms*1e3:.1f} us  {x.numel()*4/ms/1e9:.2f} TB/s")
