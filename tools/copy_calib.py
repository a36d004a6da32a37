"""Calibrate achievable HBM bandwidth on this box: device-to-device copies of W-MSA-sized
buffers (read + write bytes / time)."""
import torch

for mb in (256, 617, 2048):
    n = mb * 2**20 // 4
    x = torch.empty(n, device="cuda")
    y = torch.empty_like(x)
    for _ in range(3):
        y.copy_(x)
    s, e = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    torch.cuda.synchronize()
    s.record()
    for _ in range(20):
        y.copy_(x)
    e.record()
    torch.cuda.synchronize()
    t = s.elapsed_time(e) / 20
    print(f"copy {mb:5d} MB: {t * 1e3:8.1f} us  {2 * n * 4 / t / 1e6:7.0f} GB/s")
