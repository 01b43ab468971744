"""Lab tool (not product): achievable HBM rate of read/write mixes at the backbone's tensor
sizes, torch elementwise kernels timed with events (calibration for the 1x1-conv roofline)."""
import torch

dev = "cuda"
def t(fn, iters=20):
    fn(); torch.cuda.synchronize()
    a, b = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    a.record()
    for _ in range(iters): fn()
    b.record(); torch.cuda.synchronize()
    return a.elapsed_time(b) / iters

for mb in (88, 177, 354):
    n = mb * 1024 * 1024 // 2
    x = torch.randn(n, device=dev, dtype=torch.bfloat16)
    y = torch.randn(n, device=dev, dtype=torch.bfloat16)
    z = torch.empty_like(x)
    ms = t(lambda: z.copy_(x)); print(f"{mb:4d} MB copy  1R1W {2*mb/ms/1e3*1.048576:.2f} TB/s")
    ms = t(lambda: torch.add(x, y, out=z)); print(f"{mb:4d} MB add   2R1W {3*mb/ms/1e3*1.048576:.2f} TB/s")
    ms = t(lambda: z.fill_(1.0)); print(f"{mb:4d} MB fill  0R1W {mb/ms/1e3*1.048576:.2f} TB/s")
    ms = t(lambda: x.sum()); print(f"{mb:4d} MB sum   1R0W {mb/ms/1e3*1.048576:.2f} TB/s")
