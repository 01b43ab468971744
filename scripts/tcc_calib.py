"""TCC counter calibration: one streaming read of a known byte count (sum over a 256 MiB fp32 buffer)
and one streaming copy, for reading TCC_HIT / TCC_MISS / FETCH_SIZE in bytes (run under rocprofv3 --pmc)."""
import torch

n = 64 << 20                                   # 64 Mi floats = 256 MiB
x = torch.ones(n, dtype=torch.float32, device="cuda")
torch.cuda.synchronize()
for _ in range(2):
    s = x.sum()                                # reads 256 MiB once
    y = x.clone()                              # reads 256 MiB, writes 256 MiB
torch.cuda.synchronize()
print("done", float(s))
