"""Lab tool (not product): what the vendor GEMM (torch.matmul -> hipBLASLt) reaches on the
forward's plain-GEMM shapes, for calibrating the hand-written kernels (bf16, B = 64)."""
import torch

def t(fn, iters=20):
    fn(); torch.cuda.synchronize()
    a, b = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    a.record()
    for _ in range(iters): fn()
    b.record(); torch.cuda.synchronize()
    return a.elapsed_time(b) / iters

for name, M, N, K in [("neck s16 taps", 43264, 2304, 1024), ("ffn linear1", 173056, 2048, 256),
                      ("ffn linear2", 173056, 256, 2048), ("l3 conv1", 43264, 256, 1024),
                      ("enc qk", 173056, 512, 256), ("l2 conv3", 173056, 512, 128), ("sq 8192", 8192, 8192, 8192)]:
    A = torch.randn(M, K, device="cuda", dtype=torch.bfloat16)
    W = torch.randn(N, K, device="cuda", dtype=torch.bfloat16)
    C = torch.empty(M, N, device="cuda", dtype=torch.bfloat16)
    ms = t(lambda: torch.matmul(A, W.t(), out=C))
    print(f"{name:14s} M={M:6d} N={N:5d} K={K:5d}  {ms:.3f} ms  {2*M*N*K/ms/1e9:7.1f} TF/s  {(M*K+N*K+M*N)*2/ms/1e9:6.2f} TB/s")
