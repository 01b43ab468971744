"""Short-K GEMM microbenchmark at the bench's shapes (B=64, 416x416): each launch timed alone
through spe_debug_gemm, with the kernel family that served it, next to a torch copy of the same
byte count (the achievable read+write rate on this box).  SPE_SGEMM=0 in the environment forces
the tile-per-workgroup kernels for an A/B.

usage: python scripts/gemm_bench.py [--iters 20] [--only name,...]
"""
import argparse
import ctypes
import os
import sys

import torch

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(REPO, "satellite-pose-estimation_amd"))
from spe import _lib  # noqa: E402

B, T = 64, 2704
# name: (M, K, N, residual, ln, vt, relu)
SHAPES = {
    "l1.c1first": (B * 104 * 104, 64, 64, False, False, False, True),
    "l1.c1": (B * 104 * 104, 256, 64, False, False, False, True),
    "l1.c3": (B * 104 * 104, 64, 256, True, False, False, True),
    "l1.ds": (B * 104 * 104, 64, 256, False, False, False, False),
    "l2.c1first": (B * 104 * 104, 256, 128, False, False, False, True),
    "l2.c1": (B * 52 * 52, 512, 128, False, False, False, True),
    "l2.c3": (B * 52 * 52, 128, 512, True, False, False, True),
    "l3.c1first": (B * 52 * 52, 512, 256, False, False, False, True),
    "l3.c3": (B * 26 * 26, 256, 1024, True, False, False, True),
    "neck.s8": (B * T, 512, 256, False, False, False, False),
    "enc.qk": (B * T, 256, 512, "periodic", False, False, False),
    "enc.qk_noR": (B * T, 256, 512, False, False, False, False),
    "enc.q_R": (B * T, 256, 256, "periodic", False, False, False),
    "enc.q_noR": (B * T, 256, 256, False, False, False, False),
    "enc.o_noLN": (B * T, 256, 256, True, False, False, False),
    "enc.v": (B * T, 256, 256, False, False, True, False),
    "enc.o": (B * T, 256, 256, True, True, False, False),
}


def p(t):
    return ctypes.c_void_p(t.data_ptr()) if t is not None else None


def timeit(fn, iters):
    fn()
    torch.cuda.synchronize()
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    e0.record()
    for _ in range(iters):
        fn()
    e1.record()
    torch.cuda.synchronize()
    return e0.elapsed_time(e1) / iters


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--iters", type=int, default=20)
    ap.add_argument("--only", default="")
    a = ap.parse_args()
    L = _lib.lib()
    dev = torch.device("cuda", 0)
    bf = torch.bfloat16
    g = torch.Generator(device="cpu").manual_seed(0)
    names = [n for n in SHAPES if not a.only or n in a.only.split(",")]
    for name in names:
        M, K, N, res, ln, vt, relu = SHAPES[name]
        A = torch.randn(M, K, generator=g).to(dev, bf)
        W = (torch.randn(N, K, generator=g) / K ** 0.5).to(dev, bf)
        bias = torch.randn(N, generator=g).to(dev)
        R, ldr, rp = None, 0, 0
        if res == "periodic":
            R, ldr, rp = torch.randn(T, N, generator=g).to(dev, bf), N, T
        elif res:
            R, ldr = torch.randn(M, N, generator=g).to(dev, bf), N
        gam = torch.randn(N, generator=g).to(dev) if ln else None
        bet = torch.randn(N, generator=g).to(dev) if ln else None
        C = torch.empty(M * N, dtype=bf, device=dev)
        vt_T, vt_B = (T, M // T) if vt else (0, 0)

        def fn():
            rc = L.spe_debug_gemm(None, 0, 0, p(A), K, None, 0, 1, 0, 0, 0, 1, 1, 1, 0, p(W), K, M, N, K, p(bias), p(R),
                                  ldr, int(relu), p(C), N, 0, vt_T, vt_B, rp, p(gam), p(bet), 0)
            assert rc == 0, L.spe_last_error()

        ms = timeit(fn, a.iters)
        path = L.spe_debug_gemm_path()
        nbytes = (M * K + N * K + M * N + (M * N if res is True else 0)) * 2
        src = torch.empty(nbytes // 4, dtype=torch.int16, device=dev)
        dst = torch.empty_like(src)
        cms = timeit(lambda: dst.copy_(src), a.iters)
        del src, dst
        print(f"{name:12s} path={path} {ms * 1e3:8.1f} us  {nbytes / ms / 1e9:5.2f} TB/s   "
              f"(copy of the same bytes {cms * 1e3:7.1f} us, {nbytes / cms / 1e9:5.2f} TB/s)", flush=True)
        del A, W, R, C


if __name__ == "__main__":
    main()
