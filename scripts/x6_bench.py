"""Per-shape timing of the fp32 parity GEMM paths (exact-f32 MFMA, fp32x3, fp32x6) at the bench
workload's shapes (B = 64, 416x416), through spe_debug_gemm.  Prints ms per launch and model
TFLOP/s per dtype.

    python scripts/x6_bench.py [--iters 10]
"""
import argparse
import ctypes
import os
import sys

import torch

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(REPO, "satellite-pose-estimation_amd"))
from spe import _lib  # noqa: E402

DT = {"fp32": _lib.SPE_DTYPE_F32, "fp32x3": _lib.SPE_DTYPE_F32X3, "fp32x6": _lib.SPE_DTYPE_F32X6,
      "fp32x6bp": _lib.SPE_DTYPE_F32X6,       # bp: weights pre-split into bf16 planes, as the model has them
      "fp32h3": _lib.SPE_DTYPE_F32H3}         # scaled fp16 planes + per-channel scales, as the model has them
# name: (M, N, K) linear, or (B, H, Cin, Cout, k, stride, pad) conv
SHAPES = {
    "enc.ffn1": (64 * 2704, 2048, 256), "cross.k": (64 * 2704, 1536, 256), "enc.ffn2": (64 * 2704, 256, 2048), "enc.qk": (64 * 2704, 512, 256),
    "l1.conv1": (64 * 104 * 104, 64, 256), "l3.conv3": (64 * 26 * 26, 1024, 256),
    "l1.3x3": (64, 104, 64, 64, 3, 1, 1), "l2.3x3": (64, 52, 128, 128, 3, 1, 1), "l3.3x3": (64, 26, 256, 256, 3, 1, 1),
    "neck.3x3": (64, 52, 512, 256, 3, 1, 1), "l4.3x3": (64, 13, 512, 512, 3, 1, 1),
    "l4.conv1": (64 * 169, 512, 2048), "l4.conv3": (64 * 169, 2048, 512), "stem": (64, 416, 4, 64, 7, 2, 3),
}


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--iters", type=int, default=10)
    ap.add_argument("--only", default="")
    ap.add_argument("--dtypes", default=",".join(DT))
    ap.add_argument("--batch", type=int, default=64, help="images (the shapes' M scale with it)")
    a = ap.parse_args()
    L = _lib.lib()
    dev = torch.device("cuda", 0)
    p = lambda t: ctypes.c_void_p(t.data_ptr())
    for name, sh in SHAPES.items():
        if a.only and a.only not in name:
            continue
        if len(sh) == 3:
            M, N, K = sh
            M = M // 64 * a.batch
            conv = (0, 0, 0, 1, 1, 1, 0)
            A = torch.randn(M, K, device=dev)
            mode = 0
        else:
            B, H, Cin, N, k, st, pd = sh
            B = a.batch
            Ho = (H + 2 * pd - k) // st + 1
            M, K = B * Ho * Ho, Cin * k * k
            conv = (H, H, Cin, k, k, st, pd)
            A = torch.randn(B * H * H, Cin, device=dev)
            mode = 2
        ldb = (K + 63) // 64 * 64
        W = torch.randn(N, ldb, device=dev) / K ** 0.5
        bias = torch.randn(N, device=dev)
        C = torch.empty(M, N, device=dev)
        h = W.to(torch.bfloat16)
        r = W - h.float()
        m_ = r.to(torch.bfloat16)
        planes = torch.stack([h, m_, (r - m_.float()).to(torch.bfloat16)]).contiguous()
        am = W.abs().amax(1).double()
        sc = torch.pow(2.0, 13 - torch.frexp(am).exponent.double()).float()[:, None]
        hh = (W * sc).to(torch.float16)
        h3p = torch.stack([hh, (W * sc - hh.float()).to(torch.float16)]).contiguous()
        h3s = (1.0 / sc[:, 0]).contiguous()
        amax_a = A.abs().max().reshape(1).contiguous()
        row = [name]
        for dn, dt in DT.items():
            if dn not in a.dtypes.split(","):
                continue
            if dn == "fp32h3":
                fn = lambda: L.spe_debug_gemm_h3(None, mode, p(A), K if mode == 0 else 0, *conv, ldb, M, N, K, p(bias),
                                                 None, 0, 1, p(C), N, p(h3p), N, p(h3s), p(amax_a), None, 0.0)
            elif dn == "fp32x6bp":
                fn = lambda: L.spe_debug_gemm_planes(None, dt, mode, p(A), K if mode == 0 else 0, None, 0, 1, *conv, p(W),
                                                     ldb, M, N, K, p(bias), None, 0, 1, p(C), N, p(planes), N)
            else:
                fn = lambda: L.spe_debug_gemm(None, dt, mode, p(A), K if mode == 0 else 0, None, 0, 1, *conv, p(W), ldb,
                                              M, N, K, p(bias), None, 0, 1, p(C), N, 0, 0, 0, 0, None, None, 0)
            assert fn() == 0, L.spe_last_error()
            torch.cuda.synchronize()
            e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
            e0.record()
            for _ in range(a.iters):
                fn()
            e1.record()
            torch.cuda.synchronize()
            ms = e0.elapsed_time(e1) / a.iters
            row.append(f"{dn} {ms:.3f} ms {2.0 * M * N * K / ms / 1e9:.0f} TF/s")
        print("  ".join(row), flush=True)


if __name__ == "__main__":
    main()
