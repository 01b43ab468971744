"""GPU: each kernel family against a plain torch fp32 reference of the same op, through the
C ABI test hooks, at ragged / edge shapes (partial tiles, strides, channel slices).

Tolerances: fp32 storage (exact-f32 MFMA) max|d| <= 1e-4 * scale; bf16 storage: inputs are
pre-rounded to bf16 so only accumulation order and the bf16 output rounding remain,
max|d| <= 1e-2 * scale (scale = max|reference|, at least 1).
"""
import ctypes
import math
import os

import numpy as np

import pytest
import torch
import torch.nn.functional as F
import torch.nn.functional as F_

from spe import _lib

pytestmark = pytest.mark.gpu

DT = {"bf16": (_lib.SPE_DTYPE_BF16, torch.bfloat16, 1e-2), "fp32": (_lib.SPE_DTYPE_F32, torch.float32, 1e-4),
      "fp32x3": (_lib.SPE_DTYPE_F32X3, torch.float32, 1e-4),
      "fp32x6": (_lib.SPE_DTYPE_F32X6, torch.float32, 1e-4),
      "fp32h3": (_lib.SPE_DTYPE_F32H3, torch.float32, 1e-4),
      "fp16": (_lib.SPE_DTYPE_F16, torch.float16, 2e-3)}


def _p(t):
    return ctypes.c_void_p(t.data_ptr()) if t is not None else None


def _close(got, ref, tol):
    scale = max(1.0, ref.abs().max().item())
    err = (got.float() - ref.float()).abs().max().item()
    assert err <= tol * scale, (err, scale)


def _gemm(dtype, mode, A, W, M, N, K, lda, ldb, C, ldc, bias=None, R=None, ldr=0, relu=0, P=None, ldp=0, prow=1,
          conv=(0, 0, 0, 1, 1, 1, 0), out_f32=0, vt=(0, 0), r_period=0, ln=(None, None), out_f16=0):
    L = _lib.lib()
    H, Wd, Cin, KH, KW, stride, pad = conv
    rc = L.spe_debug_gemm(None, DT[dtype][0], mode, _p(A), lda, _p(P), ldp, prow, H, Wd, Cin, KH, KW, stride, pad,
                          _p(W), ldb, M, N, K, _p(bias), _p(R), ldr, relu, _p(C), ldc, out_f32, vt[0], vt[1], r_period,
                          _p(ln[0]), _p(ln[1]), out_f16)
    assert rc == 0, L.spe_last_error()
    torch.cuda.synchronize()


def _padded_weight(Wt, ldb, dt):
    N, K = Wt.shape
    Wp = torch.zeros(N, ldb, dtype=dt, device=Wt.device)
    Wp[:, :K] = Wt.to(dt)
    return Wp


def _pack_conv(w):
    """[Cout][Cin][kh][kw] -> [Cout][K] in the kernels' K order (spe_kernels.h conv_k_decode):
    channel-block-major ([Cin/64][kh][kw][64]) for multi-tap convs with Cin % 64 == 0, else
    [kh][kw][Cin]."""
    Cout, Cin, kh, kw = w.shape
    if Cin % 64 == 0 and kh * kw > 1:
        return w.reshape(Cout, Cin // 64, 64, kh, kw).permute(0, 1, 3, 4, 2).reshape(Cout, -1)
    return w.permute(0, 2, 3, 1).reshape(Cout, -1)


@pytest.mark.parametrize("dtype", ["bf16", "fp32"])
@pytest.mark.parametrize("M,N,K", [(300, 200, 256), (128, 64, 64), (77, 520, 2048), (5, 12, 192)])
def test_gemm_linear_epilogue(gpu_device, dtype, M, N, K):
    _, dt, tol = DT[dtype]
    g = torch.Generator(device="cpu").manual_seed(M * 7 + N)
    A = torch.randn(M, K, generator=g).to(gpu_device, dt)
    Wt = (torch.randn(N, K, generator=g) / K ** 0.5).to(gpu_device, dt)
    ldb = (K + 63) // 64 * 64
    Wp = _padded_weight(Wt, ldb, dt)
    bias = torch.randn(N, generator=g).to(gpu_device)
    ld = (N + 8 + 7) // 8 * 8                          # row strides must keep 16-byte alignment
    R = torch.randn(M, ld, generator=g).to(gpu_device, dt)
    C = torch.zeros(M, ld, dtype=dt, device=gpu_device)
    _gemm(dtype, 0, A, Wp, M, N, K, K, ldb, C, ld, bias=bias, R=R, ldr=ld, relu=1)
    ref = torch.relu(A.float() @ Wt.float().t() + bias + R[:, :N].float())
    _close(C[:, :N], ref, tol)
    assert (C[:, N:] == 0).all()                       # nothing written past N


@pytest.mark.parametrize("dtype", ["bf16", "fp32"])
@pytest.mark.parametrize("act", [2, 3])
@pytest.mark.parametrize("post", [0, 1])
@pytest.mark.parametrize("M,N,K", [(300, 200, 256), (40000, 64, 128), (33000, 256, 512)])
def test_gemm_activations(gpu_device, dtype, act, post, M, N, K):
    """SiLU / exact GELU epilogues (UNC hybrid encoder ConvNormLayer, AIFI FFN), with the
    residual added before the activation or after it (CSPRepLayer: silu(rep(x1)) + x2); shapes
    reach the few-row, 256-row-tile and 128x128 kernels."""
    _, dt, tol = DT[dtype]
    g = torch.Generator(device="cpu").manual_seed(M + N + act)
    A = torch.randn(M, K, generator=g).to(gpu_device, dt)
    Wt = (torch.randn(N, K, generator=g) / K ** 0.5).to(gpu_device, dt)
    ldb = (K + 63) // 64 * 64
    bias = torch.randn(N, generator=g).to(gpu_device)
    R = torch.randn(M, N, generator=g).to(gpu_device, dt)
    C = torch.zeros(M, N, dtype=dt, device=gpu_device)
    _gemm(dtype, 0, A, _padded_weight(Wt, ldb, dt), M, N, K, K, ldb, C, N, bias=bias, R=R, ldr=N, relu=act | (post << 8))
    y = A.float() @ Wt.float().t() + bias
    f = F.silu if act == 2 else F.gelu
    ref = f(y) + R.float() if post else f(y + R.float())
    _close(C, ref, tol)


@pytest.mark.parametrize("dtype", ["bf16", "fp32"])
@pytest.mark.parametrize("B,H,Cin,Cout", [(2, 16, 64, 128), (64, 32, 256, 512)])
def test_gemm_conv_avgpool_shortcut(gpu_device, dtype, B, H, Cin, Cout):
    """PResNet-vd shortcut AvgPool2d(2, 2, ceil_mode) + 1x1 conv as one 2x2 stride-2 conv with
    w/4 per tap (UNC/nn/backbone/presnet.py:88-101), channel-blocked K order (4 taps)."""
    _, dt, tol = DT[dtype]
    g = torch.Generator(device="cpu").manual_seed(B + Cin)
    x = torch.randn(B, Cin, H, H, generator=g).to(gpu_device, dt)
    w1 = (torch.randn(Cout, Cin, 1, 1, generator=g) / Cin ** 0.5).to(gpu_device)
    ref = F.conv2d(F.avg_pool2d(x.float(), 2, 2, 0, ceil_mode=True), w1)
    w = (w1 / 4).repeat(1, 1, 2, 2).to(dt)
    K = 4 * Cin
    Wp = _padded_weight(_pack_conv(w), K, dt)
    C = torch.zeros(B * (H // 2) ** 2, Cout, dtype=dt, device=gpu_device)
    _gemm(dtype, 2, x.permute(0, 2, 3, 1).contiguous(), Wp, C.shape[0], Cout, K, 0, K, C, Cout,
          conv=(H, H, Cin, 2, 2, 2, 0))
    _close(C, ref.permute(0, 2, 3, 1).reshape(-1, Cout), tol)


@pytest.mark.parametrize("B,S,path", [(2, 416, 2), (1, 416, 1), (1, 64, 0), (3, 130, 0)])
def test_gemm_conv_pair_packed_stem(gpu_device, B, S, path):
    """bf16 stem as registry.cpp packs it: the 7x7/s2/p3 conv over 3 channels run as a 7x8/s2
    conv over the zero-bordered 4-channel input (k = (kh*8 + kw)*4 + ci, kw = 7 and ci = 3 zero),
    16-byte chunks = two adjacent pixels; against torch conv2d on the same bf16 operands.  The
    shapes reach the streaming kernel (path 2, sgemm CP), the 256-row tiles (1) and gemm.hip (0)."""
    dt = torch.bfloat16
    g = torch.Generator(device="cpu").manual_seed(S + B)
    x = torch.randn(B, 3, S, S, generator=g).to(gpu_device, dt)
    w = (torch.randn(64, 3, 7, 7, generator=g) / 12).to(gpu_device, dt)
    bias = torch.randn(64, generator=g).to(gpu_device)
    ref = torch.relu(F.conv2d(x.float(), w.float(), bias, stride=2, padding=3))
    P = S + 6
    xp = torch.zeros(B, P, P, 4, dtype=dt, device=gpu_device)
    xp[:, 3:3 + S, 3:3 + S, :3] = x.permute(0, 2, 3, 1)
    w8 = torch.zeros(64, 7, 8, 4, dtype=dt, device=gpu_device)
    w8[:, :, :7, :3] = w.permute(0, 2, 3, 1)
    Wp = _padded_weight(w8.reshape(64, 224), 256, dt)
    Ho = (P - 7) // 2 + 1
    C = torch.zeros(B * Ho * Ho, 64, dtype=dt, device=gpu_device)
    _gemm("bf16", 2, xp, Wp, C.shape[0], 64, 224, 0, 256, C, 64, bias=bias, relu=1, conv=(P, P, 4, 7, 8, 2, 0))
    if os.environ.get("SPE_SG_STEM", "1") != "0" and os.environ.get("SPE_SGEMM", "1") != "0":
        assert _lib.lib().spe_debug_gemm_path() == path
    _close(C, ref.permute(0, 2, 3, 1).reshape(-1, 64), 2e-2)


@pytest.mark.parametrize("dtype", ["bf16", "fp32"])
def test_gemm_linear_add_and_f32_out(gpu_device, dtype):
    _, dt, tol = DT[dtype]
    M, N, K, prow = 250, 96, 256, 25
    g = torch.Generator(device="cpu").manual_seed(3)
    A = torch.randn(M, K, generator=g).to(gpu_device, dt)
    P = torch.randn(prow, K, generator=g).to(gpu_device, dt)
    Wt = (torch.randn(N, K, generator=g) / 16).to(gpu_device, dt)
    Wp = _padded_weight(Wt, 256, dt)
    C = torch.zeros(M, N, device=gpu_device)
    _gemm(dtype, 1, A, Wp, M, N, K, K, 256, C, N, P=P, ldp=K, prow=prow, out_f32=1)
    Aplus = (A.float() + P.float().repeat(M // prow, 1)).to(dt).float()   # the add is rounded to T
    _close(C, Aplus @ Wt.float().t(), tol)


@pytest.mark.parametrize("dtype", ["bf16", "fp32"])
@pytest.mark.parametrize("B,H,W,Cin,Cout,k,s,p", [(2, 13, 11, 16, 72, 3, 2, 1), (1, 20, 20, 8, 64, 7, 2, 3),
                                                  (3, 9, 9, 64, 130, 1, 2, 0), (2, 10, 10, 32, 40, 3, 1, 1),
                                                  (2, 12, 12, 128, 96, 3, 1, 1), (1, 9, 9, 192, 64, 3, 2, 1)])
def test_gemm_conv_nhwc(gpu_device, dtype, B, H, W, Cin, Cout, k, s, p):
    _, dt, tol = DT[dtype]
    g = torch.Generator(device="cpu").manual_seed(B * H + Cout)
    x = torch.randn(B, Cin, H, W, generator=g).to(gpu_device, dt)
    w = (torch.randn(Cout, Cin, k, k, generator=g) / (Cin * k * k) ** 0.5).to(gpu_device, dt)
    bias = torch.randn(Cout, generator=g).to(gpu_device)
    ref = F.conv2d(x.float(), w.float(), bias, stride=s, padding=p)
    Ho, Wo = ref.shape[2], ref.shape[3]
    K = k * k * Cin
    ldb = (K + 63) // 64 * 64
    Wp = _padded_weight(_pack_conv(w), ldb, dt)
    xn = x.permute(0, 2, 3, 1).contiguous()
    ldc = (Cout + 7) // 8 * 8
    C = torch.zeros(B * Ho * Wo, ldc, dtype=dt, device=gpu_device)
    _gemm(dtype, 2, xn, Wp, B * Ho * Wo, Cout, K, 0, ldb, C, ldc, bias=bias, conv=(H, W, Cin, k, k, s, p))
    _close(C[:, :Cout], ref.permute(0, 2, 3, 1).reshape(-1, Cout), tol)


@pytest.mark.parametrize("dtype", ["bf16", "fp32"])
@pytest.mark.parametrize("T", [16, 11])
def test_gemm_head_transposed_store(gpu_device, dtype, T):
    _, dt, tol = DT[dtype]
    B, K, N = 3, 256, 512                              # two groups of 256 (like the cross-attn V of 2 layers)
    M = B * T
    g = torch.Generator(device="cpu").manual_seed(T)
    A = torch.randn(M, K, generator=g).to(gpu_device, dt)
    Wt = (torch.randn(N, K, generator=g) / 16).to(gpu_device, dt)
    bias = torch.randn(N, generator=g).to(gpu_device)
    C = torch.zeros(2 * B * 256 * T, dtype=dt, device=gpu_device)
    _gemm(dtype, 0, A, _padded_weight(Wt, 256, dt), M, N, K, K, 256, C, 8, bias=bias, vt=(T, B))
    ref = (A.float() @ Wt.float().t() + bias).view(B, T, 2, 256).permute(2, 0, 3, 1).reshape(-1)
    _close(C, ref, tol)


# ---- large-tile (256-row, direct-to-LDS) kernel: bf16 problems with >= 256 tiles

@pytest.mark.parametrize("N,K", [(256, 256), (64, 192), (128, 520), (512, 256), (200, 64),
                                 (256, 1088), (300, 1000)])   # K >= 1024: the 4-phase half-tile loop
def test_gemm_large_tile_linear(gpu_device, N, K):
    _, dt, tol = DT["bf16"]
    M = 256 * 256 + 77                                  # >= 256 tiles of 256 rows, ragged tail
    if N > 256:
        M = 256 * 130 + 5
    g = torch.Generator(device="cpu").manual_seed(N + K)
    A = torch.randn(M, K + 8, generator=g).to(gpu_device, dt)        # lda > K
    Wt = (torch.randn(N, K, generator=g) / K ** 0.5).to(gpu_device, dt)
    ldb = (K + 63) // 64 * 64
    bias = torch.randn(N, generator=g).to(gpu_device)
    ld = (N + 8 + 7) // 8 * 8
    R = torch.randn(M, ld, generator=g).to(gpu_device, dt)
    C = torch.zeros(M, ld, dtype=dt, device=gpu_device)
    _gemm("bf16", 0, A, _padded_weight(Wt, ldb, dt), M, N, K, K + 8, ldb, C, ld, bias=bias, R=R, ldr=ld, relu=1)
    ref = A[:, :K].float() @ Wt.float().t() + bias + R[:, :N].float()
    _close(C[:, :N], torch.relu(ref), tol)
    assert (C[:, N:] == 0).all()


@pytest.mark.parametrize("inplace", [True, False])
@pytest.mark.parametrize("M", [256 * 256 + 77, 1000, 16])
def test_gemm_fused_layernorm(gpu_device, inplace, M):
    """out-proj + residual + LayerNorm in one launch (encoder norm1, lnproj.hip), optionally in
    place over R; rows off the 16-row tile and fewer tiles than waves."""
    _, dt, tol = DT["bf16"]
    N, K = 256, 256
    g = torch.Generator(device="cpu").manual_seed(11)
    A = torch.randn(M, K, generator=g).to(gpu_device, dt)
    Wt = (torch.randn(N, K, generator=g) / 16).to(gpu_device, dt)
    bias = torch.randn(N, generator=g).to(gpu_device)
    R = (torch.randn(M, N, generator=g) * 2).to(gpu_device, dt)
    gam = (torch.randn(N, generator=g) * 0.5 + 1).to(gpu_device)
    bet = torch.randn(N, generator=g).to(gpu_device)
    pre = A.float() @ Wt.float().t() + bias + R.float()
    ref = F.layer_norm(pre, (N,), gam, bet, 1e-5)
    C = R if inplace else torch.zeros(M, N, dtype=dt, device=gpu_device)
    _gemm("bf16", 0, A, _padded_weight(Wt, 256, dt), M, N, K, K, 256, C, N, bias=bias, R=R, ldr=N, ln=(gam, bet))
    assert _lib.lib().spe_debug_gemm_path() == 4, "expected the LayerNorm projection kernel"
    _close(C, ref, 3e-2)
    # not fusable (too few rows for the large-tile kernel): the hook must refuse, not ignore
    L = _lib.lib()
    small = torch.zeros(100, N, dtype=dt, device=gpu_device)
    rc = L.spe_debug_gemm(None, 0, 0, _p(A), K, None, 0, 1, 0, 0, 0, 1, 1, 1, 0, _p(_padded_weight(Wt, 256, dt)), 256,
                          100, N, K, _p(bias), None, N, 0, _p(small), N, 0, 0, 0, 0, _p(gam), _p(bet), 0)
    assert rc != 0


@pytest.mark.parametrize("M", [256 * 256 + 77, 300, 24 * 2704])
def test_gemm_row_periodic_residual(gpu_device, M):
    """C = A W^T + b + R[m % period]: the (x + pos) W^T = x W^T + pos W^T rewrite of the
    attention q/k projections (both kernels: M = 300 stays on the 128x128 one; M = 24 images x
    2704 tokens, the model's shape, with SPE_SG_RMAP=1 takes the image-interleaved tile order)."""
    _, dt, tol = DT["bf16"]
    N, K, period = 512, 256, 2704 if M > 1000 else 11
    g = torch.Generator(device="cpu").manual_seed(M)
    A = torch.randn(M, K, generator=g).to(gpu_device, dt)
    Wt = (torch.randn(N, K, generator=g) / 16).to(gpu_device, dt)
    bias = torch.randn(N, generator=g).to(gpu_device)
    Rp = torch.randn(period, N, generator=g).to(gpu_device, dt)
    C = torch.zeros(M, N, dtype=dt, device=gpu_device)
    _gemm("bf16", 0, A, _padded_weight(Wt, 256, dt), M, N, K, K, 256, C, N, bias=bias, R=Rp, ldr=N, r_period=period)
    ref = A.float() @ Wt.float().t() + bias + Rp.float()[torch.arange(M, device=gpu_device) % period]
    _close(C, ref, tol)


# (residual-free convs with Cin % 64 == 0 or 1x1 take the pinned-schedule kernel (gemm2 PIN),
#  the others the compiler-scheduled loop; Cout 320 leaves a partial 64-wide column tile)
@pytest.mark.parametrize("Cin,Cout,k,s,p", [(64, 64, 3, 1, 1), (64, 128, 1, 1, 0), (32, 256, 3, 2, 1), (8, 64, 7, 2, 3),
                                            (128, 256, 3, 2, 1), (256, 256, 3, 1, 1), (128, 320, 3, 1, 1),
                                            (64, 128, 1, 2, 0)])
def test_gemm_large_tile_conv(gpu_device, Cin, Cout, k, s, p):
    _, dt, tol = DT["bf16"]
    B = 2 if Cin == 256 else 4                          # 133 row tiles: the 128..255-tile grids
    H = 130 if s == 1 else 258
    g = torch.Generator(device="cpu").manual_seed(Cin * k + Cout)
    x = torch.randn(B, Cin, H, H, generator=g).to(gpu_device, dt)
    w = (torch.randn(Cout, Cin, k, k, generator=g) / (Cin * k * k) ** 0.5).to(gpu_device, dt)
    bias = torch.randn(Cout, generator=g).to(gpu_device)
    ref = F.conv2d(x.float(), w.float(), bias, stride=s, padding=p)
    Ho = ref.shape[2]
    K = k * k * Cin
    ldb = (K + 63) // 64 * 64
    Wp = _padded_weight(_pack_conv(w), ldb, dt)
    C = torch.zeros(B * Ho * Ho, Cout, dtype=dt, device=gpu_device)
    _gemm("bf16", 2, x.permute(0, 2, 3, 1).contiguous(), Wp, B * Ho * Ho, Cout, K, 0, ldb, C, Cout, bias=bias,
          conv=(H, H, Cin, k, k, s, p))
    _close(C, ref.permute(0, 2, 3, 1).reshape(-1, Cout), tol)


# patch-staged 3x3 kernel (pconv.hip): stride 1 / pad 1, Cin % 64 == 0, Cout % 64 == 0 (64: one
# patch buffer, two workgroups per CU; 128-multiples / 256-multiples: double-buffered patches).
# Shapes: the bench's layer 1-3 convs and neck at small B, odd image sizes (partial blocks in both
# directions), several column tiles, and the one-buffer patch refetch across channel blocks.  (32, 26, 26,
# 256, 256): the north star's 32 images per GPU at layer 3, where 256 x 128 tiles fill the chip better.
@pytest.mark.parametrize("B,H,W,Cin,Cout,relu", [(3, 104, 104, 64, 64, 1), (2, 52, 52, 128, 128, 1),
                                                 (2, 26, 26, 256, 256, 1), (1, 52, 52, 1024, 256, 0),
                                                 (2, 13, 17, 128, 64, 1), (2, 9, 40, 64, 512, 0),
                                                 (5, 7, 7, 256, 128, 1), (1, 30, 61, 192, 384, 1),
                                                 (32, 26, 26, 256, 256, 1)])
def test_patch_conv3x3(gpu_device, B, H, W, Cin, Cout, relu):
    _, dt, tol = DT["bf16"]
    g = torch.Generator(device="cpu").manual_seed(B * H * W + Cin + Cout)
    x = torch.randn(B, Cin, H, W, generator=g).to(gpu_device, dt)
    w = (torch.randn(Cout, Cin, 3, 3, generator=g) / (Cin * 9) ** 0.5).to(gpu_device, dt)
    bias = torch.randn(Cout, generator=g).to(gpu_device)
    ref = F.conv2d(x.float(), w.float(), bias, stride=1, padding=1)
    if relu:
        ref = torch.relu(ref)
    K = 9 * Cin
    Wp = _padded_weight(_pack_conv(w), K, dt)
    C = torch.full((B * H * W, Cout), float("nan"), dtype=dt, device=gpu_device)
    _gemm("bf16", 2, x.permute(0, 2, 3, 1).contiguous(), Wp, B * H * W, Cout, K, 0, K, C, Cout, bias=bias, relu=relu,
          conv=(H, W, Cin, 3, 3, 1, 1))
    assert _lib.lib().spe_debug_gemm_path() == 3, "expected the patch-staged conv kernel"
    _close(C, ref.permute(0, 2, 3, 1).reshape(-1, Cout), tol)


# fused bottleneck tail (btail.hip): the layer-1 conv3 (+ identity) + relu with the next block's
# conv1 + relu, against torch fp32 of the two convs with y rounded to bf16 in between (the
# separate launches' intermediate); row counts off the 16-row tile and off the wave grid.
@pytest.mark.parametrize("M,k1,n2,res", [(173056, 64, 64, True), (1000, 64, 64, True), (40000, 64, 128, True),
                                         (16, 128, 64, False), (69217, 128, 64, False)])
def test_btail(gpu_device, M, k1, n2, res):
    L = _lib.lib()
    dt = torch.bfloat16
    g = torch.Generator(device="cpu").manual_seed(M + k1 + n2)
    A = torch.randn(M, k1, generator=g).to(gpu_device, dt)
    R = torch.randn(M, 256, generator=g).to(gpu_device, dt) if res else None
    W3 = (torch.randn(256, k1, generator=g) / k1 ** 0.5).to(gpu_device, dt)
    b3 = (0.1 * torch.randn(256, generator=g)).to(gpu_device)
    W1 = (torch.randn(n2, 256, generator=g) / 16).to(gpu_device, dt)
    b1 = (0.1 * torch.randn(n2, generator=g)).to(gpu_device)
    perm = torch.tensor([L.spe_debug_btail_perm(k) for k in range(256)], device=gpu_device)
    assert sorted(perm.tolist()) == list(range(256))
    W1p = W1[:, perm].contiguous()
    Y = torch.full((M, 256), float("nan"), dtype=dt, device=gpu_device)
    Z = torch.full((M, n2), float("nan"), dtype=dt, device=gpu_device)
    rc = L.spe_debug_btail(None, _p(A), k1, k1, _p(R), _p(_padded_weight(W3, 64 * ((k1 + 63) // 64), dt)),
                           64 * ((k1 + 63) // 64), _p(b3), _p(Y), _p(W1p), 256, _p(b1), _p(Z), n2, M)
    assert rc == 0, L.spe_last_error()
    torch.cuda.synchronize()
    yref = A.float() @ W3.float().t() + b3 + (R.float() if res else 0)
    yref = torch.relu(yref)
    _close(Y, yref, DT["bf16"][2])
    zref = torch.relu(Y.float() @ W1.float().t() + b1)
    _close(Z, zref, DT["bf16"][2])


# the fused stem + bias + ReLU + max-pool (stempool.hip): the bench's 416^2 (one column group,
# 15 waves), a small image, 640^2 (config 5: two column groups, an idle wave) and a strided
# output row (the pool writes the right half of layer 1 block 0's [conv2 | pool] concatenation)
@pytest.mark.parametrize("B,S,ldo", [(2, 416, 64), (3, 64, 64), (1, 640, 64), (2, 416, 128)])
def test_stempool(gpu_device, B, S, ldo):
    L = _lib.lib()
    dt = torch.bfloat16
    g = torch.Generator(device="cpu").manual_seed(B * S + ldo)
    img = torch.randn(B, 3, S, S, generator=g)
    X = torch.zeros(B, S + 6, S + 6, 4)
    X[:, 3:S + 3, 3:S + 3, :3] = img.permute(0, 2, 3, 1)
    X = X.to(gpu_device, dt)
    W7 = torch.randn(64, 3, 7, 7, generator=g) / 8
    Wp = torch.zeros(64, 7, 8, 4)
    Wp[:, :, :7, :3] = W7.permute(0, 2, 3, 1)
    Wp = torch.cat([Wp.reshape(64, 224), torch.zeros(64, 32)], 1).to(gpu_device, dt)
    bias = (0.2 * torch.randn(64, generator=g)).to(gpu_device)
    Po = S // 4
    out = torch.full((B, Po, Po, ldo), float("nan"), dtype=dt, device=gpu_device)
    rc = L.spe_debug_stempool(None, _p(X), _p(Wp), 256, _p(bias), _p(out), ldo, B, S)
    assert rc == 0, L.spe_last_error()
    torch.cuda.synchronize()
    xr = X[:, 3:S + 3, 3:S + 3, :3].float().permute(0, 3, 1, 2)
    wr = Wp[:, :224].float().view(64, 7, 8, 4)[:, :, :7, :3].permute(0, 3, 1, 2)
    ref = F.max_pool2d(torch.relu(F.conv2d(xr, wr, bias, stride=2, padding=3)), 3, 2, 1).permute(0, 2, 3, 1)
    _close(out[..., :64], ref, DT["bf16"][2])
    if ldo > 64:
        assert torch.isnan(out[..., 64:].float()).all()       # nothing written past the 64 channels


def test_gemm_large_tile_head_transposed(gpu_device):
    _, dt, tol = DT["bf16"]
    B, T, K, N = 25, 2704, 256, 512
    M = B * T
    g = torch.Generator(device="cpu").manual_seed(5)
    A = torch.randn(M, K, generator=g).to(gpu_device, dt)
    Wt = (torch.randn(N, K, generator=g) / 16).to(gpu_device, dt)
    bias = torch.randn(N, generator=g).to(gpu_device)
    C = torch.zeros(2 * B * 256 * T, dtype=dt, device=gpu_device)
    _gemm("bf16", 0, A, _padded_weight(Wt, 256, dt), M, N, K, K, 256, C, 8, bias=bias, vt=(T, B))
    ref = (A.float() @ Wt.float().t() + bias).view(B, T, 2, 256).permute(2, 0, 3, 1).reshape(-1)
    _close(C, ref, tol)


@pytest.mark.parametrize("M,N,vt", [(256 * 256 + 40, 512, False), (300, 512, False), (5000, 256, False),
                                     (64 * 676, 256, True), (2 * 256, 256, True), (20 * 256, 256, True)])
def test_gemm_fp16_output(gpu_device, M, N, vt):
    """out_f16: bf16 GEMMs (large-tile, few-row and 128x128 kernels) storing fp16, row-major or
    head-transposed V^T -- the operands of the fp16 encoder attention (BASELINE config 5)."""
    g = torch.Generator(device="cpu").manual_seed(M + N)
    K = 256
    A = torch.randn(M, K, generator=g).to(gpu_device, torch.bfloat16)
    Wt = (torch.randn(N, K, generator=g) / 16).to(gpu_device, torch.bfloat16)
    bias = torch.randn(N, generator=g).to(gpu_device)
    ref = A.float() @ Wt.float().t() + bias
    if vt:
        T = 676 if M % 676 == 0 else 256
        B = M // T
        C = torch.zeros(B * N * T, dtype=torch.float16, device=gpu_device)
        _gemm("bf16", 0, A, _padded_weight(Wt, 256, torch.bfloat16), M, N, K, K, 256, C, 8, bias=bias, vt=(T, B),
              out_f16=1)
        ref = ref.view(B, T, N // 256, 256).permute(2, 0, 3, 1).reshape(-1)
    else:
        C = torch.zeros(M, N, dtype=torch.float16, device=gpu_device)
        _gemm("bf16", 0, A, _padded_weight(Wt, 256, torch.bfloat16), M, N, K, K, 256, C, N, bias=bias, out_f16=1)
    assert torch.isfinite(C.float()).all()
    _close(C, ref, 2e-3)


@pytest.mark.parametrize("M,N,K,mode", [(256 * 600 + 5, 256, 64, "res"), (256 * 1100 + 100, 128, 256, "relu"),
                                         (300 * 512, 512, 256, "periodic"), (64 * 2704, 256, 256, "vt")])
def test_gemm_one_stage_large(gpu_device, M, N, K, mode):
    """Sizes that take the one-stage, two-workgroups-per-CU kernel (short K, >= 512 tiles of
    256x128): residual, ReLU, row-periodic residual (the q/k projection's pos.W^T) and the
    head-transposed V^T store, against an fp32 torch reference."""
    g = torch.Generator(device="cpu").manual_seed(M + K)
    dt = torch.bfloat16
    A = torch.randn(M, K, generator=g).to(gpu_device, dt)
    Wt = (torch.randn(N, K, generator=g) / K ** 0.5).to(gpu_device, dt)
    bias = torch.randn(N, generator=g).to(gpu_device)
    ref = A.float() @ Wt.float().t() + bias
    W = _padded_weight(Wt, (K + 63) // 64 * 64, dt)
    ldb = W.shape[1]
    if mode == "vt":
        T = 2704
        B = M // T
        C = torch.zeros(B * N * T, dtype=dt, device=gpu_device)
        _gemm("bf16", 0, A, W, M, N, K, K, ldb, C, 8, bias=bias, vt=(T, B))
        ref = ref.view(B, T, N // 256, 256).permute(2, 0, 3, 1).reshape(-1)
    else:
        C = torch.zeros(M, N, dtype=dt, device=gpu_device)
        if mode == "res":
            R = torch.randn(M, N, generator=g).to(gpu_device, dt)
            _gemm("bf16", 0, A, W, M, N, K, K, ldb, C, N, bias=bias, R=R, ldr=N, relu=1)
            ref = torch.relu(ref + R.float())
        elif mode == "relu":
            _gemm("bf16", 0, A, W, M, N, K, K, ldb, C, N, bias=bias, relu=1)
            ref = torch.relu(ref)
        else:
            P = 512
            R = torch.randn(P, N, generator=g).to(gpu_device, dt)
            _gemm("bf16", 0, A, W, M, N, K, K, ldb, C, N, bias=bias, R=R, ldr=N, r_period=P)
            ref = ref + R.float().repeat(M // P, 1)
    _close(C, ref, 2e-2)


def _attn_ref(q, k, v, scale):
    a = torch.softmax((q.float() @ k.float().transpose(-1, -2)) * scale, -1)
    return a @ v.float()


# attention-only operand mode of bf16 models' encoder: bf16 q/k, fp16 V^T and P (attention.hip TV)
SPE_DTYPE_BF16_F16V = 3


@pytest.mark.parametrize("dtype", ["bf16", "fp16", "fp32", "bf16_f16v"])
@pytest.mark.parametrize("B,H,Tq,Tk", [(2, 8, 200, 200), (3, 8, 11, 330), (1, 8, 11, 11), (1, 2, 300, 64),
                                       (1, 8, 2704, 2704)])
def test_attention(gpu_device, dtype, B, H, Tq, Tk):
    if dtype == "bf16_f16v":
        code, dt, vdt = SPE_DTYPE_BF16_F16V, torch.bfloat16, torch.float16
    else:
        code, dt, _ = DT[dtype]
        vdt = dt
    g = torch.Generator(device="cpu").manual_seed(Tq + Tk)
    ld = H * 32 + 16                                   # row stride wider than the heads
    Q = (torch.randn(B * Tq, ld, generator=g) * 2).to(gpu_device, dt)
    K = (torch.randn(B * Tk, ld, generator=g) * 2).to(gpu_device, dt)
    V = torch.randn(B, H, Tk, 32, generator=g).to(gpu_device, vdt)
    VT = V.transpose(-1, -2).contiguous()
    # 16-bit operand kernels (bf16 / fp16) write bf16: the out-projection GEMM reads bf16
    O = torch.zeros(B * Tq, H * 32, dtype=torch.float32 if dtype == "fp32" else torch.bfloat16, device=gpu_device)
    scale = 32 ** -0.5
    rc = _lib.lib().spe_debug_attention(None, code, _p(Q), ld, _p(K), ld, _p(VT), _p(O), H * 32, B, H, Tq, Tk, scale)
    assert rc == 0
    torch.cuda.synchronize()
    q = Q[:, : H * 32].view(B, Tq, H, 32).transpose(1, 2)
    k = K[:, : H * 32].view(B, Tk, H, 32).transpose(1, 2)
    if dtype != "fp32":                                # the kernel rounds the prescaled q to 16 bits
        q = (q.float() * scale * 1.4426950408889634).to(dt).float() / (scale * 1.4426950408889634)
    ref = _attn_ref(q, k, V, scale).transpose(1, 2).reshape(B * Tq, H * 32)
    _close(O, ref, {"bf16": 2e-2, "fp16": 1e-2, "fp32": 1e-5, "bf16_f16v": 2e-2}[dtype])


def _vt_swizzle(VT):
    """[..., Tk] rows in the encoder's LDS-DMA key order: token t stored at position t with
    bits 2 and 3 swapped (spe_kernels.h vt_pos)."""
    Tk = VT.shape[-1]
    t = torch.arange(Tk)
    pos = (t & ~12) | ((t & 4) << 1) | ((t & 8) >> 1)
    out = torch.empty_like(VT)
    out[..., pos.to(VT.device)] = VT
    return out


# the encoder's LDS-DMA staging (swizzled V^T, Tk % 16 == 0): keys past a whole tile, one-tile
# and two-tile sweeps, Tq below the 128-query block, and the bench's T = 2704
@pytest.mark.parametrize("dtype", ["bf16", "fp16", "bf16_f16v"])
@pytest.mark.parametrize("B,H,Tq,Tk", [(2, 8, 200, 208), (1, 8, 64, 64), (1, 2, 300, 128), (3, 8, 256, 96),
                                       (1, 8, 2704, 2704)])
def test_attention_dma(gpu_device, dtype, B, H, Tq, Tk):
    if dtype == "bf16_f16v":
        code, dt, vdt = SPE_DTYPE_BF16_F16V, torch.bfloat16, torch.float16
    else:
        code, dt, _ = DT[dtype]
        vdt = dt
    g = torch.Generator(device="cpu").manual_seed(Tq + Tk + 7)
    ld = H * 32 + 16
    Q = (torch.randn(B * Tq, ld, generator=g) * 2).to(gpu_device, dt)
    K = (torch.randn(B * Tk, ld, generator=g) * 2).to(gpu_device, dt)
    V = torch.randn(B, H, Tk, 32, generator=g).to(gpu_device, vdt)
    VTs = _vt_swizzle(V.transpose(-1, -2).contiguous())
    O = torch.zeros(B * Tq, H * 32, dtype=torch.bfloat16, device=gpu_device)
    scale = 32 ** -0.5
    rc = _lib.lib().spe_debug_attention(None, code | 0x100, _p(Q), ld, _p(K), ld, _p(VTs), _p(O), H * 32, B, H, Tq,
                                        Tk, scale)
    assert rc == 0, _lib.lib().spe_last_error()
    torch.cuda.synchronize()
    q = Q[:, : H * 32].view(B, Tq, H, 32).transpose(1, 2)
    k = K[:, : H * 32].view(B, Tk, H, 32).transpose(1, 2)
    q = (q.float() * scale * 1.4426950408889634).to(dt).float() / (scale * 1.4426950408889634)
    ref = _attn_ref(q, k, V, scale).transpose(1, 2).reshape(B * Tq, H * 32)
    _close(O, ref, {"bf16": 2e-2, "fp16": 1e-2, "bf16_f16v": 2e-2}[dtype])


def test_gemm_vt_swizzle(gpu_device):
    """Head-transposed GEMM stores in the swizzled key order (act_code bit 9) on the streaming,
    large-tile and small kernels: the swizzled output un-permutes to the plain one."""
    dt = torch.bfloat16
    for B, T in ((64, 2704), (3, 256), (1, 64)):
        M, K, N = B * T, 256, 256
        g = torch.Generator(device="cpu").manual_seed(B + T)
        A = torch.randn(M, K, generator=g).to(gpu_device, dt)
        W = (torch.randn(N, K, generator=g) / 16).to(gpu_device, dt)
        bias = torch.randn(N, generator=g).to(gpu_device)
        plain = torch.zeros(B * N * T, dtype=dt, device=gpu_device)
        swz = torch.zeros_like(plain)
        _gemm("bf16", 0, A, W, M, N, K, K, K, plain, 8, bias=bias, vt=(T, B))
        _gemm("bf16", 0, A, W, M, N, K, K, K, swz, 8, bias=bias, vt=(T, B), relu=1 << 9)
        assert torch.equal(_vt_swizzle(plain.view(B, N, T)), swz.view(B, N, T)), (B, T)


@pytest.mark.parametrize("mode,gain", [("bf16", 12.0), ("bf16_f16v", 12.0), ("bf16_f16v_dma", 12.0),
                                       ("bf16_f16v_dma", 3.0), ("bf16_f16v_dma", 40.0)])
def test_attention_large_score_range(gpu_device, mode, gain):
    """Scores spanning > 100 in log space force rescales of the running max late in the sweep.
    DMA kernel: its tiles skip the max unless the fp16 row sum overflows the lazy limit, so a
    late jump (gain 12), a mild one (3, rescales within the slack) and one past f32 exp2's range
    (40: p = inf against the stale max) must all come out through the recompute path."""
    code, dt, _ = DT["bf16"]
    vdt = dt
    if mode.startswith("bf16_f16v"):
        code, vdt = SPE_DTYPE_BF16_F16V, torch.float16
    B, H, T = 1, 8, 256
    g = torch.Generator(device="cpu").manual_seed(0)
    Q = torch.randn(B * T, 256, generator=g).to(gpu_device, dt)
    K = torch.randn(B * T, 256, generator=g)
    K[200:] *= gain                                    # late keys dominate
    K = K.to(gpu_device, dt)
    V = torch.randn(B, H, T, 32, generator=g).to(gpu_device, vdt)
    O = torch.zeros(B * T, 256, dtype=dt, device=gpu_device)
    scale = 32 ** -0.5
    VT = V.transpose(-1, -2).contiguous()
    if mode.endswith("_dma"):
        code, VT = code | 0x100, _vt_swizzle(VT)
    assert _lib.lib().spe_debug_attention(None, code, _p(Q), 256, _p(K), 256, _p(VT), _p(O), 256, B, H, T, T,
                                          scale) == 0
    torch.cuda.synchronize()
    q = Q.view(B, T, H, 32).transpose(1, 2)
    q = (q.float() * scale * 1.4426950408889634).to(dt).float() / (scale * 1.4426950408889634)
    ref = _attn_ref(q, K.view(B, T, H, 32).transpose(1, 2), V, scale).transpose(1, 2).reshape(B * T, 256)
    _close(O, ref, 2e-2)


@pytest.mark.parametrize("chunked", [0, 1])
@pytest.mark.parametrize("M,F,inplace,splits", [(333, 2048, True, 0), (128, 64, False, 0), (1000, 2048, False, 0),
                                                (5, 32, True, 0), (704, 2048, True, 16), (300, 2048, False, 32),
                                                (77, 128, False, 2), (17003, 2048, False, 0), (640, 1024, True, 0),
                                                # whole 192-row rounds + a 128-row tail launch on 256 CUs
                                                (54152, 2048, True, 0), (70000, 2048, False, 0)])
def test_fused_ffn(gpu_device, M, F, inplace, splits, chunked):
    """bf16 fused linear1 -> ReLU -> linear2 -> +x -> LayerNorm against torch fp32 on bf16-rounded
    operands; the hidden activation is rounded to bf16 on chip exactly as the unfused path stores it.
    chunked: W2 passed chunk-packed [F/32][256][32] (ld2 = 0), the bf16 model's encoder form."""
    dt, D = torch.bfloat16, 256
    g = torch.Generator(device="cpu").manual_seed(M + F)
    ld = D + 8 if not inplace else D
    x = (torch.randn(M, ld, generator=g) * 2).to(gpu_device, dt)
    w1 = (torch.randn(F, D, generator=g) / D ** 0.5).to(gpu_device, dt)
    b1 = (torch.randn(F, generator=g) * 0.1).to(gpu_device)
    w2 = (torch.randn(D, F, generator=g) / F ** 0.5).to(gpu_device, dt)
    b2 = (torch.randn(D, generator=g) * 0.1).to(gpu_device)
    gam = (torch.randn(D, generator=g) * 0.5 + 1).to(gpu_device)
    bet = (torch.randn(D, generator=g) * 0.1).to(gpu_device)
    xs = x[:, :D].float()
    h = torch.relu(xs @ w1.float().t() + b1).to(dt).float()
    ref = F_.layer_norm(xs + h @ w2.float().t() + b2, (D,), gam, bet, 1e-5)
    y = x if inplace else torch.full((M, ld), 7.0, dtype=dt, device=gpu_device)
    part = torch.empty(max(splits, 1), M, D, device=gpu_device) if splits else None
    w2a, ld2 = (w2.view(D, F // 32, 32).permute(1, 0, 2).contiguous(), 0) if chunked else (w2, F)
    rc = _lib.lib().spe_debug_ffn(None, _p(x), ld, _p(w1), D, _p(b1), _p(w2a), ld2, _p(b2), _p(gam), _p(bet), _p(y),
                                  ld, M, D, F, _p(part), splits)
    assert rc == 0, _lib.lib().spe_last_error()
    torch.cuda.synchronize()
    _close(y[:, :D], ref, 3e-2)
    if not inplace:
        assert (y[:, D:] == 7.0).all()                 # nothing written past D


@pytest.mark.parametrize("B,Q,T,splits,amp", [(3, 11, 200, 1, 1.0), (2, 11, 203, 3, 1.0), (1, 17, 136, 2, 1.0),
                                              (2, 11, 2704, 0, 1.0), (2, 5, 640, 4, 12.0), (64, 11, 2704, 0, 1.0)])
def test_cross_attention_memory(gpu_device, B, Q, T, splits, amp):
    """decoder cross-attention against the memory (xattn.hip): u = softmax_2(q' . K^T) . V per
    (image, query, head) row, against torch fp32 on the same bf16 operands.  amp = 12 spreads the
    scores over ~100 log2 units (many lazy-rescale branches taken, split partials merged far apart).
    K rows are the model's memory + pos (the reference's key, REV/models/transformer.py:230-233).
    Tolerance: P is rounded to bf16 (2^-9 relative) before the value product; 1e-2 * scale."""
    dt, D = torch.bfloat16, 256
    g = torch.Generator(device="cpu").manual_seed(B * T + Q)
    ldq, ldv = 8 * D + 8, D + 8
    q = (torch.randn(B * Q, ldq, generator=g) * amp / 16).to(gpu_device, dt)
    k = torch.randn(B * T, D, generator=g).to(gpu_device, dt)
    v = torch.randn(B * T, ldv, generator=g).to(gpu_device, dt)          # strided rows
    if amp > 1:
        k[5] *= 4                                           # one key far above the rest
    wv = (torch.randn(D, D, generator=g) / 16).to(gpu_device, dt)
    bv = torch.randn(D, generator=g).to(gpu_device)
    u = torch.full((B * Q, ldq), 7.0, dtype=dt, device=gpu_device)
    o = torch.full((B * Q, D + 8), 7.0, dtype=dt, device=gpu_device)
    S = splits if splits > 0 else 256                     # the launch's own split count is below 256
    part = torch.empty(S * B * 8 * Q * 258, device=gpu_device)
    L = _lib.lib()
    rc = L.spe_debug_xattn(None, _p(q), ldq, _p(k), D, _p(v), ldv, _p(u), ldq, None, None, None, 0, B, Q, T,
                           splits, _p(part))
    assert rc == 0, L.spe_last_error()
    rc = L.spe_debug_xattn(None, _p(q), ldq, _p(k), D, _p(v), ldv, None, 0, _p(wv), _p(bv), _p(o), D + 8, B, Q,
                           T, splits, _p(part))
    assert rc == 0, L.spe_last_error()
    torch.cuda.synchronize()
    qh = q[:, :8 * D].float().view(B, Q * 8, D)
    kk = k.float().view(B, T, D)
    s = torch.einsum("brd,btd->brt", qh, kk)
    p = torch.softmax(s * 0.6931471805599453, dim=-1)
    ref = torch.einsum("brt,btd->brd", p, v[:, :D].float().view(B, T, D))   # [B][Q*8][D], rows q*8 + h
    _close(u[:, :8 * D], ref.reshape(B * Q, 8 * D), 1e-2)
    assert (u[:, 8 * D:] == 7.0).all()
    # o_h = Wv_h u_h + bv_h: the value projection after the weighted sum (u itself unrounded)
    ref_o = torch.einsum("bqhn,hjn->bqhj", ref.view(B, Q, 8, D), wv.float().view(8, 32, D)) + bv.view(8, 32)
    _close(o[:, :D], ref_o.reshape(B * Q, D), 1e-2)
    assert (o[:, D:] == 7.0).all()


@pytest.mark.parametrize("B,Q,T,splits,amp", [(3, 11, 200, 1, 1.0), (2, 12, 203, 3, 1.0), (1, 17, 136, 2, 1.0),
                                              (2, 11, 2704, 0, 1.0), (2, 5, 640, 4, 12.0), (64, 11, 2704, 0, 4.0)])
def test_cross_attention_memory_h3(gpu_device, B, Q, T, splits, amp):
    """fp32h3 decoder cross-attention against the memory (xattn_h3.hip): the memory split into fp16 hi / lo
    planes of (mem + pos) * 2^sk and mem * 2^sv, three fp16 products per score and value term, the
    key-split merge and o_h = Wv_h u_h + bv_h in fp32 (REV/models/transformer.py:230-233 folded), against
    fp64 on the same fp32 operands.  Q = 12 fills the 96-row group; Q = 17 takes two groups; T = 203 ends
    in a partial 32-key tile; amp spreads the scores over ~30 log2 units (one key 4x above the rest) so
    the lazy rescale and far-apart split partials are exercised.  The memory's bound is a loose LayerNorm-
    style bound (4x max |mem|: the model's ln_bound), pos in [-1, 1].  Tolerance 2e-5 * scale: the
    products' 2^-22 splits and fp32 accumulation, against the bf16 kernel's 1e-2."""
    D = 256
    g = torch.Generator(device="cpu").manual_seed(7 * B * T + Q)
    ldq, ldo = 8 * D + 4, D + 4
    q = torch.randn(B * Q, ldq, generator=g, dtype=torch.float64) * amp / 16
    mem = torch.randn(B * T, D, generator=g, dtype=torch.float64)
    pos = torch.rand(T, D, generator=g, dtype=torch.float64) * 2 - 1
    if amp > 1:
        mem[5] *= 4
    wv = torch.randn(D, D, generator=g, dtype=torch.float64) / 16
    bv = torch.randn(D, generator=g, dtype=torch.float64)
    q32, mem32, pos32 = q.float(), mem.float(), pos.float()
    wv32, bv32 = wv.float(), bv.float()
    amax = torch.tensor([4.0 * float(mem32.abs().max())], device=gpu_device)
    dq, dm, dp = q32.to(gpu_device), mem32.to(gpu_device), pos32.to(gpu_device)
    dwv, dbv = wv32.to(gpu_device), bv32.to(gpu_device)
    o = torch.full((B * Q, ldo), 7.0, device=gpu_device)
    oam = torch.zeros(1, device=gpu_device)
    S = splits if splits > 0 else 256
    part = torch.empty(S * B * 8 * Q * 258, device=gpu_device)
    planes = torch.empty(B * T * 2048, dtype=torch.uint8, device=gpu_device)
    L = _lib.lib()
    rc = L.spe_debug_xattn_h3(None, _p(dq), ldq, _p(dm), _p(dp), _p(amax), _p(dwv), _p(dbv), _p(o), ldo, _p(oam),
                              B, Q, T, splits, _p(part), _p(planes))
    assert rc == 0, L.spe_last_error()
    torch.cuda.synchronize()
    # fp64 reference on the fp32 operands (keys = the fp32 sum mem + pos, as the reference forms them)
    k = (mem32 + pos32.repeat(B, 1)).double().view(B, T, D)
    s = torch.einsum("brd,btd->brt", q32[:, :8 * D].double().view(B, Q * 8, D), k)
    p = torch.softmax(s * math.log(2.0), dim=-1)
    u = torch.einsum("brt,btd->brd", p, mem32.double().view(B, T, D))
    ref = torch.einsum("bqhn,hjn->bqhj", u.view(B, Q, 8, D), wv32.double().view(8, 32, D)) + bv32.double().view(8, 32)
    ref = ref.reshape(B * Q, D)
    got = o[:, :D].double().cpu()
    err = float((got - ref).abs().max() / ref.abs().max())
    assert err <= 2e-5, err
    assert (o[:, D:] == 7.0).all()                      # nothing written past D
    assert abs(float(oam) - float(o[:, :D].abs().max())) == 0.0   # the published max |o|


@pytest.mark.parametrize("B,Q,T,splits,amp", [(3, 11, 200, 1, 1.0), (2, 11, 203, 3, 1.0), (1, 16, 136, 2, 1.0),
                                              (64, 11, 2704, 0, 1.0), (2, 5, 640, 4, 12.0), (1, 1, 2704, 0, 1.0),
                                              (16, 40, 6400, 0, 1.0), (2, 33, 300, 5, 12.0), (1, 48, 64, 1, 1.0),
                                              (3, 17, 200, 2, 1.0)])
def test_cross_attention_tail_fused(gpu_device, B, Q, T, splits, amp):
    """decxproj (decsa.hip): the key-split merge of xattn's partials, the value projection
    o_h = Wv_h u_h + bv_h (bf16) and tgt = LN(tgt + o . Wo^T + bo) in one launch per image, 16
    queries per pass (Q = 40 at 6400 keys: BASELINE config 5's shape)
    (REV/models/transformer.py:230-234), against torch fp32 on the same bf16 operands with the
    separate path's rounding of o.  The partials come from the xattn kernel itself; 2e-2 * scale."""
    dt, D = torch.bfloat16, 256
    g = torch.Generator(device="cpu").manual_seed(3 * B * T + Q)
    ldq, ldt = 8 * D + 8, D + 8
    q = (torch.randn(B * Q, ldq, generator=g) * amp / 16).to(gpu_device, dt)
    k = torch.randn(B * T, D, generator=g).to(gpu_device, dt)
    v = torch.randn(B * T, D, generator=g).to(gpu_device, dt)
    if amp > 1:
        k[5] *= 4
    wv = (torch.randn(D, D, generator=g) / 16).to(gpu_device, dt)
    bv = torch.randn(D, generator=g).to(gpu_device)
    wo = (torch.randn(D, D, generator=g) / 16).to(gpu_device, dt)
    bo = (torch.randn(D, generator=g) * 0.1).to(gpu_device)
    gam = (1 + 0.1 * torch.randn(D, generator=g)).to(gpu_device)
    bet = (0.1 * torch.randn(D, generator=g)).to(gpu_device)
    t0 = torch.randn(B * Q, ldt, generator=g)
    t = t0.to(dt).to(gpu_device)
    u = torch.empty(B * Q, ldq, dtype=dt, device=gpu_device)
    S = splits if splits > 0 else 256
    part = torch.empty(S * B * 8 * Q * 258, device=gpu_device)
    L = _lib.lib()
    rc = L.spe_debug_xattn(None, _p(q), ldq, _p(k), D, _p(v), D, _p(u), ldq, None, None, None, 0, B, Q, T,
                           splits, _p(part))
    assert rc == 0, L.spe_last_error()
    rc = L.spe_debug_decxproj(None, _p(t), ldt, _p(part), splits, T, B, Q, _p(wv), D, _p(bv), _p(wo), D, _p(bo),
                              _p(gam), _p(bet))
    assert rc == 0, L.spe_last_error()
    torch.cuda.synchronize()
    s = torch.einsum("brd,btd->brt", q[:, :8 * D].float().view(B, Q * 8, D), k.float().view(B, T, D))
    ref_u = torch.einsum("brt,btd->brd", torch.softmax(s * 0.6931471805599453, dim=-1), v.float().view(B, T, D))
    o = torch.einsum("bqhn,hjn->bqhj", ref_u.view(B, Q, 8, D), wv.float().view(8, 32, D)) + bv.view(8, 32)
    o = o.reshape(B * Q, D).to(dt).float()
    y = torch.nn.functional.layer_norm(o @ wo.float().T + bo + t0[:, :D].to(dt).float().to(gpu_device), (D,),
                                       gam, bet, 1e-5)
    _close(t[:, :D], y, 2e-2)
    assert torch.equal(t[:, D:].cpu(), t0[:, D:].to(dt))   # nothing written past D


@pytest.mark.parametrize("M,N,period,bias", [(704, 2048, 11, False), (37, 2048, 11, True), (2816, 512, 40, False),
                                              (5, 256, 0, True)])
def test_decoder_query_projection(gpu_device, M, N, period, bias):
    """decq (decsa.hip): y = x . W^T (+ b) + R[m % period], bf16, K = 256 -- the cross-attention's
    folded query projection (xattn.hip; R = query_pos . Wqk^T + bqk), one workgroup per (16 rows,
    256 columns), against torch fp32 on the same bf16 operands; 1e-2 * scale (bf16 output)."""
    dt, D = torch.bfloat16, 256
    g = torch.Generator(device="cpu").manual_seed(M + N + period)
    ldx, ldy = D + 8, N + 8
    x = torch.randn(M, ldx, generator=g).to(dt)
    w = (torch.randn(N, D, generator=g) / 16).to(dt)
    b = torch.randn(N, generator=g) if bias else None
    r = torch.randn(max(period, 1), N, generator=g).to(dt) if period else None
    y = torch.full((M, ldy), 7.0, dtype=dt, device=gpu_device)
    dev = lambda a: a.to(gpu_device).contiguous() if a is not None else None   # noqa: E731
    xd, wd, bd, rd = dev(x), dev(w), dev(b), dev(r)
    L = _lib.lib()
    rc = L.spe_debug_decq(None, _p(xd), ldx, M, N, _p(wd), D, _p(bd) if bias else None, _p(rd) if period else None,
                          N, period, _p(y), ldy)
    assert rc == 0, L.spe_last_error()
    torch.cuda.synchronize()
    ref = x[:, :D].float() @ w.float().T
    if bias:
        ref += b
    if period:
        ref += r.float()[torch.arange(M) % period]
    _close(y[:, :N].cpu(), ref, 1e-2)
    assert (y[:, N:] == 7.0).all()


@pytest.mark.parametrize("M,F", [(704, 2048), (33, 2048), (16, 256), (2816, 1024), (1, 512)])
def test_decoder_ffn_split_chunks(gpu_device, M, F):
    """decffn (decsa.hip) + ffn.hip's reduce: y = LN(x + W2 relu(W1 x + b1) + b2) in place for the
    decoder's few rows (REV/models/transformer.py:236-238), one workgroup per (16 rows, 256 hidden
    units), against torch fp32 on the same bf16 operands with the hidden rounded to bf16 as the
    kernel does; 2e-2 * scale (bf16 output).  M = 2816: the north star's 256 images per GPU."""
    dt, D = torch.bfloat16, 256
    g = torch.Generator(device="cpu").manual_seed(M + F)
    ldx = D + 8
    x0 = torch.randn(M, ldx, generator=g)
    w1 = (torch.randn(F, D, generator=g) / 16).to(dt)
    w2 = (torch.randn(D, F, generator=g) / 45).to(dt)
    b1, b2 = torch.randn(F, generator=g) * 0.1, torch.randn(D, generator=g) * 0.1
    gam, bet = 1 + 0.1 * torch.randn(D, generator=g), 0.1 * torch.randn(D, generator=g)
    dev = lambda a: a.to(gpu_device).contiguous()          # noqa: E731
    x = x0.to(dt).to(gpu_device)
    part = torch.empty(F // 256 * M * D, device=gpu_device)
    args = [dev(w1), dev(b1), dev(w2), dev(b2), dev(gam), dev(bet)]
    L = _lib.lib()
    rc = L.spe_debug_decffn(None, _p(x), ldx, M, F, _p(args[0]), D, _p(args[1]), _p(args[2]), F, _p(args[3]),
                            _p(args[4]), _p(args[5]), _p(x), ldx, _p(part))
    assert rc == 0, L.spe_last_error()
    torch.cuda.synchronize()
    xb = x0[:, :D].to(dt).float()
    h = torch.relu(xb @ w1.float().T + b1).to(dt).float()
    y = torch.nn.functional.layer_norm(xb + h @ w2.float().T + b2, (D,), gam, bet, 1e-5)
    _close(x[:, :D].cpu(), y, 2e-2)
    assert torch.equal(x[:, D:].cpu(), x0[:, D:].to(dt))   # nothing written past D


@pytest.mark.parametrize("B,Q", [(3, 11), (2, 40), (1, 64), (4, 1), (0, 11)])
def test_decoder_self_attention_block(gpu_device, B, Q):
    """decsa.hip: tgt = LN(tgt + MHA(q = k = tgt + query_pos, v = tgt) . Wo^T + bo) in place, one
    workgroup per image (REV/models/transformer.py:218-228, forward_post), against torch fp32 on
    the same bf16 operands with the separate path's roundings (q/k/v and the attention output
    stored as bf16).  Tolerance 2e-2 * scale (bf16 output, unit-variance rows after the norm)."""
    dt, D, H = torch.bfloat16, 256, 8
    g = torch.Generator(device="cpu").manual_seed(31 * B + Q)
    ldt = D + 8
    x = torch.randn(max(B, 1) * Q, ldt, generator=g)
    wqk = (torch.randn(2 * D, D, generator=g) / 16).to(dt)
    wv = (torch.randn(D, D, generator=g) / 16).to(dt)
    wo = (torch.randn(D, D, generator=g) / 16).to(dt)
    bqk, bv, bo = (torch.randn(n, generator=g) * 0.1 for n in (2 * D, D, D))
    qpos = (torch.randn(Q, 2 * D, generator=g) * 0.5).to(dt)
    gam, bet = 1 + 0.1 * torch.randn(D, generator=g), 0.1 * torch.randn(D, generator=g)
    t = x.to(dt).to(gpu_device)
    dev = lambda a: a.to(gpu_device).contiguous()          # noqa: E731
    args = [dev(wqk), dev(bqk), dev(wv), dev(bv), dev(qpos), dev(wo), dev(bo), dev(gam), dev(bet)]
    L = _lib.lib()
    rc = L.spe_debug_decsa(None, _p(t), ldt, B, Q, _p(args[0]), D, _p(args[1]), _p(args[2]), D, _p(args[3]),
                           _p(args[4]), _p(args[5]), D, _p(args[6]), _p(args[7]), _p(args[8]), 32 ** -0.5)
    assert rc == 0, L.spe_last_error()
    torch.cuda.synchronize()
    if B == 0:
        assert torch.equal(t.cpu(), x.to(dt))
        return
    r = lambda a: a.to(dt).float()                         # noqa: E731  (bf16 rounding)
    xb = x[:, :D].to(dt).float()
    qk = r(xb @ wqk.float().T + bqk + qpos.float().repeat(B, 1))
    v = r(xb @ wv.float().T + bv)
    q, k = qk[:, :D].view(B, Q, H, 32), qk[:, D:].view(B, Q, H, 32)
    s = torch.einsum("bihc,bjhc->bhij", q * 32 ** -0.5, k)
    o = r(torch.einsum("bhij,bjhc->bihc", torch.softmax(s, -1), v.view(B, Q, H, 32)).reshape(B * Q, D))
    y = torch.nn.functional.layer_norm(o @ wo.float().T + bo + xb, (D,), gam, bet, 1e-5)
    _close(t[:, :D].cpu(), y, 2e-2)
    assert torch.equal(t[:, D:].cpu(), x[:, D:].to(dt))   # nothing written past D


@pytest.mark.parametrize("B,Q", [(3, 11), (2, 40), (1, 64), (0, 11)])
def test_decoder_out_projection_norm(gpu_device, B, Q):
    """decproj (decsa.hip): tgt = LN(tgt + x . Wo^T + bo) in place, one workgroup per image
    (REV/models/transformer.py:233-234, the cross-attention's out-projection + norm2), against
    torch fp32 on the same bf16 operands; 2e-2 * scale (bf16 output)."""
    dt, D = torch.bfloat16, 256
    g = torch.Generator(device="cpu").manual_seed(7 * B + Q)
    ld = D + 8
    t0 = torch.randn(max(B, 1) * Q, ld, generator=g)
    x = torch.randn(max(B, 1) * Q, ld, generator=g).to(dt)
    wo = (torch.randn(D, D, generator=g) / 16).to(dt)
    bo = torch.randn(D, generator=g) * 0.1
    gam, bet = 1 + 0.1 * torch.randn(D, generator=g), 0.1 * torch.randn(D, generator=g)
    t = t0.to(dt).to(gpu_device)
    dev = lambda a: a.to(gpu_device).contiguous()          # noqa: E731
    xd, wod, bod, gd, bd = dev(x), dev(wo), dev(bo), dev(gam), dev(bet)
    L = _lib.lib()
    rc = L.spe_debug_decproj(None, _p(t), ld, _p(xd), ld, B, Q, _p(wod), D, _p(bod), _p(gd), _p(bd))
    assert rc == 0, L.spe_last_error()
    torch.cuda.synchronize()
    if B == 0:
        assert torch.equal(t.cpu(), t0.to(dt))
        return
    y = torch.nn.functional.layer_norm(x[:, :D].float() @ wo.float().T + bo + t0[:, :D].to(dt).float(), (D,), gam,
                                       bet, 1e-5)
    _close(t[:, :D].cpu(), y, 2e-2)
    assert torch.equal(t[:, D:].cpu(), t0[:, D:].to(dt))


@pytest.mark.parametrize("dtype", ["bf16", "fp32"])
def test_layernorm(gpu_device, dtype):
    code, dt, tol = DT[dtype]
    M = 333
    g = torch.Generator(device="cpu").manual_seed(1)
    x = (torch.randn(M, 256, generator=g) * 3 + 1).to(gpu_device, dt)
    gam = torch.randn(256, generator=g).to(gpu_device)
    bet = torch.randn(256, generator=g).to(gpu_device)
    out = torch.zeros(M, 256, dtype=dt, device=gpu_device)
    out32 = torch.zeros(M, 256, device=gpu_device)
    assert _lib.lib().spe_debug_layernorm(None, code, _p(x), _p(gam), _p(bet), _p(out), _p(out32), M, 256) == 0
    torch.cuda.synchronize()
    ref = F.layer_norm(x.float(), (256,), gam, bet, 1e-5)
    _close(out32, ref, 1e-5)
    _close(out, ref, tol)


@pytest.mark.parametrize("dtype", ["bf16", "fp32"])
@pytest.mark.parametrize("B,H,W,Cin,Cout", [(2, 26, 26, 1024, 256), (3, 5, 7, 64, 16), (1, 1, 3, 32, 8),
                                            (2, 5, 7, 64, 32), (1, 1, 3, 32, 64), (2, 40, 40, 128, 96)])
def test_upconv_low_resolution(gpu_device, dtype, B, H, W, Cin, Cout):
    """bf16 neck: conv3x3(pad 1)(UpsamplingBilinear2d(x2)(x)) (REV/models/backbone.py:141) as one
    per-tap GEMM at the low resolution + spe_debug_upconv's bilinear combine, written into a
    channel slice of a wider concat buffer, against torch's upsample-then-conv in fp32."""
    _, dt, tol = DT[dtype]
    g = torch.Generator(device="cpu").manual_seed(B * H + Cin + W)
    x = torch.randn(B, Cin, H, W, generator=g).to(gpu_device, dt)
    w = (torch.randn(Cout, Cin, 3, 3, generator=g) / (Cin * 9) ** 0.5).to(gpu_device, dt)
    ref = F.conv2d(F.interpolate(x.float(), scale_factor=2, mode="bilinear", align_corners=True), w.float(), padding=1)
    taps = w.permute(2, 3, 0, 1).reshape(9 * Cout, Cin)              # row t*Cout + co, t = kh*3 + kw
    ldb = (Cin + 63) // 64 * 64
    M = B * H * W
    Z = torch.zeros(M, 9 * Cout, dtype=dt, device=gpu_device)
    _gemm(dtype, 0, x.permute(0, 2, 3, 1).contiguous(), _padded_weight(taps, ldb, dt), M, 9 * Cout, Cin, Cin, ldb, Z,
          9 * Cout)
    ldo = 2 * Cout + 8
    out = torch.zeros(B * 4 * H * W, ldo, dtype=dt, device=gpu_device)
    rc = _lib.lib().spe_debug_upconv(None, DT[dtype][0], _p(Z), _p(out[:, Cout:]), ldo, B, H, W, Cout)
    assert rc == 0, _lib.lib().spe_last_error()
    torch.cuda.synchronize()
    _close(out[:, Cout:2 * Cout], ref.permute(0, 2, 3, 1).reshape(-1, Cout), tol)
    assert (out[:, :Cout] == 0).all() and (out[:, 2 * Cout:] == 0).all()


# (K, N, epilogue): the short-K linear problems of the bench (ResNet 1x1 convs, neck, encoder
# projections) at sizes large enough for the persistent streaming kernel (gemm_stream.hip)
SGEMM_CASES = [(64, 64, "relu"), (256, 64, "relu"), (256, 64, "plain"), (256, 128, "relu"), (256, 128, "res_relu"),
               (512, 128, "relu"), (512, 64, "res_relu"), (512, 256, "bias"), (256, 1024, "res_relu"),
               (256, 512, "res_periodic_f16"), (256, 256, "vt"), (256, 256, "vt_f16"), (256, 256, "res_ln")]


@pytest.mark.parametrize("K,N,epi", SGEMM_CASES)
def test_gemm_streaming_short_k(gpu_device, K, N, epi):
    """Persistent weight-stationary kernel: W slice resident in LDS, row tiles streamed through
    registers, epilogues (bias, residual before ReLU, row-periodic residual, fp16 store, V^T
    store, fused LayerNorm) straight from the accumulators; ragged M (rows past M computed, not
    stored), output strides wider than N, N split over workgroup slices."""
    dt, tol = torch.bfloat16, 1e-2
    T = 2704
    M = 52 * T if epi.startswith("vt") else 140003
    g = torch.Generator(device="cpu").manual_seed(K * 3 + N + len(epi))
    A = torch.randn(M, K, generator=g).to(gpu_device, dt)
    Wt = (torch.randn(N, K, generator=g) / K ** 0.5).to(gpu_device, dt)
    bias = torch.randn(N, generator=g).to(gpu_device)
    ldc = N + 8 if not epi.startswith("vt") else N
    f16 = epi.endswith("f16")
    C = torch.zeros(M, ldc, dtype=torch.float16 if f16 else dt, device=gpu_device)
    y = A.float() @ Wt.float().t() + bias
    kw = {}
    if epi.startswith("res"):
        if "periodic" in epi:
            R = torch.randn(T, N, generator=g).to(gpu_device, dt)
            kw = dict(R=R, ldr=N, r_period=T)
            y = y + R.float().repeat(M // T + 1, 1)[:M]
        else:
            R = torch.randn(M, N, generator=g).to(gpu_device, dt)
            kw = dict(R=R, ldr=N)
            y = y + R.float()
    if "relu" in epi:
        kw["relu"] = 1
        y = torch.relu(y)
    if "ln" in epi:
        gam = torch.randn(N, generator=g).to(gpu_device)
        bet = torch.randn(N, generator=g).to(gpu_device)
        kw["ln"] = (gam, bet)
        y = F.layer_norm(y, (N,), gam, bet, 1e-5)
    if epi.startswith("vt"):
        B = M // T
        C = torch.zeros(B * N * T, dtype=torch.float16 if f16 else dt, device=gpu_device)
        _gemm("bf16", 0, A, _padded_weight(Wt, K, dt), M, N, K, K, K, C, 8, bias=bias, vt=(T, B), out_f16=int(f16))
        got = C.view(N // 256, B, 256, T).permute(1, 3, 0, 2).reshape(M, N)
    else:
        _gemm("bf16", 0, A, _padded_weight(Wt, K, dt), M, N, K, K, K, C, ldc, bias=None if epi == "plain" else bias,
              out_f16=int(f16), **kw)
        got = C[:, :N]
        assert (C[:, N:] == 0).all()
        if epi == "plain":
            y = y - bias
    # (K = N = 256 with the LayerNorm epilogue is the out-projection + norm1 kernel, lnproj.hip)
    want = 4 if (epi == "res_ln" and K == 256 and N == 256) else 2
    assert _lib.lib().spe_debug_gemm_path() == want, "expected the streaming kernel"
    _close(got, y, tol)


@pytest.mark.parametrize("rows", [52 * 2704, 2 * 2704])
def test_gemm_f16_store_saturates(gpu_device, rows):
    """fp16 GEMM outputs (the encoder's V^T / config-5 q,k operands) saturate at +-65504 rather
    than overflowing to inf (an inf V entry would make the attention output NaN); in-range values
    are unchanged.  Both the streaming kernel (large M) and the tiled kernels (small M)."""
    T, K, N = 2704, 256, 256
    g = torch.Generator(device="cpu").manual_seed(91)
    A = torch.randn(rows, K, generator=g).to(gpu_device, torch.bfloat16)
    Wt = (torch.randn(N, K, generator=g) / K ** 0.5).to(gpu_device, torch.bfloat16)
    bias = torch.randn(N, generator=g).to(gpu_device)
    bias[::7] = 1e6
    bias[3::7] = -1e6
    B = rows // T
    C = torch.zeros(B * N * T, dtype=torch.float16, device=gpu_device)
    _gemm("bf16", 0, A, _padded_weight(Wt, K, torch.bfloat16), rows, N, K, K, K, C, 8, bias=bias, vt=(T, B), out_f16=1)
    got = C.view(N // 256, B, 256, T).permute(1, 3, 0, 2).reshape(rows, N).float()
    assert torch.isfinite(got).all()
    big = torch.zeros(N, dtype=torch.bool, device=gpu_device)
    big[::7] = True
    big[3::7] = True
    assert (got[:, big].abs() == 65504).all()
    y = A.float() @ Wt.float().t() + bias
    _close(got[:, ~big], y[:, ~big], 1e-2)


# ---------------------------------------------------------------- fp32x3 (split-bf16) parity mode
def _weight_planes(Wp):
    """fp32 [N][ldb] -> bf16 [3][N][ldb] h, m, l (RNE each; what spe_model_finalize writes)."""
    h = Wp.to(torch.bfloat16)
    r = Wp - h.float()
    m = r.to(torch.bfloat16)
    return torch.stack([h, m, (r - m.float()).to(torch.bfloat16)]).contiguous()


def _gemm_planes(mode, A, Wp, M, N, K, lda, C, ldc, bias=None, R=None, ldr=0, relu=0, conv=(0, 0, 0, 1, 1, 1, 0)):
    L = _lib.lib()
    H, Wd, Cin, KH, KW, stride, pad = conv
    planes = _weight_planes(Wp)
    rc = L.spe_debug_gemm_planes(None, _lib.SPE_DTYPE_F32X6, mode, _p(A), lda, None, 0, 1, H, Wd, Cin, KH, KW, stride,
                                 pad, _p(Wp), Wp.shape[1], M, N, K, _p(bias), _p(R), ldr, relu, _p(C), ldc, _p(planes),
                                 Wp.shape[0])
    assert rc == 0, L.spe_last_error()
    torch.cuda.synchronize()
    return L.spe_debug_gemm_path()


def _h3_planes(Wp):
    """fp32 [N][ldb] -> (fp16 [2][N][ldb] hi, lo of W[n] * 2^e_n, fp32 2^-e_n [N]) with max |W[n]| 2^e_n
    in [2^12, 2^13) (what spe_model_finalize writes for fp32h3 models)."""
    am = Wp.abs().amax(1).double()
    e = torch.where(am > 0, torch.frexp(am).exponent.double(), torch.zeros_like(am))
    sc = torch.where(am > 0, torch.pow(2.0, 13 - e), torch.ones_like(am)).float()[:, None]
    x = Wp * sc
    h = x.to(torch.float16)
    lo = (x - h.float()).to(torch.float16)
    return torch.stack([h, lo]).contiguous(), (1.0 / sc[:, 0]).contiguous()


def _gemm_h3(mode, A, Wp, M, N, K, lda, C, ldc, bias=None, R=None, ldr=0, relu=0, conv=(0, 0, 0, 1, 1, 1, 0)):
    """one fp32h3 launch (gemm path 7) with A's max |x| on the device; checks the published max |C|."""
    L = _lib.lib()
    H, Wd, Cin, KH, KW, stride, pad = conv
    planes, sinv = _h3_planes(Wp)
    amax_a = A.abs().max().reshape(1).contiguous()
    amax_c = torch.zeros(1, device=A.device)
    rc = L.spe_debug_gemm_h3(None, mode, _p(A), lda, H, Wd, Cin, KH, KW, stride, pad, Wp.shape[1], M, N, K, _p(bias),
                             _p(R), ldr, relu, _p(C), ldc, _p(planes), Wp.shape[0], _p(sinv), _p(amax_a),
                             _p(amax_c), 0.0)
    assert rc == 0, L.spe_last_error()
    torch.cuda.synchronize()
    path = L.spe_debug_gemm_path()
    assert path in (7, 8), path
    stored = C[:, :N] if C.dim() == 2 else C
    assert amax_c.item() == stored.abs().max().item(), (amax_c.item(), stored.abs().max().item())
    return path


def _split_gemm_err(gpu_device, case, dtype, planes=False, want_path=None, amp=1.0):
    """max |C - C_fp64| / max |C_fp64| of one launch of `dtype` on `case` (planes: fp32x6 with the
    weights pre-split, as the models launch it; dtype fp32h3: the scaled fp16 split with its
    finalize-form planes; want_path: the kernel that must have run; amp scales A)."""
    g = torch.Generator(device="cpu").manual_seed(len(case))
    dev, f = gpu_device, torch.float32
    if case.startswith("conv"):
        B, H, Cin, Cout, k, st, pd = {"conv3x3": (2, 26, 256, 256, 3, 1, 1), "conv3x3_n64": (2, 26, 64, 64, 3, 1, 1),
                                      "conv1x1s2": (2, 52, 512, 256, 1, 2, 0), "conv3x3_big": (16, 104, 64, 128, 3, 1, 1),
                                      "conv7x7s2_c8": (2, 40, 8, 64, 7, 2, 3)}[case]
        x = torch.randn(B, Cin, H, H, generator=g, dtype=torch.float64) * amp
        w = torch.randn(Cout, Cin, k, k, generator=g, dtype=torch.float64) / (Cin * k * k) ** 0.5
        ref = F.conv2d(x, w, stride=st, padding=pd).permute(0, 2, 3, 1).reshape(-1, Cout)
        A = x.permute(0, 2, 3, 1).contiguous().to(dev, f)
        Wp = _pack_conv(w).to(dev, f).contiguous()
        Ho = (H + 2 * pd - k) // st + 1
        M, K = B * Ho * Ho, Cin * k * k
        if K % 64:                                     # weight rows padded to 64 elements
            Wp = torch.nn.functional.pad(Wp, (0, 64 - K % 64))
        C = torch.zeros(M, Cout, dtype=f, device=dev)
        if dtype == "fp32h3":
            path = _gemm_h3(2, A, Wp, M, Cout, K, 0, C, Cout, conv=(H, H, Cin, k, k, st, pd))
            assert want_path is None or path == want_path, path
        elif planes:
            path = _gemm_planes(2, A, Wp, M, Cout, K, 0, C, Cout, conv=(H, H, Cin, k, k, st, pd))
            assert want_path is None or path == want_path, path
        else:
            _gemm(dtype, 2, A, Wp, M, Cout, K, 0, Wp.shape[1], C, Cout, conv=(H, H, Cin, k, k, st, pd))
        got = C
    else:
        M, N, K = {"vt": (2 * 2704, 256, 256), "linear_n64": (3000, 64, 256), "linear_n40": (3000, 40, 256),
                   "linear_many_res": (150001, 256, 64), "linear_many_n64": (150001, 64, 128),
                   "linear_big_res": (150001, 256, 256), "linear_longk_res": (704, 256, 2048),
                   "linear_longk": (77, 520, 2048)}.get(case, (3000, 200, 512))
        A = torch.randn(M, K, generator=g, dtype=torch.float64) * amp
        Wt = torch.randn(N, K, generator=g, dtype=torch.float64) / K ** 0.5
        bias = torch.randn(N, generator=g, dtype=torch.float64)
        ref = A @ Wt.t() + bias
        kw = {}
        ldc = N + 8
        if case in ("linear_add_relu_res", "linear_many_res", "linear_big_res", "linear_longk_res"):
            R = torch.randn(M, ldc, generator=g, dtype=torch.float64)
            ref = torch.relu(ref + R[:, :N])
            kw = dict(R=R.to(dev, f), ldr=ldc, relu=1)
        C = torch.zeros(M, ldc, dtype=f, device=dev)
        if case == "vt":
            T, Bv = 2704, 2
            C = torch.zeros(Bv * N * T, dtype=f, device=dev)
            _gemm(dtype, 0, A.to(dev, f), _padded_weight(Wt.to(dev, f), K, f), M, N, K, K, K, C, 4,
                  bias=bias.to(dev, f), vt=(T, Bv))
            got = C.view(N // 256, Bv, 256, T).permute(1, 3, 0, 2).reshape(M, N)
        elif dtype == "fp32h3":
            path = _gemm_h3(0, A.to(dev, f), _padded_weight(Wt.to(dev, f), K, f), M, N, K, K, C, ldc,
                            bias=bias.to(dev, f), **kw)
            assert want_path is None or path == want_path, path
            got = C[:, :N]
        elif planes:
            path = _gemm_planes(0, A.to(dev, f), _padded_weight(Wt.to(dev, f), K, f), M, N, K, K, C, ldc,
                                bias=bias.to(dev, f), **kw)
            assert want_path is None or path == want_path, path
            got = C[:, :N]
        else:
            _gemm(dtype, 0, A.to(dev, f), _padded_weight(Wt.to(dev, f), K, f), M, N, K, K, K, C, ldc,
                  bias=bias.to(dev, f), **kw)
            got = C[:, :N]
    return (got.double().cpu() - ref).abs().max().item() / ref.abs().max().item()


@pytest.mark.parametrize("dtype", ["fp32x3", "fp32x6"])
@pytest.mark.parametrize("case", ["linear", "linear_add_relu_res", "conv3x3", "conv1x1s2", "vt"])
def test_gemm_x3_close_to_fp64(gpu_device, case, dtype):
    """fp32 storage, split-bf16 MFMA: fp32x3 (hi.hi + hi.lo + lo.hi) within 2e-5 relative of an
    fp64 reference, i.e. far inside the fp32 parity tolerances and ~100x tighter than bf16;
    fp32x6 (three-way split, six products) at the exact-f32 MFMA kernel's own error on the same
    problem (fp32 accumulation over K = 256 .. 2304): <= max(1e-6, 2x that error)."""
    err = _split_gemm_err(gpu_device, case, dtype)
    if dtype == "fp32x3":
        assert err <= 2e-5, err
    else:
        e32 = _split_gemm_err(gpu_device, case, "fp32")
        assert err <= max(1e-6, 2 * e32), (err, e32)


@pytest.mark.parametrize("case", ["linear", "linear_add_relu_res", "conv3x3", "conv1x1s2", "linear_n64", "linear_n40",
                                  "conv3x3_n64", "conv7x7s2_c8"])
def test_gemm_x6_dma_close_to_fp64(gpu_device, case):
    """fp32x6 with the weights pre-split (the models' launch): the LDS-DMA kernel (gemm path 6)
    runs -- ragged M and N tiles, residual + ReLU epilogue, padded 3x3 and strided 1x1 implicit
    GEMMs, the 128 x 64 tile of N <= 64, the stem's 8-channel 7x7 with per-lane tap decode and a
    partial last K-step -- at the exact-f32 kernel's own error, like the register-staged x6
    kernel."""
    err = _split_gemm_err(gpu_device, case, "fp32x6", planes=True, want_path=6)
    e32 = _split_gemm_err(gpu_device, case, "fp32")
    assert err <= max(1e-6, 2 * e32), (err, e32)


@pytest.mark.parametrize("case,amp", [("linear", 1.0), ("linear_add_relu_res", 1.0), ("conv3x3", 1.0), ("conv1x1s2", 1.0),
                                      ("linear_n64", 1.0), ("linear_n40", 1.0), ("conv3x3_n64", 1.0),
                                      ("conv7x7s2_c8", 1.0), ("linear", 1e-7), ("linear", 1e6), ("conv3x3", 3e-5),
                                      ("linear_many_res", 1.0), ("linear_many_n64", 1.0), ("linear_big_res", 1.0),
                                      ("conv3x3_big", 1.0), ("linear_longk_res", 1.0), ("linear_longk", 1.0)])
def test_gemm_h3_close_to_fp64(gpu_device, case, amp):
    """fp32h3 (the scaled two-way fp16 split, three fp16 MFMAs) at the exact-f32 MFMA kernel's own
    error on the same problem -- ragged M and N tiles, residual + ReLU epilogue, padded 3x3 / strided
    1x1 implicit GEMMs, the 128 x 64 tile, the stem's 8-channel 7x7 with per-lane tap decode -- also
    for activations far below fp16's normal range (amp 1e-7, 3e-5) and far above its maximum (1e6):
    the power-of-two scale from max |A| keeps them at fp32 accuracy.  These row-store problems run
    the persistent form (gemm path 8); the *_many / *_big cases give each workgroup several tiles
    with a ragged last tile (linear_many_res at K = 64: a tile boundary every second step, 2344
    tiles on 512 slots; linear_many_n64, linear_big_res, conv3x3_big: K = 128, 256, 576); the
    linear_longk* cases (few rows, K = 2048: the decoder's linear2 shape, ragged M / N) the six-stage
    few-row form.  The published max |C| equals the stored output's exactly."""
    # (K = 2304, the layer-3 3x3: the non-persistent kernel, path 7; every other case persistent)
    err = _split_gemm_err(gpu_device, case, "fp32h3", amp=amp, want_path=7 if case == "conv3x3" else 8)
    e32 = _split_gemm_err(gpu_device, case, "fp32", amp=amp)
    assert err <= max(1e-6, 2 * e32), (err, e32)


def _h3_row_planes(W):
    """fp32 [N][K] -> (fp16 [2][N][K] hi, lo of W[n] 2^e_n, 2^-e_n) -- the h3 finalize form."""
    am = W.abs().amax(1).double()
    e = torch.where(am > 0, torch.frexp(am).exponent.double(), torch.zeros_like(am))
    sc = torch.where(am > 0, torch.pow(2.0, 13 - e), torch.ones_like(am)).float()[:, None]
    x = W * sc
    h = x.to(torch.float16)
    return torch.stack([h, (x - h.float()).to(torch.float16)]).contiguous(), (1.0 / sc[:, 0]).contiguous()


@pytest.mark.parametrize("M,F,inplace,loose", [(2 * 2704, 2048, True, False), (1000, 2048, False, True),
                                               (77, 96, True, False), (0, 64, False, False)])
def test_ffn_h3_one_pass(gpu_device, M, F, inplace, loose):
    """fp32h3 one-pass encoder FFN (ffn_h3.hip; REV/models/transformer.py:164-167): LayerNorm(x +
    ReLU(x W1^T + b1) W2^T + b2) with x a LayerNorm output, against fp64, within 2e-5 (the fused
    LayerNorm GEMM's bound) -- whole 128-row tiles and a ragged one, 64 / 3 hidden chunks, in place
    (y = x, as the model runs it) and not, the hidden scale from the tight bound and from one 2^10
    too loose (the split keeps fp32-level error); M = 0 launches nothing."""
    L = _lib.lib()
    dev, f = gpu_device, torch.float32
    g = torch.Generator(device="cpu").manual_seed(M + F)
    D = 256
    x = F_.layer_norm(torch.randn(max(M, 1), D, generator=g, dtype=torch.float64), (D,)) * 1.3 + 0.05
    x = x[:M]
    W1 = torch.randn(F, D, generator=g, dtype=torch.float64) / 16
    b1 = torch.randn(F, generator=g, dtype=torch.float64) * 0.1
    W2 = torch.randn(D, F, generator=g, dtype=torch.float64) / F ** 0.5
    b2 = torch.randn(D, generator=g, dtype=torch.float64) * 0.1
    gam = 1 + 0.1 * torch.randn(D, generator=g, dtype=torch.float64)
    bet = 0.1 * torch.randn(D, generator=g, dtype=torch.float64)
    hid = torch.relu(x @ W1.t() + b1)
    ref = F_.layer_norm(x + hid @ W2.t() + b2, (D,), gam, bet, 1e-5)
    hmax = hid.abs().max().item() if M else 1.0
    bound = hmax * (1024.0 if loose else 1.0) * (1 + 1e-6)
    sh = 2.0 ** (13 - math.frexp(bound)[1])
    w1p, s1 = _h3_row_planes(W1.to(f))
    meta = torch.stack([s1.view(F // 32, 32), b1.to(f).view(F // 32, 32)], 1).reshape(-1).contiguous()
    perm = torch.tensor([L.spe_debug_ffn_h3_perm(p) for p in range(32)])
    cols = (torch.arange(F) // 32) * 32 + perm[torch.arange(F) % 32]
    w2p, s2 = _h3_row_planes(W2.to(f)[:, cols].contiguous())
    xd = x.to(dev, f).contiguous()
    yd = xd if inplace else torch.zeros_like(xd)
    amax = (xd.abs().max() if M else torch.ones(())).reshape(1).to(dev).contiguous()
    keep = [t.to(dev).contiguous() for t in (w1p, meta, w2p, s2, b2.to(f), gam.to(f), bet.to(f))]
    rc = L.spe_debug_ffn_h3(None, _p(xd), D, _p(yd), D, M, F, _p(keep[0]), D, _p(keep[1]), _p(keep[2]), F,
                            _p(keep[3]), _p(keep[4]), _p(keep[5]), _p(keep[6]), _p(amax), sh)
    assert rc == 0, L.spe_last_error()
    torch.cuda.synchronize()
    if M:
        err = (yd.double().cpu() - ref).abs().max().item()
        assert err <= 2e-5, err


def _bf16_planes(x):
    """fp32 tensor -> bf16 hi plane followed by its lo plane (RNE both), flattened."""
    h = x.to(torch.bfloat16)
    return torch.cat([h.reshape(-1), (x - h.float()).to(torch.bfloat16).reshape(-1)])


@pytest.mark.parametrize("B,H,Tq,Tk", [(1, 8, 304, 336), (2, 8, 2704, 2704), (3, 8, 11, 2704)])
def test_attention_x3_presplit_equals_in_kernel_split(gpu_device, B, H, Tq, Tk):
    """K and V^T handed over as the bf16 hi / lo planes the projection epilogues write
    (GemmArgs::S, AttnArgs::presplit): the same RNE split the kernel does per tile, so the
    output is bit-identical to the fp32-operand launch."""
    g = torch.Generator(device="cpu").manual_seed(Tq + Tk)
    ld = H * 32
    Q = (torch.randn(B * Tq, ld, generator=g) * 2).to(gpu_device)
    K = (torch.randn(B * Tk, ld, generator=g) * 2).to(gpu_device)
    VT = torch.randn(B, H, 32, Tk, generator=g).to(gpu_device)
    Kp, VTp = _bf16_planes(K), _bf16_planes(VT)
    O = torch.zeros(B * Tq, ld, device=gpu_device)
    Op = torch.zeros_like(O)
    L = _lib.lib()
    assert L.spe_debug_attention(None, _lib.SPE_DTYPE_F32X3, _p(Q), ld, _p(K), ld, _p(VT), _p(O), ld, B, H, Tq, Tk,
                                 32 ** -0.5) == 0
    assert L.spe_debug_attention(None, _lib.SPE_DTYPE_F32X3 | 0x200, _p(Q), ld, _p(Kp), ld, _p(VTp), _p(Op), ld, B,
                                 H, Tq, Tk, 32 ** -0.5) == 0
    torch.cuda.synchronize()
    assert torch.equal(O, Op), (O - Op).abs().max().item()


@pytest.mark.parametrize("B,H,Tq,Tk", [(1, 8, 300, 333), (2, 8, 2704, 2704), (3, 8, 11, 2704), (2, 8, 11, 11)])
def test_attention_x3_close_to_fp64(gpu_device, B, H, Tq, Tk):
    g = torch.Generator(device="cpu").manual_seed(Tq * 3 + Tk)
    ld = H * 32 + 16
    Q = torch.randn(B * Tq, ld, generator=g, dtype=torch.float64) * 2
    K = torch.randn(B * Tk, ld, generator=g, dtype=torch.float64) * 2
    V = torch.randn(B, H, Tk, 32, generator=g, dtype=torch.float64)
    dev = gpu_device
    O = torch.zeros(B * Tq, H * 32, dtype=torch.float32, device=dev)
    scale = 32 ** -0.5
    Qd, Kd = Q.to(dev, torch.float32), K.to(dev, torch.float32)     # kept alive across the call
    VTd = V.transpose(-1, -2).contiguous().to(dev, torch.float32)
    rc = _lib.lib().spe_debug_attention(None, _lib.SPE_DTYPE_F32X3, _p(Qd), ld, _p(Kd), ld, _p(VTd), _p(O), H * 32, B,
                                        H, Tq, Tk, scale)
    assert rc == 0
    torch.cuda.synchronize()
    q = Q[:, : H * 32].view(B, Tq, H, 32).transpose(1, 2)
    k = K[:, : H * 32].view(B, Tk, H, 32).transpose(1, 2)
    ref = torch.softmax(q @ k.transpose(-1, -2) * scale, -1) @ V
    ref = ref.transpose(1, 2).reshape(B * Tq, H * 32)
    err = (O.double().cpu() - ref).abs().max().item() / ref.abs().max().item()
    assert err <= 5e-5, err


def _vt_pos(T):
    """the 16-bit attention operands' key order (spe_kernels.h vt_pos): stored position of key t"""
    t = torch.arange(T)
    return (t & ~12) | ((t & 4) << 1) | ((t & 8) >> 1)


def _split_planes(K, VT, f16v):
    """K -> bf16 hi / lo planes; V^T [B][H][32][T] -> hi / lo planes in vt_pos key order, bf16 or fp16"""
    vs = torch.empty_like(VT)
    vs[..., _vt_pos(VT.shape[-1]).to(VT.device)] = VT
    dt = torch.float16 if f16v else torch.bfloat16
    h = vs.to(dt)
    return _bf16_planes(K), torch.cat([h.reshape(-1), (vs - h.float()).to(dt).reshape(-1)])


@pytest.mark.parametrize("f16v", [0, 1])
@pytest.mark.parametrize("B,H,Tq,Tk", [(1, 8, 300, 336), (2, 8, 2704, 2704), (3, 8, 11, 2704), (2, 8, 40, 48),
                                       (1, 8, 64, 64), (1, 8, 130, 192)])
def test_attention_split_dma_close_to_fp64(gpu_device, f16v, B, H, Tq, Tk):
    """The LDS-DMA split-operand encoder attention (attn_split.hip) on the planes the fp32 models'
    projection epilogues write: K bf16 hi / lo, V^T hi / lo in vt_pos order (bf16, or fp16 as in
    fp32h3), against an fp64 softmax.  The scores carry the bf16 split's ~2^-17 per product; the
    value product ~2^-17 (bf16 P) or ~2^-21 (fp16 P)."""
    g = torch.Generator(device="cpu").manual_seed(Tq * 7 + Tk + f16v)
    ld = H * 32
    Q = torch.randn(B * Tq, ld + 16, generator=g, dtype=torch.float64) * 2
    K = torch.randn(B * Tk, ld, generator=g, dtype=torch.float64) * 2
    V = torch.randn(B, H, Tk, 32, generator=g, dtype=torch.float64)
    dev = gpu_device
    Qd, Kd = Q.to(dev, torch.float32), K.to(dev, torch.float32)
    VTd = V.transpose(-1, -2).contiguous().to(dev, torch.float32)
    Kp, VTp = _split_planes(Kd, VTd, f16v)
    O = torch.full((B * Tq, ld), float("nan"), dtype=torch.float32, device=dev)
    code = _lib.SPE_DTYPE_F32X3 | 0x100 | 0x200 | (0x400 if f16v else 0)
    rc = _lib.lib().spe_debug_attention(None, code, _p(Qd), ld + 16, _p(Kp), ld, _p(VTp), _p(O), ld, B, H, Tq, Tk,
                                        32 ** -0.5)
    assert rc == 0
    torch.cuda.synchronize()
    q = Qd.double().cpu()[:, :ld].view(B, Tq, H, 32).transpose(1, 2)
    k = Kd.double().cpu().view(B, Tk, H, 32).transpose(1, 2)
    ref = torch.softmax(q @ k.transpose(-1, -2) * 32 ** -0.5, -1) @ VTd.double().cpu().transpose(-1, -2)
    ref = ref.transpose(1, 2).reshape(B * Tq, ld)
    err = (O.double().cpu() - ref).abs().max().item() / ref.abs().max().item()
    assert err <= 5e-5, err


@pytest.mark.parametrize("f16v", [0, 1])
@pytest.mark.parametrize("gain", [3.0, 12.0, 40.0])
def test_attention_split_dma_large_score_range(gpu_device, f16v, gain):
    """The split kernel's lazy softmax when late keys dominate: a stale running max lets some p pass
    2^12, the lane-sum test must send that tile through the recompute + rescale path."""
    B, H, T = 2, 8, 336
    g = torch.Generator(device="cpu").manual_seed(int(gain) + 100 * f16v)
    Q = torch.randn(B * T, 256, generator=g, dtype=torch.float64)
    K = torch.randn(B * T, 256, generator=g, dtype=torch.float64)
    K[T - 90:T] *= gain
    K[2 * T - 20:] *= gain / 2
    V = torch.randn(B, H, T, 32, generator=g, dtype=torch.float64)
    dev = gpu_device
    Qd, Kd = Q.to(dev, torch.float32), K.to(dev, torch.float32)
    VTd = V.transpose(-1, -2).contiguous().to(dev, torch.float32)
    Kp, VTp = _split_planes(Kd, VTd, f16v)
    O = torch.zeros(B * T, 256, dtype=torch.float32, device=dev)
    code = _lib.SPE_DTYPE_F32X3 | 0x100 | 0x200 | (0x400 if f16v else 0)
    assert _lib.lib().spe_debug_attention(None, code, _p(Qd), 256, _p(Kp), 256, _p(VTp), _p(O), 256, B, H, T, T,
                                          32 ** -0.5) == 0
    torch.cuda.synchronize()
    q = Qd.double().cpu().view(B, T, H, 32).transpose(1, 2)
    k = Kd.double().cpu().view(B, T, H, 32).transpose(1, 2)
    ref = torch.softmax(q @ k.transpose(-1, -2) * 32 ** -0.5, -1) @ V
    ref = ref.transpose(1, 2).reshape(B * T, 256)
    err = (O.double().cpu() - ref).abs().max().item() / ref.abs().max().item()
    assert err <= 5e-5 * max(1.0, gain / 8), err


@pytest.mark.parametrize("dtype,gain", [("fp32x3", 3.0), ("fp32x3", 12.0), ("fp32x3", 40.0), ("fp32", 12.0),
                                        ("fp32", 40.0)])
def test_attention_fp32_modes_large_score_range(gpu_device, dtype, gain):
    """fp32 / fp32x3 attention when late keys dominate (scores spanning > 100 in log2 space): the
    x3 kernel keeps a stale running max until a tile passes it by more than the rescale slack,
    so late jumps must go through its rescale path; both against an fp64 softmax."""
    B, H, T = 2, 8, 333
    g = torch.Generator(device="cpu").manual_seed(int(gain))
    Q = torch.randn(B * T, 256, generator=g, dtype=torch.float64)
    K = torch.randn(B * T, 256, generator=g, dtype=torch.float64)
    K[T - 90:T] *= gain                              # late keys of image 0 dominate
    K[2 * T - 20:] *= gain / 2                       # image 1: a milder jump in its last tile
    V = torch.randn(B, H, T, 32, generator=g, dtype=torch.float64)
    dev = gpu_device
    Qd, Kd = Q.to(dev, torch.float32), K.to(dev, torch.float32)
    VTd = V.transpose(-1, -2).contiguous().to(dev, torch.float32)
    O = torch.zeros(B * T, 256, dtype=torch.float32, device=dev)
    scale = 32 ** -0.5
    rc = _lib.lib().spe_debug_attention(None, DT[dtype][0], _p(Qd), 256, _p(Kd), 256, _p(VTd), _p(O), 256, B, H, T,
                                        T, scale)
    assert rc == 0
    torch.cuda.synchronize()
    q = Qd.double().cpu().view(B, T, H, 32).transpose(1, 2)
    k = Kd.double().cpu().view(B, T, H, 32).transpose(1, 2)
    ref = torch.softmax(q @ k.transpose(-1, -2) * scale, -1) @ V
    ref = ref.transpose(1, 2).reshape(B * T, 256)
    err = (O.double().cpu() - ref).abs().max().item() / ref.abs().max().item()
    # x3: each score carries ~2^-17 of sum |q_i k_i| (the split's product error), so the bound
    # grows with the score magnitude (gain 40: scores of ~200 log2 units, error ~1e-3 of a p)
    assert err <= (5e-5 * max(1.0, gain / 8) if dtype == "fp32x3" else 1e-5), err
