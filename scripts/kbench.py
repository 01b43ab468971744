"""Per-kernel microbenchmark at the bench workload's shapes (B=64, 416x416 -> 2704 tokens),
through the C-ABI kernel test hooks.  Run alone for timings, or under rocprofv3 --pmc for
counters of one kernel family.

usage: python scripts/kbench.py [attn|ffn|all] [--iters 20]
"""
import argparse
import ctypes
import os
import sys

import torch

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(REPO, "satellite-pose-estimation_amd"))
from spe import _lib  # noqa: E402


def p(t):
    return ctypes.c_void_p(t.data_ptr())


def _pack(L, w):
    """bf16 rows [N][256] -> the decoder kernels' fragment-packed layout (spe_debug_wfrag_pack)"""
    out = torch.empty_like(w)
    assert L.spe_debug_wfrag_pack(None, p(w), w.shape[1], w.shape[0], p(out)) == 0
    return out


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
    ap.add_argument("which", nargs="?", default="all")
    ap.add_argument("--iters", type=int, default=20)
    ap.add_argument("--batch", type=int, default=64)
    ap.add_argument("--only", default="")
    ap.add_argument("--attn-dtype", type=int, default=0, help="0 bf16, 1 fp32, 2 fp16, 3 bf16 q/k + fp16 V^T/P, 4 fp32x3")
    ap.add_argument("--dma", action="store_true", help="the encoder's LDS-DMA attention kernel (V^T key order as stored)")
    ap.add_argument("--presplit", action="store_true", help="fp32x3: K and V^T as the bf16 hi / lo planes the models pass")
    ap.add_argument("--split-dma", action="store_true",
                    help="with --presplit: V^T planes in vt_pos key order -> the LDS-DMA split kernel (attn_split.hip)")
    ap.add_argument("--f16v", action="store_true", help="with --split-dma: fp16 V^T planes (the fp32h3 model's form)")
    a = ap.parse_args()
    L = _lib.lib()
    dev = torch.device("cuda", 0)
    B, H, T, D, F = a.batch, 8, 2704, 256, 2048
    g = torch.Generator(device="cpu").manual_seed(0)
    if a.which in ("attn", "all"):
        f32 = a.attn_dtype in (1, 4)               # exact fp32 / fp32x3 parity kernels: fp32 operands
        qk = torch.randn(B * T, 512, generator=g).to(dev, torch.float32 if f32 else torch.bfloat16)
        vdt = torch.float16 if a.attn_dtype in (2, 3) else torch.float32 if f32 else torch.bfloat16
        if a.attn_dtype == 2:
            qk = qk.to(torch.float16)
        vt = torch.randn(B, H, 32, T, generator=g).to(dev, vdt)
        o = torch.empty(B * T, D, dtype=torch.float32 if f32 else torch.bfloat16, device=dev)
        kp = ctypes.c_void_p(qk.data_ptr() + 256 * qk.element_size())
        code = a.attn_dtype | (0x100 if a.dma else 0)
        ldk = 512
        if a.presplit and a.attn_dtype == 4:             # (the planes kept alive in `keep`)
            kf = qk[:, 256:].contiguous()
            kh = kf.to(torch.bfloat16)
            vdt2 = torch.bfloat16
            if a.split_dma:                              # keys to vt_pos order (a permutation: timing only)
                t = torch.arange(T, device=dev)
                vs = torch.empty_like(vt)
                vs[..., (t & ~12) | ((t & 4) << 1) | ((t & 8) >> 1)] = vt
                vt, code = vs, code | 0x100 | (0x400 if a.f16v else 0)
                vdt2 = torch.float16 if a.f16v else torch.bfloat16
            vh = vt.to(vdt2)
            keep = [torch.cat([kh.reshape(-1), (kf - kh.float()).to(torch.bfloat16).reshape(-1)]),
                    torch.cat([vh.reshape(-1), (vt - vh.float()).to(vdt2).reshape(-1)])]
            kp, vt, ldk, code = ctypes.c_void_p(keep[0].data_ptr()), keep[1], 256, code | 0x200
        fn = lambda: L.spe_debug_attention(None, code, p(qk), 512, kp, ldk, p(vt), p(o), D, B, H, T, T, 32 ** -0.5)
        ms = timeit(fn, a.iters)
        fl = 4.0 * B * H * T * T * 32
        print(f"attn.enc  {ms:.3f} ms  {fl / ms / 1e9:.1f} TF/s")
    if a.which in ("ffn", "all"):
        x = torch.randn(B * T, D, generator=g).to(dev, torch.bfloat16)
        w1 = (torch.randn(F, D, generator=g) / 16).to(dev, torch.bfloat16)
        w2 = (torch.randn(D, F, generator=g) / 45).to(dev, torch.bfloat16)
        b1 = torch.zeros(F, device=dev)
        b2 = torch.zeros(D, device=dev)
        gm = torch.ones(D, device=dev)
        bt = torch.zeros(D, device=dev)
        y = torch.empty_like(x)
        fn = lambda: L.spe_debug_ffn(None, p(x), D, p(w1), D, p(b1), p(w2), F, p(b2), p(gm), p(bt), p(y), D,
                                     B * T, D, F, None, 0)
        ms = timeit(fn, a.iters)
        fl = 4.0 * B * T * D * F
        print(f"ffn.enc   {ms:.3f} ms  {fl / ms / 1e9:.1f} TF/s")
        w2c = w2.view(D, F // 32, 32).permute(1, 0, 2).contiguous()     # chunk-packed W2 (the model's form)
        fn = lambda: L.spe_debug_ffn(None, p(x), D, p(w1), D, p(b1), p(w2c), 0, p(b2), p(gm), p(bt), p(y), D,
                                     B * T, D, F, None, 0)
        ms = timeit(fn, a.iters)
        print(f"ffn.enc chunk-packed W2  {ms:.3f} ms  {fl / ms / 1e9:.1f} TF/s")
    if a.which in ("ffnh3",):
        # the fp32h3 one-pass encoder FFN (ffn_h3.hip) at the bench's M = B * 2704 rows, weights in the
        # finalize form (h3 row planes, W2 columns in spe_ffn_h3_perm order); numerics: test_ffn_h3_one_pass
        import math
        M = B * T
        x = torch.nn.functional.layer_norm(torch.randn(M, D, generator=g), (D,)).to(dev)
        W1 = torch.randn(F, D, generator=g) / 16
        W2 = torch.randn(D, F, generator=g) / F ** 0.5

        def planes(W):
            am = W.abs().amax(1)
            e = torch.frexp(am).exponent.float()
            sc = torch.pow(2.0, 13 - e)[:, None]
            xx = W * sc
            h = xx.to(torch.float16)
            return torch.stack([h, (xx - h.float()).to(torch.float16)]).contiguous(), (1.0 / sc[:, 0]).contiguous()
        w1p, s1 = planes(W1)
        meta = torch.stack([s1.view(F // 32, 32), torch.zeros(F // 32, 32)], 1).reshape(-1).contiguous()
        perm = torch.tensor([L.spe_debug_ffn_h3_perm(q) for q in range(32)])
        cols = (torch.arange(F) // 32) * 32 + perm[torch.arange(F) % 32]
        w2p, s2 = planes(W2[:, cols].contiguous())
        keep = [t.to(dev).contiguous() for t in (w1p, meta, w2p, s2, torch.zeros(D), torch.ones(D), torch.zeros(D))]
        amax = x.abs().max().reshape(1).contiguous()
        sh = 2.0 ** (13 - math.frexp(64.0)[1])
        y = torch.empty_like(x)
        fn = lambda: L.spe_debug_ffn_h3(None, p(x), D, p(y), D, M, F, p(keep[0]), D, p(keep[1]), p(keep[2]), F,
                                         p(keep[3]), p(keep[4]), p(keep[5]), p(keep[6]), p(amax), sh)
        assert fn() == 0
        ms = timeit(fn, a.iters)
        fl = 4.0 * M * D * F
        print(f"ffn.enc h3  {ms:.3f} ms  {fl / ms / 1e9:.1f} TF/s")
    if a.which in ("ffndec", "all"):
        # the decoder's few-row FFN (M = B * 11): split-F partials over `splits` workgroups per
        # 128-row tile, then the reduce + LayerNorm kernel
        M = B * 11
        x = torch.randn(M, D, generator=g).to(dev, torch.bfloat16)
        w1 = (torch.randn(F, D, generator=g) / 16).to(dev, torch.bfloat16)
        w2 = (torch.randn(D, F, generator=g) / 45).to(dev, torch.bfloat16)
        b1, b2 = torch.zeros(F, device=dev), torch.zeros(D, device=dev)
        gm, bt = torch.ones(D, device=dev), torch.zeros(D, device=dev)
        y = torch.empty_like(x)
        part = torch.empty(64 * M * D, device=dev)
        for sp in (1, 2, 4, 8, 16, 32, 64):
            fn = lambda: L.spe_debug_ffn(None, p(x), D, p(w1), D, p(b1), p(w2), F, p(b2), p(gm), p(bt), p(y), D,
                                         M, D, F, p(part) if sp > 1 else None, sp)
            if fn() != 0:
                print(f"ffn.dec splits={sp}: rejected")
                continue
            ms = timeit(fn, a.iters)
            print(f"ffn.dec M={M} splits={sp}: {ms * 1e3:.1f} us")
        # decsa.hip's decffn: (16 rows, 256 hidden) workgroups over packed weights, + the reduce
        f1 = _pack(L, w1)
        f2 = torch.cat([_pack(L, w2[:, c:c + 256].contiguous()) for c in range(0, F, 256)])
        fn = lambda: L.spe_debug_decffn(None, p(x), D, M, F, p(f1), 0, p(b1), p(f2), 0, p(b2), p(gm), p(bt), p(y),
                                        D, p(part))
        assert fn() == 0
        print(f"decffn M={M}: {timeit(fn, a.iters) * 1e3:.1f} us")
        # the cross-attention's folded query projection q' (2048 columns, row-periodic residual)
        wq = (torch.randn(8 * D, D, generator=g) / 16).to(dev, torch.bfloat16)
        rq = torch.randn(11, 8 * D, generator=g).to(dev, torch.bfloat16)
        yq = torch.empty(M, 8 * D, dtype=torch.bfloat16, device=dev)
        fq = _pack(L, wq)
        fn = lambda: L.spe_debug_decq(None, p(x), D, M, 8 * D, p(fq), 0, None, p(rq), 8 * D, 11, p(yq), 8 * D)
        assert fn() == 0
        print(f"decq M={M} N=2048: {timeit(fn, a.iters) * 1e3:.1f} us")
    if a.which in ("decsa", "all"):
        # the decoder's fused self-attention block (decsa.hip), B images of Q = 11 rows
        Q = 11
        t = torch.randn(B * Q, D, generator=g).to(dev, torch.bfloat16)
        wqk = (torch.randn(2 * D, D, generator=g) / 16).to(dev, torch.bfloat16)
        wv = (torch.randn(D, D, generator=g) / 16).to(dev, torch.bfloat16)
        wo = (torch.randn(D, D, generator=g) / 16).to(dev, torch.bfloat16)
        qpos = torch.zeros(Q, 2 * D, device=dev, dtype=torch.bfloat16)
        bqk, bv, bo, bt = (torch.zeros(n, device=dev) for n in (2 * D, D, D, D))
        gm = torch.ones(D, device=dev)
        pk = lambda w: _pack(L, w)                      # noqa: E731  (fragment-packed once, ld = 0)
        fqk, fv, fo = pk(wqk), pk(wv), pk(wo)
        fn = lambda: L.spe_debug_decsa(None, p(t), D, B, Q, p(fqk), 0, p(bqk), p(fv), 0, p(bv), p(qpos), p(fo), 0,
                                       p(bo), p(gm), p(bt), 32 ** -0.5)
        ms = timeit(fn, a.iters)
        print(f"decsa B={B} Q={Q}: {ms * 1e3:.1f} us")
    if a.which in ("xattn", "all"):
        Q = 11
        q = (torch.randn(B * Q, 8 * D, generator=g) / 16).to(dev, torch.bfloat16)
        k = torch.randn(B * T, D, generator=g).to(dev, torch.bfloat16)
        v = torch.randn(B * T, D, generator=g).to(dev, torch.bfloat16)
        wv = (torch.randn(D, D, generator=g) / 16).to(dev, torch.bfloat16)
        bv = torch.zeros(D, device=dev)
        u = torch.empty(B * Q, 8 * D, dtype=torch.bfloat16, device=dev)
        o = torch.empty(B * Q, D, dtype=torch.bfloat16, device=dev)
        part = torch.empty(256 * B * 8 * Q * 258, device=dev)
        for sp in (0, 2, 8):
            fn = lambda: L.spe_debug_xattn(None, p(q), 8 * D, p(k), D, p(v), D, None, 0, p(wv), p(bv), p(o), D,
                                           B, Q, T, sp, p(part))
            ms = timeit(fn, a.iters)
            fn_u = lambda: L.spe_debug_xattn(None, p(q), 8 * D, p(k), D, p(v), D, p(u), 8 * D, None, None, None,
                                             0, B, Q, T, sp, p(part))
            ms_u = timeit(fn_u, a.iters)
            byts = 2 * B * T * D * 2                      # K and V reads
            print(f"xattn splits={sp}: {ms:.3f} ms with Wv, {ms_u:.3f} ms u only ({byts / ms_u / 1e9:.2f} TB/s)")
        # the cross-attention's tail: separate merge + Wv kernel then decproj, against decxproj
        t = torch.randn(B * Q, D, generator=g).to(dev, torch.bfloat16)
        wo = (torch.randn(D, D, generator=g) / 16).to(dev, torch.bfloat16)
        bo, bt, gm = torch.zeros(D, device=dev), torch.zeros(D, device=dev), torch.ones(D, device=dev)
        L.spe_debug_xattn(None, p(q), 8 * D, p(k), D, p(v), D, p(u), 8 * D, None, None, None, 0, B, Q, T, 0, p(part))
        fwo, fwv = _pack(L, wo), _pack(L, wv)
        fn_dp = lambda: L.spe_debug_decproj(None, p(t), D, p(o), D, B, Q, p(fwo), 0, p(bo), p(gm), p(bt))
        fn_xp = lambda: L.spe_debug_decxproj(None, p(t), D, p(part), 0, T, B, Q, p(fwv), 0, p(bv), p(fwo), 0, p(bo),
                                             p(gm), p(bt))
        print(f"decproj B={B} Q={Q}: {timeit(fn_dp, a.iters) * 1e3:.1f} us; "
              f"decxproj (merge + Wv + Wo + LN): {timeit(fn_xp, a.iters) * 1e3:.1f} us")
    if a.which in ("gemm", "all"):
        # name, mode, M, N, K, residual rows (0 none, -1 full, >0 period), conv geometry
        cases = [("l1.c3 1x1+res", 0, B * 104 * 104, 256, 64, -1, None),
                 ("l1.c3 1x1 nores", 0, B * 104 * 104, 256, 64, 0, None),
                 ("l1.c3 N128+res", 0, B * 104 * 104, 128, 64, -1, None),
                 ("l1.c1 1x1", 0, B * 104 * 104, 64, 256, 0, None),
                 ("enc.qk +posW", 0, B * T, 512, 256, T, None),
                 ("cross_k +posW", 0, B * T, 1536, 256, T, None),
                 ("enc.o +res", 0, B * T, 256, 256, -1, None),
                 ("neck s16 3x3", 2, B * T, 256, 9 * 1024, 0, (52, 52, 1024, 3, 3, 1, 1)),
                 ("neck out 3x3", 2, B * T, 512, 9 * 512, 0, (52, 52, 512, 3, 3, 1, 1)),
                 ("l1 3x3", 2, B * 104 * 104, 64, 9 * 64, 0, (104, 104, 64, 3, 3, 1, 1)),
                 ("l2 3x3", 2, B * T, 128, 9 * 128, 0, (52, 52, 128, 3, 3, 1, 1)),
                 ("l3 3x3", 2, B * 676, 256, 9 * 256, 0, (26, 26, 256, 3, 3, 1, 1)),
                 ("l3.c3 1x1+res", 0, B * 676, 1024, 256, -1, None),
                 ("l3.c1 1x1", 0, B * 676, 256, 1024, 0, None),
                 ("l2.c3 1x1+res", 0, B * T, 512, 128, -1, None),
                 ("l2.c1 1x1", 0, B * T, 128, 512, 0, None),
                 ("sq8192 linear", 0, 8192, 8192, 8192, 0, None),
                 ("neck as linear", 0, B * T, 256, 9 * 1024, 0, None)]
        if a.only:
            cases = [c for c in cases if a.only in c[0]]
        for name, mode, M, N, K, rr, conv in cases:
            if conv:
                H, W, Cin, KH, KW, st, pd = conv
                A = torch.randn(B, H, W, Cin, generator=g).to(dev, torch.bfloat16)
            else:
                H = W = Cin = 0; KH = KW = st = 1; pd = 0
                A = torch.randn(M, K, generator=g).to(dev, torch.bfloat16)
            ldb = (K + 63) // 64 * 64
            Wt = (torch.randn(N, ldb, generator=g) / K ** 0.5).to(dev, torch.bfloat16)
            bias = torch.zeros(N, device=dev)
            R = None if rr == 0 else torch.randn(M if rr < 0 else rr, N, generator=g).to(dev, torch.bfloat16)
            C = torch.empty(M, N, dtype=torch.bfloat16, device=dev)
            rp = 0 if rr <= 0 else rr
            fn = lambda: L.spe_debug_gemm(None, 0, mode, p(A), K if not conv else 0, None, 0, 1, H, W, Cin, KH, KW,
                                          st, pd, p(Wt), ldb, M, N, K, p(bias), p(R) if R is not None else None,
                                          N, 1, p(C), N, 0, 0, 0, rp, None, None, 0)
            ms = timeit(fn, a.iters)
            abytes = (B * H * W * Cin if conv else M * K) * 2
            byts = abytes + N * ldb * 2 + M * N * 2 + (0 if R is None else R.numel() * 2)
            print(f"{name:16s} {ms:.3f} ms  {2.0 * M * N * K / ms / 1e9:7.1f} TF/s  {byts / ms / 1e9:6.2f} TB/s")
    if a.which in ("btail", "all"):
        # the fused layer-1 bottleneck tail (btail.hip): conv3 (+ identity) + relu and the next
        # conv1, the bench's three layer-1 shapes
        M = B * 104 * 104
        for k1, n2, res in ((64, 64, True), (64, 128, True), (128, 64, False)):
            A = torch.randn(M, k1, generator=g).to(dev, torch.bfloat16)
            R = torch.randn(M, 256, generator=g).to(dev, torch.bfloat16) if res else None
            W3 = (torch.randn(256, 64 * ((k1 + 63) // 64), generator=g) / k1 ** 0.5).to(dev, torch.bfloat16)
            W1 = (torch.randn(n2, 256, generator=g) / 16).to(dev, torch.bfloat16)
            b3, b1 = torch.zeros(256, device=dev), torch.zeros(n2, device=dev)
            Y = torch.empty(M, 256, dtype=torch.bfloat16, device=dev)
            Z = torch.empty(M, n2, dtype=torch.bfloat16, device=dev)
            fn = lambda: L.spe_debug_btail(None, p(A), k1, k1, p(R) if R is not None else None, p(W3), W3.shape[1], p(b3), p(Y), p(W1), 256, p(b1),
                                           p(Z), n2, M)
            ms = timeit(fn, a.iters)
            byts = M * (k1 + 256 + n2 + (256 if res else 0)) * 2
            print(f"btail k1={k1} n2={n2} res={int(res)}  {ms:.3f} ms  {byts / ms / 1e9:6.2f} TB/s")


if __name__ == "__main__":
    main()
