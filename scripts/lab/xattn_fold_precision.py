"""CPU study: how far the fp32h3 decoder cross-attention fold (xattn_h3.hip) sits from exact
arithmetic, next to the reference's own fp32 order.

Runs the torch restatement (oracle/model_ref.py) of config 2 on the bench fixture weights with the
decoder cross-attention replaced by one of:
  ref_fp32   the reference's order in fp32 (q = Wq x, k = Wk (m + p), softmax(q k^T) v, out_proj)
  ref_fp64   the same in fp64 (the "truth" every variant is measured against)
  fold_fp32  the fold (q' = Wk^T q per head against m + p, o = Wv (P m) + bv) in plain fp32
  fold_h3    the fold with xattn_h3.hip's arithmetic emulated: fp16 hi / lo splits of the scaled
             q' (per row and 128-dim half, 2^(13-e)), of (m + p) * 2^sk and m * 2^sv, three products
             per score / value term, P split as RTZ fp16 hi + RNE fp16 remainder
  fold_h3_rne  fold_h3 with the P split's hi rounded to nearest
and prints the max |pred_points - truth| over the foreground queries for each.  Everything else
runs in fp32 as the reference does.  Usage: python scripts/lab/xattn_fold_precision.py [n_images]
"""
import math
import os
import sys

import numpy as np
import torch
import torch.nn.functional as F

REPO = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path.insert(0, os.path.join(REPO, "oracle"))
sys.path.insert(0, os.path.join(REPO, "satellite-pose-estimation_amd"))
import model_ref  # noqa: E402
from spe.config import SpeConfig  # noqa: E402
from spe.synthetic import bench_images, fixed_bench_weights  # noqa: E402


def split16(x):
    """fp16 hi = RNE(x), lo = RNE(x - hi), returned as float64."""
    hi = x.to(torch.float16)
    lo = (x - hi.to(torch.float32)).to(torch.float16)
    return hi.double(), lo.double()


def pow2_scale(bound, top):
    e = math.frexp(float(bound))[1]
    return 2.0 ** (top - e)


def rtz16(x):
    """fp32 -> fp16 rounded toward zero (v_cvt_pkrtz_f16_f32): RNE, then one step back where it
    rounded away from zero."""
    h = x.to(torch.float16)
    over = (h.to(torch.float32).abs() > x.abs()) & (h != 0)
    return torch.where(over, (h.view(torch.int16) - 1).view(torch.float16), h)


def make_mha(mode, mem_bound):
    def mha(q_in, k_in, v_in, sd, p, nheads):
        W, bvec = sd[p + ".in_proj_weight"], sd[p + ".in_proj_bias"]
        d = W.shape[1]
        hd = d // nheads
        Wo, bo = sd[p + ".out_proj.weight"], sd[p + ".out_proj.bias"]
        B, Lq, _ = q_in.shape
        Lk = k_in.shape[1]
        if mode in ("ref_fp32", "ref_fp64"):
            dt = torch.float64 if mode == "ref_fp64" else torch.float32
            qi, ki, vi = q_in.to(dt), k_in.to(dt), v_in.to(dt)
            Wd, bd = W.to(dt), bvec.to(dt)
            q = F.linear(qi, Wd[:d], bd[:d]).view(B, Lq, nheads, hd).transpose(1, 2) * (hd ** -0.5)
            k = F.linear(ki, Wd[d:2 * d], bd[d:2 * d]).view(B, Lk, nheads, hd).transpose(1, 2)
            v = F.linear(vi, Wd[2 * d:], bd[2 * d:]).view(B, Lk, nheads, hd).transpose(1, 2)
            a = torch.softmax(q @ k.transpose(-1, -2), dim=-1) @ v
            a = a.transpose(1, 2).reshape(B, Lq, d)
            return F.linear(a, Wo.to(dt), bo.to(dt)).float()
        # the fold (registry.cpp fold_cross_attention): Wqk in double, stored fp32, exp2 domain
        W64, b64 = W.double(), bvec.double()
        sc = hd ** -0.5 * 1.4426950408889634
        Wq, Wk, Wv = W64[:d], W64[d:2 * d], W64[2 * d:]
        wqk = torch.stack([sc * Wk[h * hd:(h + 1) * hd].T @ Wq[h * hd:(h + 1) * hd] for h in range(nheads)])   # [H, d(n), d(k)]
        bqk = torch.stack([sc * Wk[h * hd:(h + 1) * hd].T @ b64[h * hd:(h + 1) * hd] for h in range(nheads)])  # [H, d]
        wqk, bqk = wqk.float(), bqk.float()
        qp = torch.einsum("bqk,hnk->bqhn", q_in, wqk) + bqk[None, None]       # [B, Q, H, d] fp32
        mem, kin = v_in, k_in                                                    # memory, memory + pos
        if mode == "fold_fp32":
            s = torch.einsum("bqhn,btn->bhqt", qp, kin)
            pm = torch.exp2(s - s.amax(-1, keepdim=True))
            u = torch.einsum("bhqt,btn->bhqn", pm, mem) / pm.sum(-1, keepdim=True)
        else:
            sk = pow2_scale(mem_bound + 1.0, 14)
            sv = pow2_scale(mem_bound, 14)
            kh, kl = split16(kin * sk)
            vh, vl = split16(mem * sv)
            qp2 = qp.view(B, Lq, nheads, 2, d // 2)
            am = qp2.abs().amax(-1, keepdim=True).clamp_min(1e-30)
            e = torch.floor(torch.log2(am)) + 1                                     # am in [2^(e-1), 2^e)
            sq = torch.exp2(13 - e)
            qh, ql = split16((qp2 * sq).view(B, Lq, nheads, d))
            inv = (1.0 / (sq * sk)).double()
            s = torch.zeros(B, nheads, Lq, Lk, dtype=torch.float64)
            for half in range(2):
                sl = slice(half * 128, half * 128 + 128)
                part = (torch.einsum("bqhn,btn->bhqt", qh[..., sl], kl[..., sl]) +
                        torch.einsum("bqhn,btn->bhqt", ql[..., sl], kh[..., sl]) +
                        torch.einsum("bqhn,btn->bhqt", qh[..., sl], kh[..., sl]))
                part = part.float().double() * inv[:, :, :, half, 0].permute(0, 2, 1)[..., None]
                s = s + part.float().double()
            s = s.float()
            pm = torch.exp2(s - s.amax(-1, keepdim=True))                          # fp32 p
            ph = rtz16(pm) if mode == "fold_h3" else pm.to(torch.float16)
            pl = (pm - ph.float()).to(torch.float16)
            ph, pl = ph.double(), pl.double()
            u = (torch.einsum("bhqt,btn->bhqn", ph, vl) + torch.einsum("bhqt,btn->bhqn", pl, vh) +
                 torch.einsum("bhqt,btn->bhqn", ph, vh)).float() / sv
            u = u / pm.sum(-1, keepdim=True)
        # o_h = Wv_h u_h + bv_h (fp32), then the out-projection
        Wvf, bvf = W[2 * d:], bvec[2 * d:]
        o = torch.stack([u[:, h] @ Wvf[h * hd:(h + 1) * hd].T + bvf[h * hd:(h + 1) * hd] for h in range(nheads)], 2)
        o = o.reshape(B, Lq, d)
        return F.linear(o, Wo, bo)
    return mha


def main():
    n = int(sys.argv[1]) if len(sys.argv) > 1 else 4
    torch.set_num_threads(min(16, os.cpu_count() or 1))
    cfg = SpeConfig(input_size=416, num_queries=11, enc_layers=6, dec_layers=6)
    w, _ = fixed_bench_weights(cfg, 0)
    data = bench_images(cfg, 0, n)
    sd = {k: torch.as_tensor(v, dtype=torch.float32) for k, v in w.items()}
    # the memory's LayerNorm bound (registry.cpp ln_bound: |gamma| * sqrt(d - 1) + |beta|)
    p = f"transformer.encoder.layers.{cfg.enc_layers - 1}.norm2"
    mem_bound = float(sd[p + ".weight"].abs().max() * math.sqrt(cfg.hidden_dim - 1) + sd[p + ".bias"].abs().max())
    orig = model_ref._mha
    res = {}
    for mode in ("ref_fp64", "ref_fp32", "fold_fp32", "fold_h3", "fold_h3_rne"):
        cross = make_mha(mode, mem_bound)

        def mha(q_in, k_in, v_in, sd_, p_, nh, _cross=cross):
            if p_.endswith("multihead_attn"):
                return _cross(q_in, k_in, v_in, sd_, p_, nh)
            return orig(q_in, k_in, v_in, sd_, p_, nh)
        model_ref._mha = mha
        with torch.no_grad():
            res[mode] = model_ref.forward(data["images"], w, cfg)
        model_ref._mha = orig
        print(mode, "done", flush=True)
    truth = res["ref_fp64"]
    fg = truth["pred_logits"].argmax(-1) < 11
    for mode in ("ref_fp32", "fold_fp32", "fold_h3", "fold_h3_rne"):
        d = (res[mode]["pred_points"] - truth["pred_points"]).abs().amax(-1)[fg]
        h = (res[mode]["hs"] - truth["hs"]).norm(dim=-1) / truth["hs"].norm(dim=-1)
        print(f"{mode:10s} kpt max {float(d.max()):.3e} mean {float(d.mean()):.3e}  hs rel mean {float(h.mean()):.3e}")


if __name__ == "__main__":
    main()
