// Native runtime of the keypoint-set predictor, part 1: parameter registry in the
// reference's state_dict key space (REV/models/detr_speed.py:296-336 -> 412 keys), FrozenBN
// folding (REV/models/backbone.py:44-54), weight packing ([N][KH][KW][Cin] rows, bf16/fp32),
// workspace planning.  The launch sequence lives in forward.cpp.
#include <hip/hip_runtime.h>

#include <algorithm>
#include <cmath>
#include <cstdlib>
#include <cstdio>
#include <cstring>

#include "model_state.h"
#include "registry.h"

namespace {
thread_local std::string g_err;
}  // namespace

uint16_t f2bf(float f) {
  uint32_t u;
  std::memcpy(&u, &f, 4);
  if ((u & 0x7fffffffu) > 0x7f800000u) return (uint16_t)((u >> 16) | 0x40);  // quiet NaN
  u += 0x7fffu + ((u >> 16) & 1u);
  return (uint16_t)(u >> 16);
}

int spe_fail(int code, const std::string& msg) {
  g_err = msg;
  return code;
}
#define fail spe_fail

namespace {

std::vector<std::pair<std::string, std::vector<int64_t>>> build_spec(const spe_model_config& c) {
  std::vector<std::pair<std::string, std::vector<int64_t>>> s;
  const int64_t d = c.hidden_dim, ff = c.dim_feedforward;
  auto add = [&](const std::string& k, std::vector<int64_t> sh) { s.emplace_back(k, std::move(sh)); };
  auto bn = [&](const std::string& p, int64_t ch) {
    for (const char* n : {"weight", "bias", "running_mean", "running_var"}) add(p + "." + n, {ch});
  };
  for (int i = 0; i < c.enc_layers; ++i) {
    std::string p = "transformer.encoder.layers." + std::to_string(i);
    add(p + ".self_attn.in_proj_weight", {3 * d, d}); add(p + ".self_attn.in_proj_bias", {3 * d});
    add(p + ".self_attn.out_proj.weight", {d, d}); add(p + ".self_attn.out_proj.bias", {d});
    add(p + ".linear1.weight", {ff, d}); add(p + ".linear1.bias", {ff});
    add(p + ".linear2.weight", {d, ff}); add(p + ".linear2.bias", {d});
    for (const char* n : {"norm1", "norm2"}) { add(p + "." + n + ".weight", {d}); add(p + "." + n + ".bias", {d}); }
  }
  for (int i = 0; i < c.dec_layers; ++i) {
    std::string p = "transformer.decoder.layers." + std::to_string(i);
    for (const char* a : {"self_attn", "multihead_attn"}) {
      add(p + "." + a + ".in_proj_weight", {3 * d, d}); add(p + "." + a + ".in_proj_bias", {3 * d});
      add(p + "." + a + ".out_proj.weight", {d, d}); add(p + "." + a + ".out_proj.bias", {d});
    }
    add(p + ".linear1.weight", {ff, d}); add(p + ".linear1.bias", {ff});
    add(p + ".linear2.weight", {d, ff}); add(p + ".linear2.bias", {d});
    for (const char* n : {"norm1", "norm2", "norm3"}) { add(p + "." + n + ".weight", {d}); add(p + "." + n + ".bias", {d}); }
  }
  add("transformer.decoder.norm.weight", {d}); add("transformer.decoder.norm.bias", {d});
  add("cls_embed.weight", {12, d}); add("cls_embed.bias", {12});
  add("point_embed.layers.0.weight", {d, d}); add("point_embed.layers.0.bias", {d});
  add("point_embed.layers.1.weight", {d, d}); add("point_embed.layers.1.bias", {d});
  add("point_embed.layers.2.weight", {2, d}); add("point_embed.layers.2.bias", {2});
  add("query_embed.weight", {c.num_queries, d});
  add("input_proj.weight", {d, 512, 1, 1}); add("input_proj.bias", {d});
  const std::string b = "backbone.0.body";
  add(b + ".conv1.weight", {64, 3, 7, 7});
  bn(b + ".bn1", 64);
  int64_t cin = 64;
  const int widths[3] = {64, 128, 256}, nblk[3] = {3, 4, 6};
  for (int li = 0; li < 3; ++li)
    for (int k = 0; k < nblk[li]; ++k) {
      const int64_t w = widths[li];
      std::string p = b + ".layer" + std::to_string(li + 1) + "." + std::to_string(k);
      add(p + ".conv1.weight", {w, cin, 1, 1}); bn(p + ".bn1", w);
      add(p + ".conv2.weight", {w, w, 3, 3}); bn(p + ".bn2", w);
      add(p + ".conv3.weight", {4 * w, w, 1, 1}); bn(p + ".bn3", 4 * w);
      if (k == 0) { add(p + ".downsample.0.weight", {4 * w, cin, 1, 1}); bn(p + ".downsample.1", 4 * w); }
      cin = 4 * w;
    }
  add("backbone.0.s8_latern.weight", {256, 512, 1, 1});
  add("backbone.0.s16_latern.weight", {256, 1024, 3, 3});
  add("backbone.0.output_conv.weight", {512, 512, 3, 3});
  add("backbone.0.output_conv.bias", {512});
  if (c.sigma_head) {
    add("sigma_embed.layers.0.weight", {d, d}); add("sigma_embed.layers.0.bias", {d});
    add("sigma_embed.layers.1.weight", {d, d}); add("sigma_embed.layers.1.bias", {d});
    add("sigma_embed.layers.2.weight", {1, d}); add("sigma_embed.layers.2.bias", {1});
  }
  return s;
}

}  // namespace

// ---- packing helpers shared with the RT-DETR runtime (registry.h)
void* dalloc(spe_model* m, size_t bytes) {
  size_t off = (m->dused + 255) & ~size_t(255);
  m->dused = off + bytes;
  return m->dmem ? (void*)(m->dmem + off) : nullptr;
}

// bf16 bits -> the float they represent
static float bf2f(uint16_t b) {
  const uint32_t u = (uint32_t)b << 16;
  float f;
  std::memcpy(&f, &u, 4);
  return f;
}

// pack host fp32 [N][K] rows (already in K order) into device T [N][Kpad]; fp32x6 models also
// get the rows' three-way bf16 split x = hi + mid + lo (RNE each, remainders exact in fp32) as
// planes [3][N][Kpad] right after them, registered in m->w6 for the x6 GEMM
void* upload_rows(spe_model* m, const std::vector<float>& rows, int N, int K, int Kpad) {
  const size_t n = (size_t)N * Kpad;
  void* dst = dalloc(m, n * m->esz);
  void* pl = (m->x6 && m->esz == 4) ? dalloc(m, 3 * n * 2) : nullptr;   // sized in both passes
  void* ph = (m->h3 && m->esz == 4) ? dalloc(m, 2 * n * 2) : nullptr;
  float* sinv = (m->h3 && m->esz == 4) ? (float*)dalloc(m, (size_t)N * 4) : nullptr;
  if (!m->dmem) return nullptr;
  if (m->esz == 2) {
    std::vector<uint16_t> h(n, 0);
    for (int r = 0; r < N; ++r)
      for (int k = 0; k < K; ++k) h[(size_t)r * Kpad + k] = f2bf(rows[(size_t)r * K + k]);
    m->upload_err |= (int)hipMemcpy(dst, h.data(), h.size() * 2, hipMemcpyHostToDevice);
  } else {
    std::vector<float> h(n, 0.f);
    for (int r = 0; r < N; ++r) std::memcpy(&h[(size_t)r * Kpad], &rows[(size_t)r * K], (size_t)K * 4);
    m->upload_err |= (int)hipMemcpy(dst, h.data(), h.size() * 4, hipMemcpyHostToDevice);
    if (pl) {
      std::vector<uint16_t> b(3 * n);
      for (size_t i = 0; i < n; ++i) {
        const uint16_t hi = f2bf(h[i]);
        const float r = h[i] - bf2f(hi);
        const uint16_t mid = f2bf(r);
        b[i] = hi;
        b[n + i] = mid;
        b[2 * n + i] = f2bf(r - bf2f(mid));
      }
      m->upload_err |= (int)hipMemcpy(pl, b.data(), b.size() * 2, hipMemcpyHostToDevice);
      m->w6[dst] = {pl, N};
    }
    if (ph) {
      // fp32h3: row r scaled by 2^e_r (max |w_r| 2^e_r in [2^12, 2^13)), split into fp16 hi = RNE(x),
      // lo = RNE(x - hi) (x - hi exact in fp32); 2^-e_r undoes the scale in the GEMM epilogue
      std::vector<_Float16> b(2 * n, (_Float16)0.f);
      std::vector<float> si(N, 1.f);
      for (int r = 0; r < N; ++r) {
        float am = 0.f;
        for (int k = 0; k < K; ++k) am = std::max(am, std::fabs(h[(size_t)r * Kpad + k]));
        int ex = 0;
        if (am > 0.f && std::isfinite(am)) std::frexp(am, &ex);
        const float sc = am > 0.f ? std::ldexp(1.f, 13 - ex) : 1.f;
        si[r] = am > 0.f ? std::ldexp(1.f, ex - 13) : 1.f;
        for (int k = 0; k < K; ++k) {
          const size_t i = (size_t)r * Kpad + k;
          const float x = h[i] * sc;
          const _Float16 hi = (_Float16)x;
          b[i] = hi;
          b[n + i] = (_Float16)(x - (float)hi);
        }
      }
      m->upload_err |= (int)hipMemcpy(ph, b.data(), b.size() * 2, hipMemcpyHostToDevice);
      m->upload_err |= (int)hipMemcpy(sinv, si.data(), si.size() * 4, hipMemcpyHostToDevice);
      m->wh3[dst] = {ph, N, sinv};
    }
  }
  return dst;
}

float* upload_f32(spe_model* m, const float* p, size_t n) {
  float* dst = (float*)dalloc(m, n * 4);
  if (m->dmem) m->upload_err |= (int)hipMemcpy(dst, p, n * 4, hipMemcpyHostToDevice);
  return dst;
}

// fp32h3, the one-pass encoder FFN (ffn_h3.hip): e.ffn_meta1 = (2^-e1, b1) per 32-unit hidden chunk
// (e1 as upload_rows scales linear1's rows), e.ffn_w2p = linear2's fp16 planes with each chunk's
// columns in spe_ffn_h3_perm order (rows scaled as upload_rows does: the same 2^-e2 as e.l2's planes),
// e.ffn_sh = 2^(13 - e) for the bound B on |ReLU(x W1^T + b1)| in [2^(e-1), 2^e): B = max_j |b1_j| +
// ||W1_j||_2 (max|gamma1| sqrt(D) + ||beta1||_2), ||x||_2 of a LayerNorm output never exceeding the
// latter (sum of the normalised squares = D var / (var + eps) <= D)
static void ffn_h3_prepare(spe_model* m, Enc& e, const std::string& p, int d, int ff) {
  if (!m->h3 || d != 256 || ff % 32 || ff % 8) return;
  const size_t n2 = (size_t)d * ff;
  e.ffn_meta1 = (float*)dalloc(m, (size_t)ff * 2 * 4);
  e.ffn_w2p = dalloc(m, 2 * n2 * 2);
  if (!m->dmem) return;
  const auto& w1 = m->host[p + ".linear1.weight"];
  const auto& b1 = m->host[p + ".linear1.bias"];
  const auto& w2 = m->host[p + ".linear2.weight"];
  const auto& g1 = m->host[p + ".norm1.weight"];
  const auto& be1 = m->host[p + ".norm1.bias"];
  double gmax = 0.0, bn = 0.0;
  for (float v : g1) gmax = std::max(gmax, (double)std::fabs(v));
  for (float v : be1) bn += (double)v * v;
  const double rx = gmax * std::sqrt((double)d) + std::sqrt(bn);
  std::vector<float> meta((size_t)ff * 2);
  double bound = 0.0;
  for (int j = 0; j < ff; ++j) {
    float am = 0.f;
    double nn = 0.0;
    for (int k = 0; k < d; ++k) {
      const float v = w1[(size_t)j * d + k];
      am = std::max(am, std::fabs(v));
      nn += (double)v * v;
    }
    int ex = 0;
    if (am > 0.f && std::isfinite(am)) std::frexp(am, &ex);
    const int c = j / 32, u = j % 32;
    meta[(size_t)c * 64 + u] = am > 0.f ? std::ldexp(1.f, ex - 13) : 1.f;
    meta[(size_t)c * 64 + 32 + u] = b1[j];
    bound = std::max(bound, std::fabs((double)b1[j]) + std::sqrt(nn) * rx);
  }
  int eb = 0;
  std::frexp(bound > 0.0 ? bound * (1.0 + 1e-6) : 1.0, &eb);
  e.ffn_sh = std::ldexp(1.f, 13 - eb);
  std::vector<_Float16> planes(2 * n2);
  for (int n = 0; n < d; ++n) {
    float am = 0.f;
    for (int k = 0; k < ff; ++k) am = std::max(am, std::fabs(w2[(size_t)n * ff + k]));
    int ex = 0;
    if (am > 0.f && std::isfinite(am)) std::frexp(am, &ex);
    const float sc = am > 0.f ? std::ldexp(1.f, 13 - ex) : 1.f;
    for (int k = 0; k < ff; ++k) {
      const int src = (k / 32) * 32 + spe_ffn_h3_perm(k % 32);
      const float x = w2[(size_t)n * ff + src] * sc;
      const _Float16 hi = (_Float16)x;
      planes[(size_t)n * ff + k] = hi;
      planes[n2 + (size_t)n * ff + k] = (_Float16)(x - (float)hi);
    }
  }
  m->upload_err |= (int)hipMemcpy(e.ffn_meta1, meta.data(), meta.size() * 4, hipMemcpyHostToDevice);
  m->upload_err |= (int)hipMemcpy(e.ffn_w2p, planes.data(), planes.size() * 2, hipMemcpyHostToDevice);
}

// fp32h3: a device bound on |LayerNorm `key` output| of width D: max|gamma| sqrt(D - 1) + max|beta|
// (|x_i - mean| / std <= sqrt(D - 1) for any row) -- the scale input of the GEMMs reading it
float* ln_bound(spe_model* m, const std::string& key, int D) {
  float g = 0.f, b = 0.f;
  if (m->dmem) {
    for (float v : m->host[key + ".weight"]) g = std::max(g, std::fabs(v));
    for (float v : m->host[key + ".bias"]) b = std::max(b, std::fabs(v));
  }
  const float v = g * std::sqrt((float)(D - 1)) + b;
  return upload_f32(m, &v, 1);
}

void* upload_T(spe_model* m, const std::vector<float>& v) {
  void* dst = dalloc(m, v.size() * m->esz);
  if (!m->dmem) return nullptr;
  if (m->esz == 2) {
    std::vector<uint16_t> h(v.size());
    for (size_t i = 0; i < v.size(); ++i) h[i] = f2bf(v[i]);
    m->upload_err |= (int)hipMemcpy(dst, h.data(), h.size() * 2, hipMemcpyHostToDevice);
  } else {
    m->upload_err |= (int)hipMemcpy(dst, v.data(), v.size() * 4, hipMemcpyHostToDevice);
  }
  return dst;
}

int pad64(int k) { return (k + 63) / 64 * 64; }

// folded conv weight [cout][cin][kh][kw] (host fp32) -> [Cout][KH][KW][Cin_pad] rows in the
// kernels' K order (spe_kernels.h conv_k_decode), bias fp32
Conv pack_conv(spe_model* m, const std::vector<float>& w, const std::vector<float>& bias, int cout, int cin, int kh,
               int kw, int cin_pad, int stride, int pad) {
  const int cp = cin_pad > 0 ? cin_pad : cin;
  const int K = kh * kw * cp;
  std::vector<float> rows((size_t)cout * K, 0.f);
  const bool cblk = conv_channel_blocked(cp, kh * kw);
  if (m->dmem)                                     // pass 1 only sizes the device block
    for (int co = 0; co < cout; ++co)
      for (int ci = 0; ci < cin; ++ci)
        for (int y = 0; y < kh; ++y)
          for (int x = 0; x < kw; ++x) {
            const int tap = y * kw + x;
            const int k = cblk ? ((ci / 64) * kh * kw + tap) * 64 + ci % 64 : tap * cp + ci;
            rows[(size_t)co * K + k] = w[(((size_t)co * cin + ci) * kh + y) * kw + x];
          }
  Conv c;
  c.N = cout; c.K = K; c.Kpad = pad64(K); c.Cin = cp; c.KH = kh; c.KW = kw; c.stride = stride; c.pad = pad;
  c.w = upload_rows(m, rows, c.N, c.K, c.Kpad);
  c.bias = upload_f32(m, bias.data(), bias.size());
  return c;
}

std::vector<int64_t> param_shape(const spe_model* m, const std::string& key) {
  for (auto& s : m->spec)
    if (s.first == key) return s.second;
  return {};
}

// conv weight `wkey` [cout][cin][kh][kw] with an eval BatchNorm `bnkey` (weight, bias,
// running_mean, running_var; eps 1e-5) and/or a conv bias folded in (double arithmetic)
void fold_conv(spe_model* m, const std::string& wkey, const std::string& bnkey, const std::string& biaskey,
               std::vector<float>& w, std::vector<float>& bias) {
  const auto sh = param_shape(m, wkey);
  const int64_t cout = sh[0], per = sh[1] * sh[2] * sh[3];
  const auto& src = m->host[wkey];
  std::vector<double> scale(cout, 1.0), shift(cout, 0.0);
  if (!bnkey.empty()) {
    const auto& g = m->host[bnkey + ".weight"];
    const auto& b = m->host[bnkey + ".bias"];
    const auto& rm = m->host[bnkey + ".running_mean"];
    const auto& rv = m->host[bnkey + ".running_var"];
    for (int64_t c = 0; c < cout; ++c) {
      scale[c] = (double)g[c] / std::sqrt((double)rv[c] + 1e-5);
      shift[c] = (double)b[c] - (double)rm[c] * scale[c];
    }
  }
  if (!biaskey.empty()) {
    const auto& bb = m->host[biaskey];
    for (int64_t c = 0; c < cout; ++c) shift[c] += bb[c];
  }
  w.assign((size_t)cout * per, 0.f);
  if (!src.empty())
    for (int64_t co = 0; co < cout; ++co)
      for (int64_t i = 0; i < per; ++i) w[co * per + i] = (float)(src[co * per + i] * scale[co]);
  bias.assign(shift.begin(), shift.end());
}

// conv weight [Cout][Cin][KH][KW] (+FrozenBN) -> [Cout][KH][KW][Cin_pad] rows, folded bias
Conv make_conv(spe_model* m, const std::string& wkey, const std::string& bnkey, const std::string& biaskey, int cin_pad,
               int stride, int pad) {
  const auto sh = param_shape(m, wkey);
  std::vector<float> w, bias;
  fold_conv(m, wkey, bnkey, biaskey, w, bias);
  return pack_conv(m, w, bias, (int)sh[0], (int)sh[1], (int)sh[2], (int)sh[3], cin_pad, stride, pad);
}

// linear rows [r0, r0+n) of a [*, K] weight + bias slice
Conv make_linear(spe_model* m, const std::string& wkey, const std::string& bkey, int r0, int n, int K) {
  const auto& w = m->host[wkey];
  std::vector<float> rows(w.begin() + (size_t)r0 * K, w.begin() + (size_t)(r0 + n) * K);
  Conv c;
  c.N = n; c.K = K; c.Kpad = pad64(K); c.Cin = K;
  c.w = upload_rows(m, rows, n, K, c.Kpad);
  const auto& b = m->host[bkey];
  c.bias = upload_f32(m, b.data() + r0, n);
  for (int r = 0; r < n; ++r) {
    double s = 0.0;
    for (int k = 0; k < K; ++k) s += std::fabs(rows[(size_t)r * K + k]);
    c.l1max = std::max(c.l1max, (float)(s * (1.0 + 1e-6)));     // (rounded up past the fp32 sum's error)
    c.bmax = std::max(c.bmax, std::fabs(b[r0 + r]));
  }
  return c;
}

float* upload_key(spe_model* m, const std::string& k) {
  const auto& v = m->host[k];
  return upload_f32(m, v.data(), v.size());
}

float* upload_transposed(spe_model* m, const std::string& k, int out, int in) {
  const auto& v = m->host[k];
  std::vector<float> t((size_t)in * out);
  for (int o = 0; o < out; ++o)
    for (int i = 0; i < in; ++i) t[(size_t)i * out + o] = v[(size_t)o * in + i];
  return upload_f32(m, t.data(), t.size());
}

bool spe_use_neckfold(const spe_model* m) {
  static const int on = [] { const char* e = getenv("SPE_NECK_FOLD"); return e ? atoi(e) : 1; }();
  return on && (m->cfg.dtype == SPE_DTYPE_BF16_ || m->x3);
}

namespace {

// sine position table for an all-valid mask (REV/models/position_encoding.py:30-53),
// [h*w][256] in token order h*W + w
std::vector<float> sine_pos(int h, int w, int d) {
  const int npf = d / 2;
  const float eps = 1e-6f, scale = 6.283185307179586f;
  std::vector<float> out((size_t)h * w * d);
  std::vector<float> dim_t(npf);
  for (int i = 0; i < npf; ++i) dim_t[i] = std::pow(10000.0f, (float)(2 * (i / 2)) / (float)npf);
  for (int y = 0; y < h; ++y)
    for (int x = 0; x < w; ++x) {
      const float ye = (float)(y + 1) / ((float)h + eps) * scale;
      const float xe = (float)(x + 1) / ((float)w + eps) * scale;
      float* o = &out[((size_t)y * w + x) * d];
      for (int i = 0; i < npf; ++i) {
        const float py = ye / dim_t[i], px = xe / dim_t[i];
        o[i] = (i & 1) ? std::cos(py) : std::sin(py);
        o[npf + i] = (i & 1) ? std::cos(px) : std::sin(px);
      }
    }
  return out;
}

// Cross-attention of decoder layer p folded for xattn.hip (header there).  Per head h
// (hd = 32 dims, s = softmax scale * log2 e):
//   Wqk[h*256 + n][k] = s * sum_i Wk[h*32+i][n] Wq[h*32+i][k]     (q' = x . Wqk^T + bqk)
//   bqk[h*256 + n]    = s * sum_i bq[h*32+i] Wk[h*32+i][n]         (bk drops out of the softmax)
//   xq_r[q][j]        = query_pos[q] . Wqk[j] + bqk[j]             (the `+ query_pos` of the query)
// Sums in double, stored bf16 (the reference's fp32 chain differs by the usual bf16 rounding).
// Wv (+bv) stays a plain [256][256] matrix: it is applied per row after the weighted sum.
void fold_cross_attention(spe_model* m, const std::string& p, Dec& e) {
  const auto& c = m->cfg;
  const int d = c.hidden_dim, H = c.nheads, hd = d / H, Q = c.num_queries, HD = H * d;
  std::vector<float> wqk((size_t)HD * d, 0.f), rqk((size_t)Q * HD, 0.f);
  if (m->dmem) {                                   // pass 2 only: pass 1 just sizes the block
    const auto& W = m->host[p + ".multihead_attn.in_proj_weight"];
    const auto& Bi = m->host[p + ".multihead_attn.in_proj_bias"];
    const auto& qe = m->host["query_embed.weight"];
    const double sc = 1.0 / std::sqrt((double)hd) * 1.4426950408889634;
    std::vector<double> acc((size_t)d), bqk((size_t)HD, 0.0);
    for (int h = 0; h < H; ++h)
      for (int n = 0; n < d; ++n) {
        std::fill(acc.begin(), acc.end(), 0.0);
        double bsum = 0.0;
        for (int i = 0; i < hd; ++i) {
          const double wk = W[(size_t)(d + h * hd + i) * d + n];
          const float* wq = &W[(size_t)(h * hd + i) * d];
          for (int k = 0; k < d; ++k) acc[k] += wk * wq[k];
          bsum += wk * Bi[h * hd + i];
        }
        float* dst = &wqk[((size_t)h * d + n) * d];
        for (int k = 0; k < d; ++k) dst[k] = (float)(acc[k] * sc);
        bqk[(size_t)h * d + n] = bsum * sc;
      }
    for (int q = 0; q < Q; ++q)
      for (int j = 0; j < HD; ++j) {
        double sum = bqk[j];
        const float* wr = &wqk[(size_t)j * d];
        for (int k = 0; k < d; ++k) sum += (double)qe[(size_t)q * d + k] * wr[k];
        rqk[(size_t)q * HD + j] = (float)sum;
      }
  }
  e.xq.N = HD; e.xq.K = d; e.xq.Kpad = pad64(d); e.xq.Cin = d;
  e.xq.w = upload_rows(m, wqk, HD, d, e.xq.Kpad);
  e.xq.bias = nullptr;
  e.xq_r = upload_T(m, rqk);
  e.xv = make_linear(m, p + ".multihead_attn.in_proj_weight", p + ".multihead_attn.in_proj_bias", 2 * d, d, d);
}

int build_device(spe_model* m) {
  const auto& c = m->cfg;
  const int d = c.hidden_dim, ff = c.dim_feedforward, Q = c.num_queries;
  const std::string b = "backbone.0.body";
  static const int stem_pairs = [] { const char* e = getenv("SPE_STEM_PAIRS"); return e ? atoi(e) : 1; }();
  if (m->esz == 2 && stem_pairs) {
    // bf16: the pair-packed stem (SPE_STEM_PAIRS=0: the 8-channel tap-major stem, A/B knob).  The 7x7/s2/p3 conv over 3 channels runs as a 7x8/s2 conv
    // over the zero-bordered 4-channel input (spe_launch_pack_input_pad4): k = (kh*8 + kw)*4 + ci,
    // kw = 7 and ci = 3 have zero weights, K = 224 (4 K-steps) instead of 7*7*8 = 392 (7 K-steps),
    // and each 16-byte chunk is the taps kw, kw+1 of one row.
    std::vector<float> w, bias;
    fold_conv(m, b + ".conv1.weight", b + ".bn1", "", w, bias);
    constexpr int KH = 7, KW = 8, CI = 4, K = KH * KW * CI;
    std::vector<float> rows((size_t)64 * K, 0.f);
    if (m->dmem)
      for (int co = 0; co < 64; ++co)
        for (int ci = 0; ci < 3; ++ci)
          for (int y = 0; y < 7; ++y)
            for (int x = 0; x < 7; ++x)
              rows[(size_t)co * K + (y * KW + x) * CI + ci] = w[(((size_t)co * 3 + ci) * 7 + y) * 7 + x];
    Conv c;
    c.N = 64; c.K = K; c.Kpad = pad64(K); c.Cin = CI; c.KH = KH; c.KW = KW; c.stride = 2; c.pad = 0;
    c.w = upload_rows(m, rows, c.N, c.K, c.Kpad);
    c.bias = upload_f32(m, bias.data(), bias.size());
    m->stem = c;
  } else {
    // fp32 models: 3 channels padded to 4 (K = 7*7*4 = 196: half the 8-channel form's products; the
    // 16-byte chunk is one pixel); bf16 with SPE_STEM_PAIRS=0: 8 channels (a 16-byte bf16 chunk)
    m->stem = make_conv(m, b + ".conv1.weight", b + ".bn1", "", m->esz == 4 ? 4 : 8, 2, 3);
  }
  m->blocks.clear();
  const int nblk[3] = {3, 4, 6};
  for (int li = 0; li < 3; ++li)
    for (int k = 0; k < nblk[li]; ++k) {
      std::string p = b + ".layer" + std::to_string(li + 1) + "." + std::to_string(k);
      Block blk;
      blk.stride = (k == 0 && li > 0) ? 2 : 1;
      blk.c1 = make_conv(m, p + ".conv1.weight", p + ".bn1", "", 0, 1, 0);
      blk.c2 = make_conv(m, p + ".conv2.weight", p + ".bn2", "", 0, blk.stride, 1);
      blk.c3 = make_conv(m, p + ".conv3.weight", p + ".bn3", "", 0, 1, 0);
      if (k == 0) {
        blk.has_ds = true;
        blk.ds = make_conv(m, p + ".downsample.0.weight", p + ".downsample.1", "", 0, blk.stride, 0);
        if (blk.stride == 1 && m->esz == 2) {
          // conv3 + downsample of a stride-1 first block as ONE K = w + cin GEMM over the
          // channel concatenation [conv2 output | block input] (forward.cpp lays them out side by
          // side): relu(W3 t2 + b3 + Wds x + bds) with no downsample output round trip
          std::vector<float> w3, b3, wd, bd;
          fold_conv(m, p + ".conv3.weight", p + ".bn3", "", w3, b3);
          fold_conv(m, p + ".downsample.0.weight", p + ".downsample.1", "", wd, bd);
          const int n = blk.c3.N, k3 = blk.c3.K, kd = blk.ds.K;
          std::vector<float> rows((size_t)n * (k3 + kd));
          if (m->dmem)
            for (int r = 0; r < n; ++r) {
              for (int c = 0; c < k3; ++c) rows[(size_t)r * (k3 + kd) + c] = w3[(size_t)r * k3 + c];
              for (int c = 0; c < kd; ++c) rows[(size_t)r * (k3 + kd) + k3 + c] = wd[(size_t)r * kd + c];
            }
          std::vector<float> bias(n);
          for (int r = 0; r < n; ++r) bias[r] = b3[r] + bd[r];
          Conv& f = blk.c3ds;
          f.N = n; f.K = k3 + kd; f.Kpad = pad64(f.K); f.Cin = f.K;
          f.w = upload_rows(m, rows, f.N, f.K, f.Kpad);
          f.bias = upload_f32(m, bias.data(), bias.size());
        }
      }
      // conv1 of the blocks whose input is a layer-1 block output (blocks 1-3: layer 1 blocks 1
      // and 2, layer 2 block 0) as the second product of the previous block's fused tail:
      // columns permuted into spe_btail_perm order (btail.hip)
      // (the layer-2 / layer-3 boundaries stay separate launches: their weights do not fit in
      // LDS, and a split-N form streaming them through LDS measured slower)
      const int gi = li == 0 ? k : (li == 1 && k == 0 ? 3 : -1);
      if (m->esz == 2 && spe_btail_enabled() && gi >= 1 && blk.c1.K == 256) {
        std::vector<float> w1, b1;
        fold_conv(m, p + ".conv1.weight", p + ".bn1", "", w1, b1);
        const int n = blk.c1.N, K = blk.c1.K;
        std::vector<float> rows((size_t)n * K, 0.f);
        if (m->dmem)
          for (int r = 0; r < n; ++r)
            for (int c = 0; c < K; ++c) rows[(size_t)r * K + c] = w1[(size_t)r * K + spe_btail_perm(c)];
        Conv& f = blk.c1p;
        f.N = n; f.K = K; f.Kpad = pad64(K); f.Cin = K;
        f.w = upload_rows(m, rows, f.N, f.K, f.Kpad);
        f.bias = upload_f32(m, b1.data(), b1.size());
      }
      m->blocks.push_back(blk);
    }
  m->s8 = make_conv(m, "backbone.0.s8_latern.weight", "", "", 0, 1, 0);
  m->s16 = make_conv(m, "backbone.0.s16_latern.weight", "", "", 0, 1, 1);
  m->s16taps = Conv{};
  if (spe_use_upconv(m)) {
    // per-tap rows for the low-resolution form of s16_latern(up16sto8s(x)) (elementwise.hip
    // upconv_combine): row t*256 + co = weight[co][:][kh][kw], t = kh*3 + kw
    const auto sh = param_shape(m, "backbone.0.s16_latern.weight");
    const int co_n = (int)sh[0], ci_n = (int)sh[1];
    std::vector<float> rows;
    if (m->dmem) {
      const auto& src = m->host["backbone.0.s16_latern.weight"];
      rows.assign((size_t)9 * co_n * ci_n, 0.f);
      for (int t = 0; t < 9; ++t)
        for (int co = 0; co < co_n; ++co)
          for (int ci = 0; ci < ci_n; ++ci)
            rows[((size_t)t * co_n + co) * ci_n + ci] = src[((size_t)co * ci_n + ci) * 9 + t];
    }
    Conv& c = m->s16taps;
    c.N = 9 * co_n; c.K = ci_n; c.Kpad = pad64(ci_n); c.Cin = ci_n;
    c.w = upload_rows(m, rows, c.N, c.K, c.Kpad);
  }
  m->outc = make_conv(m, "backbone.0.output_conv.weight", "", "backbone.0.output_conv.bias", 0, 1, 1);
  m->inproj = make_conv(m, "input_proj.weight", "", "input_proj.bias", 0, 1, 0);
  m->neckip = Conv{};
  if (spe_use_neckfold(m)) {
    const auto so = param_shape(m, "backbone.0.output_conv.weight");   // [512][512][3][3]
    const auto sp = param_shape(m, "input_proj.weight");                // [hidden][512][1][1]
    const int cm = (int)so[0], ci_n = (int)so[1], co_n = (int)sp[0], taps = (int)(so[2] * so[3]);
    std::vector<float> w((size_t)co_n * ci_n * taps, 0.f), bias(co_n, 0.f);
    if (m->dmem) {
      const auto& wo = m->host["backbone.0.output_conv.weight"];
      const auto& bo = m->host["backbone.0.output_conv.bias"];
      const auto& wp = m->host["input_proj.weight"];
      const auto& bp = m->host["input_proj.bias"];
      std::vector<double> acc((size_t)ci_n * taps);
      for (int co = 0; co < co_n; ++co) {
        std::fill(acc.begin(), acc.end(), 0.0);
        double b = bp[co];
        for (int j = 0; j < cm; ++j) {
          const double a = wp[(size_t)co * cm + j];
          const float* src = &wo[(size_t)j * ci_n * taps];
          for (size_t k = 0; k < acc.size(); ++k) acc[k] += a * src[k];
          b += a * bo[j];
        }
        for (size_t k = 0; k < acc.size(); ++k) w[(size_t)co * ci_n * taps + k] = (float)acc[k];
        bias[co] = (float)b;
      }
    }
    m->neckip = pack_conv(m, w, bias, co_n, ci_n, (int)so[2], (int)so[3], 0, 1, 1);
  }

  m->enc.clear();
  for (int i = 0; i < c.enc_layers; ++i) {
    std::string p = "transformer.encoder.layers." + std::to_string(i);
    Enc e;
    e.qk = make_linear(m, p + ".self_attn.in_proj_weight", p + ".self_attn.in_proj_bias", 0, 2 * d, d);
    e.v = make_linear(m, p + ".self_attn.in_proj_weight", p + ".self_attn.in_proj_bias", 2 * d, d, d);
    e.o = make_linear(m, p + ".self_attn.out_proj.weight", p + ".self_attn.out_proj.bias", 0, d, d);
    e.l1 = make_linear(m, p + ".linear1.weight", p + ".linear1.bias", 0, ff, d);
    e.l2 = make_linear(m, p + ".linear2.weight", p + ".linear2.bias", 0, d, ff);
    e.n1g = upload_key(m, p + ".norm1.weight"); e.n1b = upload_key(m, p + ".norm1.bias");
    e.n2g = upload_key(m, p + ".norm2.weight"); e.n2b = upload_key(m, p + ".norm2.bias");
    if (m->h3) {
      e.n1_bound = ln_bound(m, p + ".norm1", d);
      e.n2_bound = ln_bound(m, p + ".norm2", d);
      ffn_h3_prepare(m, e, p, d, ff);
    }
    // bf16 fused FFN: linear2 chunk-packed at finalize (each 32-unit chunk's columns contiguous)
    if (m->cfg.dtype == SPE_DTYPE_BF16_ && d == 256 && ff % 32 == 0) e.ffn_w2c = dalloc(m, (size_t)d * ff * 2);
    m->enc.push_back(e);
  }
  m->dec.clear();
  std::vector<float> kall, vall, kb, vb;
  for (int i = 0; i < c.dec_layers; ++i) {
    std::string p = "transformer.decoder.layers." + std::to_string(i);
    Dec e;
    e.sqk = make_linear(m, p + ".self_attn.in_proj_weight", p + ".self_attn.in_proj_bias", 0, 2 * d, d);
    e.sv = make_linear(m, p + ".self_attn.in_proj_weight", p + ".self_attn.in_proj_bias", 2 * d, d, d);
    e.so = make_linear(m, p + ".self_attn.out_proj.weight", p + ".self_attn.out_proj.bias", 0, d, d);
    e.cq = make_linear(m, p + ".multihead_attn.in_proj_weight", p + ".multihead_attn.in_proj_bias", 0, d, d);
    e.co = make_linear(m, p + ".multihead_attn.out_proj.weight", p + ".multihead_attn.out_proj.bias", 0, d, d);
    e.l1 = make_linear(m, p + ".linear1.weight", p + ".linear1.bias", 0, ff, d);
    e.l2 = make_linear(m, p + ".linear2.weight", p + ".linear2.bias", 0, d, ff);
    e.n1g = upload_key(m, p + ".norm1.weight"); e.n1b = upload_key(m, p + ".norm1.bias");
    e.n2g = upload_key(m, p + ".norm2.weight"); e.n2b = upload_key(m, p + ".norm2.bias");
    e.n3g = upload_key(m, p + ".norm3.weight"); e.n3b = upload_key(m, p + ".norm3.bias");
    if (m->h3) {
      e.n1_bound = ln_bound(m, p + ".norm1", d);
      e.n2_bound = ln_bound(m, p + ".norm2", d);
      e.n3_bound = ln_bound(m, p + ".norm3", d);
    }
    if (spe_use_xattn(m)) fold_cross_attention(m, p, e);
    if (m->esz == 2 && d == 256) {              // filled at finalize (spe_launch_wfrag_pack)
      e.fsqk = dalloc(m, (size_t)2 * d * d * 2);
      e.fsv = dalloc(m, (size_t)d * d * 2);
      e.fso = dalloc(m, (size_t)d * d * 2);
      e.fco = dalloc(m, (size_t)d * d * 2);
      if (spe_use_xattn(m)) {
        e.fxv = dalloc(m, (size_t)d * d * 2);
        e.fxq = dalloc(m, (size_t)e.xq.N * d * 2);
      }
      if (ff % 256 == 0) {
        e.fl1 = dalloc(m, (size_t)ff * d * 2);
        e.fl2 = dalloc(m, (size_t)d * ff * 2);
      }
    }
    m->dec.push_back(e);
    const auto& w = m->host[p + ".multihead_attn.in_proj_weight"];
    const auto& bb = m->host[p + ".multihead_attn.in_proj_bias"];
    kall.insert(kall.end(), w.begin() + (size_t)d * d, w.begin() + (size_t)2 * d * d);
    vall.insert(vall.end(), w.begin() + (size_t)2 * d * d, w.begin() + (size_t)3 * d * d);
    kb.insert(kb.end(), bb.begin() + d, bb.begin() + 2 * d);
    vb.insert(vb.end(), bb.begin() + 2 * d, bb.begin() + 3 * d);
  }
  // all decoder layers' cross-attention K/V projections of the (fixed) memory, batched
  // (not needed when the cross-attention runs against the memory itself)
  if (spe_use_xattn(m)) { kall.clear(); vall.clear(); kb.clear(); vb.clear(); }
  m->crossK.N = m->crossV.N = spe_use_xattn(m) ? 0 : c.dec_layers * d;
  m->crossK.K = m->crossV.K = d;
  m->crossK.Kpad = m->crossV.Kpad = pad64(d);
  m->crossK.w = upload_rows(m, kall, m->crossK.N, d, m->crossK.Kpad);
  m->crossK.bias = upload_f32(m, kb.data(), kb.size());
  m->crossV.w = upload_rows(m, vall, m->crossV.N, d, m->crossV.Kpad);
  m->crossV.bias = upload_f32(m, vb.data(), vb.size());

  const int fs = c.input_size / 8;
  m->pos = upload_T(m, sine_pos(fs, fs, d));
  m->qpos = upload_T(m, m->host["query_embed.weight"]);
  if (m->esz == 2 || m->x6) {
    // bf16 throughput path and fp32x6: the `+ pos` of the q/k projections is applied as
    // (pos . W^T), a row-periodic residual filled by spe_model_finalize (gemm2.hip header) -- for
    // fp32x6 in fp32, computed by the exact-f32 kernel, so the projection is a plain GEMM that the
    // LDS-DMA x6 kernel takes; fp32 / fp32x3 keep the reference's (x + pos) . W^T order.
    const size_t T = (size_t)fs * fs, Q = c.num_queries, es = m->esz;
    for (auto& e : m->enc) e.pos_qk = dalloc(m, T * 2 * d * es);
    m->pos_crossK = spe_use_xattn(m) ? nullptr : dalloc(m, T * c.dec_layers * d * es);
    for (auto& e : m->dec) {
      e.qpos_sqk = dalloc(m, Q * 2 * d * es);
      e.qpos_cq = spe_use_xattn(m) ? nullptr : dalloc(m, Q * d * es);
    }
  }
  m->dng = upload_key(m, "transformer.decoder.norm.weight");
  m->dnb = upload_key(m, "transformer.decoder.norm.bias");

  HeadArgs& h = m->head;
  h.D = d;
  h.cls_wt = upload_transposed(m, "cls_embed.weight", 12, d); h.cls_b = upload_key(m, "cls_embed.bias");
  h.pt_w0t = upload_transposed(m, "point_embed.layers.0.weight", d, d); h.pt_b0 = upload_key(m, "point_embed.layers.0.bias");
  h.pt_w1t = upload_transposed(m, "point_embed.layers.1.weight", d, d); h.pt_b1 = upload_key(m, "point_embed.layers.1.bias");
  h.pt_w2t = upload_transposed(m, "point_embed.layers.2.weight", 2, d); h.pt_b2 = upload_key(m, "point_embed.layers.2.bias");
  if (c.sigma_head) {
    h.sg_w0t = upload_transposed(m, "sigma_embed.layers.0.weight", d, d); h.sg_b0 = upload_key(m, "sigma_embed.layers.0.bias");
    h.sg_w1t = upload_transposed(m, "sigma_embed.layers.1.weight", d, d); h.sg_b1 = upload_key(m, "sigma_embed.layers.1.bias");
    h.sg_w2t = upload_transposed(m, "sigma_embed.layers.2.weight", 1, d); h.sg_b2 = upload_key(m, "sigma_embed.layers.2.bias");
  } else {
    h.sg_w0t = h.sg_b0 = h.sg_w1t = h.sg_b1 = h.sg_w2t = h.sg_b2 = nullptr;
  }
  (void)Q;
  return 0;
}

}  // namespace

Ws spe_plan(const spe_model* m, int B) {
  const auto& c = m->cfg;
  const size_t E = m->esz;
  const size_t S = c.input_size, H2 = S / 2, H4 = S / 4, H8 = S / 8, H16 = S / 16;
  const size_t T = H8 * H8, Q = c.num_queries, d = c.hidden_dim, ff = c.dim_feedforward, L = c.dec_layers;
  Ws w{};
  size_t off = 0;
  auto take = [&](size_t bytes) { size_t o = off; off += (bytes + 255) & ~size_t(255); return o; };
  const size_t big = (size_t)B * std::max(H4 * H4 * 256, H2 * H2 * 64) * E;
  w.bufA = take(big);
  w.bufB = take(big);
  w.stem = w.bufB;                                   // consumed by the max-pool before layer1 writes bufB
  w.pool = w.bufA;
  w.t1 = take((size_t)B * std::max(std::max(H4 * H4 * 128, S * S * 8), H8 * H8 * 256) * E);
  w.x0 = w.t1;                                       // consumed by the stem before t1 is used
  w.t2 = take((size_t)B * std::max(H4 * H4 * 64, std::max(H8 * H8 * 128, H16 * H16 * 256)) * E);
  w.ds = take((size_t)B * H4 * H4 * 256 * E);
  w.xs8 = take((size_t)B * H8 * H8 * 512 * E);
  w.up = take((size_t)B * H8 * H8 * 1024 * E);
  w.cat = take((size_t)B * H8 * H8 * 512 * E);
  w.neck = take((size_t)B * H8 * H8 * 512 * E);
  w.src = take((size_t)B * T * d * E);
  w.srcpos = take((size_t)B * T * d * E);   // memory + pos (bf16 fused path: cross-attention K input)
  w.qkv = take((size_t)B * T * 3 * d * E);
  w.vt = take((size_t)B * T * d * E);
  w.kpl = m->x3 ? take((size_t)B * T * d * 4) : 0;     // (offset 0 is bufA: nonzero = planes present)
  w.ao = take((size_t)B * T * d * E);
  w.tmp = take((size_t)B * T * d * E);
  w.ffn = take((size_t)B * T * ff * E);
  const bool xa = spe_use_xattn(m);
  w.ck = take(xa ? 0 : (size_t)B * T * L * d * E);
  w.cvt = take(xa ? 0 : (size_t)B * T * L * d * E);
  const size_t R = 8 * Q, XS = xa ? (size_t)spe_xattn_splits(B, (int)Q, (int)T) : 0;
  w.xq = take(xa ? (size_t)B * Q * 8 * d * E : 0);
  w.xu = take(xa ? (size_t)B * Q * 8 * d * E : 0);
  // (the cross-attention writes its per-split partials for every split count, 1 included: from
  // B = 256 on a single split covers the chip, and unallocated partials aliased tgt -- NaN decoder)
  w.xpm = take(xa ? XS * B * R * 4 : 0);
  w.xpl = take(xa ? XS * B * R * 4 : 0);
  w.xpu = take(xa ? XS * B * R * d * 4 : 0);
  w.xvp = take(xa && m->h3 ? (size_t)B * T * d * 4 : 0);   // [B*T][512] fp16 (srcpos holds the key planes)
  w.tgt = take((size_t)B * Q * d * E);
  w.dtmp = take((size_t)B * Q * d * E);
  w.dqkv = take((size_t)B * Q * 3 * d * E);
  w.dvt = take((size_t)B * Q * d * E);
  w.dao = take((size_t)B * Q * d * E);
  w.dqc = take((size_t)B * Q * d * E);
  w.dffn = take((size_t)B * Q * ff * E);
  // split-F partials (ffn.hip's split count, or one per 256-wide hidden chunk for decsa.hip's decffn)
  const int fsplit = std::max(spe_ffn_splits((int)(B * Q), (int)ff), m->esz == 2 && d == 256 && ff % 256 == 0 ? (int)ff / 256 : 1);
  w.dffnpart = take((size_t)std::max(1, fsplit) * B * Q * d * 4);
  w.hs = take((size_t)B * Q * d * 4);
  w.amax = take(m->h3 ? SPE_AMAX_SLOTS * 4 : 0);
  w.total = off;
  return w;
}

extern "C" {

int spe_abi_version(void) { return SPE_ABI_VERSION; }
const char* spe_last_error(void) { return g_err.c_str(); }

int spe_model_create(const spe_model_config* cfg, spe_model** out) {
  if (!cfg || !out) return fail(SPE_E_ARG, "null argument");
  if (cfg->hidden_dim != 256 || cfg->nheads * 32 != cfg->hidden_dim)
    return fail(SPE_E_ARG, "only hidden_dim=256 with head_dim=32 is supported");
  if (cfg->input_size % 16 || cfg->input_size < 32) return fail(SPE_E_ARG, "input_size must be a multiple of 16");
  if (cfg->num_queries < 1 || cfg->num_queries > 64) return fail(SPE_E_ARG, "num_queries must be in [1, 64]");
  if (cfg->dim_feedforward % 64) return fail(SPE_E_ARG, "dim_feedforward must be a multiple of 64");
  if (cfg->dtype != SPE_DTYPE_BF16_ && cfg->dtype != SPE_DTYPE_F32_ && cfg->dtype != SPE_DTYPE_F32X3_ &&
      cfg->dtype != SPE_DTYPE_F32X6_ && cfg->dtype != SPE_DTYPE_F32H3_)
    return fail(SPE_E_ARG, "bad dtype");
  if (cfg->attn_dtype != 0 && cfg->attn_dtype != cfg->dtype &&
      !(cfg->attn_dtype == SPE_DTYPE_F16_ && cfg->dtype == SPE_DTYPE_BF16_))
    return fail(SPE_E_ARG, "attn_dtype: 0, the model dtype, or SPE_DTYPE_F16_ for bf16 models");
  spe_model* m = new spe_model();
  m->cfg = *cfg;
  // fp32x3: the fp32 model (storage, layouts, kernels' fp32 paths) with split-bf16 MFMA compute;
  // fp32x6: the same with the GEMMs / convolutions on the three-way split (x6) path
  m->h3 = cfg->dtype == SPE_DTYPE_F32H3_;
  m->x6 = cfg->dtype == SPE_DTYPE_F32X6_ || m->h3;
  m->x3 = cfg->dtype == SPE_DTYPE_F32X3_ || m->x6;
  if (m->x3) { m->cfg.dtype = SPE_DTYPE_F32_; if (m->cfg.attn_dtype) m->cfg.attn_dtype = SPE_DTYPE_F32_; }
  m->esz = cfg->dtype == SPE_DTYPE_BF16_ ? 2 : 4;
  m->spec = build_spec(*cfg);
  *out = m;
  return 0;
}

void spe_model_destroy(spe_model* m) {
  if (!m) return;
  if (m->dmem) (void)hipFree(m->dmem);
  for (auto e : m->prof.pool) (void)hipEventDestroy(e);
  delete m->rt;
  delete m;
}

int spe_model_num_params(const spe_model* m) { return m ? (int)m->spec.size() : 0; }
const char* spe_model_param_name(const spe_model* m, int i) {
  return (m && i >= 0 && i < (int)m->spec.size()) ? m->spec[i].first.c_str() : nullptr;
}

int spe_model_set_param(spe_model* m, const char* key, const float* data, int64_t numel) {
  if (!m || !key || !data) return fail(SPE_E_ARG, "null argument");
  if (m->finalized) return fail(SPE_E_STATE, "model already finalized");
  for (auto& s : m->spec)
    if (s.first == key) {
      int64_t n = 1;
      for (auto v : s.second) n *= v;
      if (n != numel) return fail(SPE_E_KEY, std::string("wrong element count for ") + key);
      m->host[key].assign(data, data + numel);
      return 0;
    }
  return fail(SPE_E_KEY, std::string("unknown parameter key ") + key);
}

int spe_model_finalize(spe_model* m) {
  if (!m) return fail(SPE_E_ARG, "null model");
  if (m->finalized) return fail(SPE_E_STATE, "model already finalized");
  for (auto& s : m->spec)
    if (!m->host.count(s.first)) return fail(SPE_E_MISSING, "missing parameter " + s.first);
  // pass 1 sizes the device block, pass 2 packs and uploads
  m->dmem = nullptr;
  m->dused = 0;
  auto build = [&] { return m->family == 1 ? spe_rtdetr_build_device(m) : build_device(m); };
  int rc0 = build();
  if (rc0) return rc0;
  m->dbytes = m->dused;
  hipError_t e = hipMalloc((void**)&m->dmem, m->dbytes);
  if (e != hipSuccess) return fail((int)e, "hipMalloc of weights failed");
  m->dused = 0;
  m->upload_err = 0;
  rc0 = build();
  if (rc0) return rc0;
  e = hipDeviceSynchronize();
  if (e != hipSuccess || m->upload_err) return fail(e != hipSuccess ? (int)e : m->upload_err, "weight upload failed");
  if ((m->esz == 2 || m->x6) && m->family == 0) {
    const int d = m->cfg.hidden_dim, fs = m->cfg.input_size / 8, T = fs * fs, Q = m->cfg.num_queries;
    auto proj = [&](const void* A, int rows, const Conv& w, void* out) {
      GemmArgs g{};
      g.A = A; g.lda = d; g.B = w.w; g.ldb = w.Kpad;
      g.M = rows; g.N = w.N; g.K = w.K; g.C = out; g.ldc = w.N;
      return spe_launch_gemm(g, m->esz == 2 ? SPE_DTYPE_BF16 : SPE_DTYPE_F32, GEMM_LINEAR, nullptr);
    };
    int rc = 0;
    for (auto& l : m->enc) {
      rc |= proj(m->pos, T, l.qk, l.pos_qk);
      if (l.ffn_w2c) rc |= spe_launch_ffn_w2_chunk_pack(l.l2.w, l.l2.Kpad, l.l2.K, l.ffn_w2c, nullptr);
    }
    if (m->pos_crossK) rc |= proj(m->pos, T, m->crossK, m->pos_crossK);
    for (auto& l : m->dec) {
      rc |= proj(m->qpos, Q, l.sqk, l.qpos_sqk);
      if (l.qpos_cq) rc |= proj(m->qpos, Q, l.cq, l.qpos_cq);
      auto pack = [&](const Conv& w, void* dst) { return dst ? spe_launch_wfrag_pack(w.w, w.Kpad, w.N, dst, nullptr) : 0; };
      rc |= pack(l.sqk, l.fsqk) | pack(l.sv, l.fsv) | pack(l.so, l.fso) | pack(l.co, l.fco) | pack(l.xv, l.fxv) | pack(l.xq, l.fxq);
      if (l.fl1) {
        rc |= pack(l.l1, l.fl1);
        for (int c0 = 0; c0 < l.l2.K; c0 += 256)
          rc |= spe_launch_wfrag_pack((const char*)l.l2.w + (size_t)c0 * 2, l.l2.Kpad, d, (char*)l.fl2 + (size_t)c0 * d * 2, nullptr);
      }
    }
    e = hipDeviceSynchronize();
    if (rc || e != hipSuccess) return fail(SPE_E_LAUNCH, "positional projection precompute failed");
  }
  m->host.clear();
  m->finalized = true;
  return 0;
}

int64_t spe_model_workspace_bytes(const spe_model* m, int batch) {
  if (!m || batch <= 0) return -1;
  if (m->family == 1) return spe_rtdetr_workspace(m, batch);
  return (int64_t)spe_plan(m, batch).total;
}

}  // extern "C"
