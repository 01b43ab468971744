// Native runtime of the keypoint-set predictor, part 2: the launch sequence of one forward
// pass (REV/models/detr_speed.py:59-92 -> backbone.py:133-149 -> transformer.py:51-63 ->
// heads + PostProcess) on one HIP stream, and the solver / score entry points.  No allocation
// or synchronisation happens inside spe_forward / spe_pnp_batch / spe_speed_score, so a caller
// may capture them into a hipGraph.  Every launch goes through run_gemm / run_attn / run_other,
// which bracket it with HIP events when the per-launch profiler is on (bench roofline).
#include <hip/hip_runtime.h>
#include <hip/hip_ext.h>

#include <cmath>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <functional>
#include <map>
#include <mutex>
#include <tuple>

#include "model_state.h"
#include "spe_pnp.h"
#include "launch.h"

#define fail spe_fail

namespace {

hipEvent_t next_event(spe_model* m) {
  Profiler& p = m->prof;
  if (p.next_event == p.pool.size()) {
    hipEvent_t e;
    if (hipEventCreate(&e) != hipSuccess) return nullptr;
    p.pool.push_back(e);
  }
  return p.pool[p.next_event++];
}

// fp32h3 activation-scale ledger (one per forward call): every slot of a range the call zeroes must be
// raised by an earlier launch of the same call (GemmArgs::amax_c, the input pack, the cross-attention
// merge) before a launch reads it as its scale (amax_a and the like) -- a consumer without a producer
// would otherwise run at scale 1 in silence (h3_scale), losing precision or overflowing fp16.  Slots
// of ranges this call did not zero (a stage run by an earlier call) are not checked.
struct AmaxLedger {
  const float* base = nullptr;
  unsigned char state[SPE_AMAX_SLOTS] = {};     // 0 unchecked, 1 zeroed and awaiting a producer, 2 raised
  int index(const float* p) const {
    const long d = base && p ? (long)(p - base) : -1;
    return d >= 0 && d < SPE_AMAX_SLOTS ? (int)d : -1;
  }
  void zeroed(int first, int n) {
    for (int i = first; i < first + n; ++i) state[i] = 1;
  }
  void raised(const float* p) {
    const int i = index(p);
    if (i >= 0) state[i] = 2;
  }
  bool ok(const float* p) const {
    const int i = index(p);
    return i < 0 || state[i] != 1;
  }
};
thread_local AmaxLedger* g_ledger = nullptr;
struct LedgerScope {
  AmaxLedger ledger;
  explicit LedgerScope(const float* base) {
    ledger.base = base;
    g_ledger = base ? &ledger : nullptr;
  }
  ~LedgerScope() { g_ledger = nullptr; }
};
// a launch reading `in` and raising `out`: SPE_E_STATE if `in` has no producer yet
int ledger_use(const float* in, const float* out, const char* kind) {
  if (!g_ledger) return 0;
  if (!g_ledger->ok(in)) {
    char b[160];
    snprintf(b, sizeof b, "fp32h3: %s reads activation-scale slot %d before any launch raised it", kind,
             g_ledger->index(in));
    return spe_fail(SPE_E_STATE, b);
  }
  g_ledger->raised(out);
  return 0;
}

bool prof_match(const spe_model* m, const char* kind) {
  return m->prof.on && std::strncmp(kind, m->prof.filter.c_str(), m->prof.filter.size()) == 0;
}

}  // namespace

// ---- launch helpers shared with rtdetr.cpp (launch.h)
int run_other(spe_model* m, const char* kind, double flops, double bytes, hipStream_t s, const std::function<int()>& fn) {
  if (!prof_match(m, kind)) return fn();
  ProfRecord r{kind, kind, flops, bytes, next_event(m), next_event(m)};
  if (!r.beg || !r.end) return (int)hipErrorOutOfMemory;
  (void)hipEventRecord(r.beg, s);
  int rc = fn();
  (void)hipEventRecord(r.end, s);
  m->prof.recs.push_back(r);
  return rc;
}

// fp32x3 models: split-bf16 MFMA.  fp32x6 models run the decoder's attention (self and cross,
// Q = 11 query rows: ~1 % of the model's flops) on the exact-f32 kernels: the per-stage study
//  found its split-bf16 scores to carry most of the mode's keypoint error
// (1.6e-4 -> 5.7e-5 on the bench weights at equal step time).
static bool x3_for(const spe_model* m, const char* kind) {
  if (!m->x3) return false;
  if (m->x6 && std::strncmp(kind, "attn.dec", 8) == 0) return false;
  return true;
}

int run_gemm(spe_model* m, const char* kind, const GemmArgs& g, int mode, hipStream_t s) {
  if (const int rc = ledger_use(g.amax_a, g.amax_c, kind)) return rc;
  const double E = m->esz;
  const double a_elems = mode == GEMM_CONV ? (double)(g.M / (g.Ho * g.Wo)) * g.H * g.W * g.Cin : (double)g.M * g.K;
  const double r_rows = g.R ? (g.r_period > 0 ? (double)g.r_period : (double)g.M) : 0.0;
  const double bytes = (a_elems + (double)g.N * g.K + (double)g.M * g.N + r_rows * g.N) * E +
                       (mode == GEMM_LINEAR_ADD ? (double)g.prow * g.K * E : 0.0);
  int dt = !x3_for(m, kind) ? m->cfg.dtype : m->x6 ? (int)SPE_DTYPE_F32X6 : (int)SPE_DTYPE_F32X3;
  GemmArgs ga = g;
  if (dt == SPE_DTYPE_F32X6) {
    const auto it = m->w6.find(g.B);
    if (it != m->w6.end()) { ga.B6 = it->second.first; ga.b6_rows = it->second.second; }
    // fp32h3: the GEMMs whose A operand has a known max |A| (published by its producer, or a LayerNorm
    // / attention bound) take the scaled fp16 split (gemm.hip gemm_h3d / gemm_h3p); the rest stay on x6
    const auto ih = m->wh3.find(g.B);
    if (m->h3 && g.amax_a && ih != m->wh3.end()) {
      ga.H3 = ih->second.planes; ga.h3_rows = ih->second.rows; ga.h3_sinv = ih->second.sinv;
      dt = SPE_DTYPE_F32H3;
    }
  }
  return run_other(m, kind, 2.0 * g.M * g.N * g.K, bytes, s, [&] { return spe_launch_gemm(ga, dt, mode, s); });
}

int run_attn(spe_model* m, const char* kind, const AttnArgs& a, int dtype, hipStream_t s) {
  const double flops = 4.0 * a.B * a.H * (double)a.Tq * a.Tk * 32;
  const double bytes = (double)a.B * a.H * 32 * (2.0 * a.Tq + 2.0 * a.Tk) * m->esz;
  const int dt = (x3_for(m, kind) && dtype == SPE_DTYPE_F32) ? (int)SPE_DTYPE_F32X3 : dtype;
  if (const int rc = ledger_use(a.v_amax, nullptr, kind)) return rc;
  return run_other(m, kind, flops, bytes, s, [&] { return spe_launch_attention(a, dt, s); });
}

GemmArgs linear_args(const Conv& c, const void* A, int lda, int M, void* C, int ldc) {
  GemmArgs g{};
  g.A = A; g.lda = lda;
  g.B = c.w; g.ldb = c.Kpad;
  g.M = M; g.N = c.N; g.K = c.K;
  g.bias = c.bias;
  g.C = C; g.ldc = ldc;
  return g;
}

// Fused linear1 -> ReLU -> linear2 -> +residual -> LayerNorm over x (in place), bf16 models.
int run_ffn(spe_model* m, const char* kind, const Conv& l1, const Conv& l2, const float* g, const float* b,
            void* x, int M, hipStream_t s, const void* pos, void* ypos, int period, float* partial,
            const void* w2_chunked) {
  FfnArgs a{};
  a.pos = pos; a.ypos = ypos; a.pos_period = period;
  a.splits = partial ? spe_ffn_splits(M, l1.N) : 1;
  a.partial = a.splits > 1 ? partial : nullptr;
  a.x = x; a.ldx = l1.K;
  a.w1 = l1.w; a.ld1 = l1.Kpad; a.b1 = l1.bias;
  a.w2 = w2_chunked ? w2_chunked : l2.w; a.ld2 = l2.Kpad; a.b2 = l2.bias;
  a.w2_chunked = w2_chunked != nullptr;        // W2 chunk-packed at finalize (ffn.hip)
  a.gamma = g; a.beta = b;
  a.y = x; a.ldy = l1.K;
  a.M = M; a.D = l1.K; a.F = l1.N;
  const double flops = 4.0 * M * (double)l1.K * l1.N;
  const double bytes = 2.0 * M * l1.K * m->esz + 2.0 * (double)l1.K * l1.N * m->esz;
  return run_other(m, kind, flops, bytes, s, [&] { return spe_launch_ffn_ln(a, s); });
}

namespace {

bool use_fused_ffn(const spe_model* m) {
  return m->cfg.dtype == SPE_DTYPE_BF16 && m->cfg.hidden_dim == 256 && m->cfg.dim_feedforward % 32 == 0;
}

// `(x + pos) . W^T`: fp32 / fp32x3 models add pos to the A operand as the reference does; bf16
// and fp32x6 models add the precomputed pos . W^T as a row-periodic residual (see gemm2.hip).
int add_pos(const spe_model* m, GemmArgs& g, const void* pos, int ldp, int period, const void* posw, int ldw) {
  if ((m->esz == 2 || m->x6) && posw) {
    g.R = posw; g.ldr = ldw; g.r_period = period;
    return GEMM_LINEAR;
  }
  g.P = pos; g.ldp = ldp; g.prow = period;
  return GEMM_LINEAR_ADD;
}

}  // namespace

GemmArgs conv_args(const Conv& c, const void* X, int B, int H, int W, void* Y, int ldc) {
  GemmArgs g{};
  g.A = X;
  g.H = H; g.W = W; g.Cin = c.Cin; g.KH = c.KH; g.KW = c.KW; g.stride = c.stride; g.pad = c.pad;
  g.Ho = (H + 2 * c.pad - c.KH) / c.stride + 1;
  g.Wo = (W + 2 * c.pad - c.KW) / c.stride + 1;
  g.B = c.w; g.ldb = c.Kpad;
  g.M = B * g.Ho * g.Wo; g.N = c.N; g.K = c.K;
  g.bias = c.bias;
  g.C = Y; g.ldc = ldc;
  return g;
}

namespace {
#define CK(x)                                                                   \
  do {                                                                          \
    int _r = (x);                                                               \
    if (_r != 0) {                                                              \
      char _b[256];                                                             \
      snprintf(_b, sizeof _b, "%s failed (%d) at %s:%d", #x, _r, __FILE__, __LINE__); \
      return fail(_r < 0 ? SPE_E_LAUNCH : _r, _b);                              \
    }                                                                           \
  } while (0)



}  // namespace

extern "C" {

int spe_forward(spe_model* m, void* stream, const float* images, int B, void* workspace, int64_t ws_bytes,
                const spe_forward_outputs* out) {
  return spe_forward_stages(m, stream, images, B, workspace, ws_bytes, out, SPE_STAGE_ENCODE | SPE_STAGE_DECODE);
}

static int forward_stages(spe_model* m, void* stream, const ImageSrc& images, int B, void* workspace, int64_t ws_bytes,
                          const spe_forward_outputs* out, int stages);

int spe_forward_stages(spe_model* m, void* stream, const float* images, int B, void* workspace, int64_t ws_bytes,
                       const spe_forward_outputs* out, int stages) {
  return forward_stages(m, stream, ImageSrc{images, nullptr, 0}, B, workspace, ws_bytes, out, stages);
}

int spe_forward_stages_u8(spe_model* m, void* stream, const uint8_t* crops, int channels, int B, void* workspace,
                          int64_t ws_bytes, const spe_forward_outputs* out, int stages) {
  if ((stages & (SPE_STAGE_ENCODE | SPE_STAGE_BACKBONE)) && (!crops || (channels != 1 && channels != 3)))
    return fail(SPE_E_ARG, "u8 crops: device pointer, 1 or 3 channels");
  return forward_stages(m, stream, ImageSrc{nullptr, crops, channels}, B, workspace, ws_bytes, out, stages);
}

static int forward_stages(spe_model* m, void* stream, const ImageSrc& images, int B, void* workspace, int64_t ws_bytes,
                          const spe_forward_outputs* out, int stages) {
  if (!m || !workspace || B <= 0 ||
      (stages & ~(SPE_STAGE_ENCODE | SPE_STAGE_DECODE | SPE_STAGE_BACKBONE | SPE_STAGE_TRANSFORMER)) || !stages)
    return fail(SPE_E_ARG, "bad argument");
  if (stages & SPE_STAGE_ENCODE) stages |= SPE_STAGE_BACKBONE | SPE_STAGE_TRANSFORMER;
  if ((stages & SPE_STAGE_BACKBONE) && !images.f32 && !images.u8) return fail(SPE_E_ARG, "null images");
  if ((stages & SPE_STAGE_DECODE) && (!out || !out->logits || !out->points)) return fail(SPE_E_ARG, "null outputs");
  if (m->family != 0) return fail(SPE_E_ARG, "not a DETR model (use spe_rtdetr_forward)");
  if (!m->finalized) return fail(SPE_E_STATE, "model not finalized");
  const Ws w = spe_plan(m, B);
  if ((int64_t)w.total > ws_bytes) return fail(SPE_E_WORKSPACE, "workspace too small");
  hipStream_t s = (hipStream_t)stream;
  const auto& c = m->cfg;
  const int dt = c.dtype, S = c.input_size, d = c.hidden_dim, ff = c.dim_feedforward, Q = c.num_queries;
  const int L = c.dec_layers;
  char* ws = (char*)workspace;
  auto P = [&](size_t off) { return (void*)(ws + off); };

  const int F = S / 8, T = F * F;
  const float scale = 1.0f / std::sqrt(32.0f);
  const int Mt = B * T;
  const bool xa = spe_use_xattn(m);
  // fp32h3: each tensor a GEMM reads carries a device max |x| (the producer's published maximum,
  // or a bound), the scale input of the scaled fp16 split (gemm.hip gemm_h3d).  Slots: backbone
  // [0, SPE_AMAX_BB), the neck output (the encoder's first input) at SPE_AMAX_BB - 1, transformer
  // [SPE_AMAX_BB, SPE_AMAX_SLOTS); each stage zeroes its own range first.
  float* const amx = m->h3 ? (float*)P(w.amax) : nullptr;
  float* const src_amax0 = amx ? amx + SPE_AMAX_BB - 1 : nullptr;
  LedgerScope ledger_scope(amx);
  // (the slot counts are checked before anything is launched: a slot handed out past its range would
  // be the encoder's input scale or a transformer slot, overwritten before an error could return)
  if (amx && (stages & SPE_STAGE_BACKBONE) && 2 + 3 * (int)m->blocks.size() + 2 > SPE_AMAX_BB - 1)
    return fail(SPE_E_STATE, "fp32h3: backbone activation-scale slots exhausted");
  if (amx && (stages & SPE_STAGE_TRANSFORMER) && 2 * (int)m->enc.size() > SPE_AMAX_DEC - SPE_AMAX_BB - 1)
    return fail(SPE_E_STATE, "fp32h3: encoder activation-scale slots exhausted");
  if (amx && (stages & SPE_STAGE_DECODE) && 3 * c.dec_layers > SPE_AMAX_SLOTS - SPE_AMAX_DEC)
    return fail(SPE_E_STATE, "fp32h3: decoder activation-scale slots exhausted");
  if (stages & SPE_STAGE_BACKBONE) {
  int na = 0;
  auto slot = [&]() -> float* { return amx ? amx + na++ : nullptr; };
  if (amx) CK((int)hipMemsetAsync(amx, 0, SPE_AMAX_BB * 4, s));
  if (amx) ledger_scope.ledger.zeroed(0, SPE_AMAX_BB);
  // ---------------- backbone (REV/models/backbone.py:133-149)
  const bool pairs = m->esz == 2 && m->stem.Cin == 4;  // bf16: pair-packed stem (registry.cpp)
  float* const x0_amax = slot();
  if (pairs)
    CK(run_other(m, "eltwise.pack", 0.0, (double)B * S * S * 12 + (double)B * (S + 6) * (S + 6) * 8, s,
                 [&] { return spe_launch_pack_input_pad4(images, P(w.x0), B, S, s); }));
  else
    CK(run_other(m, "eltwise.pack", 0.0, (double)B * S * S * (12 + m->stem.Cin * m->esz), s,
                 [&] { return spe_launch_pack_input(images, P(w.x0), B, S, dt, s, x0_amax, m->stem.Cin); }));
  CK(ledger_use(nullptr, x0_amax, "eltwise.pack"));
  int H = S / 2;
  float* const stem_amax = slot();
  const int Hp = (H + 2 - 3) / 2 + 1;
  // bf16: layer1 block 0's conv3 + downsample run as one GEMM over [conv2 output | pool output]
  // (Block::c3ds), so the max-pool writes the right half of that concatenation (w.ds region,
  // row stride c3ds.K) and conv2 the left half
  const Block& b0 = m->blocks[0];
  const bool fuse0 = b0.c3ds.w != nullptr;
  const int uld = fuse0 ? b0.c3ds.K : 64;
  const size_t pool_at = fuse0 ? w.ds + (size_t)b0.c2.N * m->esz : w.pool;
  if (pairs && spe_stempool_enabled() && spe_stempool_fits(S)) {
    // stem + bias + ReLU + max-pool in one pass (stempool.hip): the stem output stays in registers
    const double flops = 2.0 * B * H * H * 64 * 7 * 8 * 4;
    const double bytes = (double)B * (S + 6) * (S + 6) * 8 + (double)B * Hp * Hp * 64 * m->esz;
    CK(run_other(m, "conv.stem", flops, bytes, s, [&] {
      return spe_launch_stempool(P(w.x0), m->stem.w, m->stem.Kpad, m->stem.bias, P(pool_at), uld, B, S, s);
    }));
  } else {
    {
      GemmArgs g = pairs ? conv_args(m->stem, P(w.x0), B, S + 6, S + 6, P(w.stem), 64)
                         : conv_args(m->stem, P(w.x0), B, S, S, P(w.stem), 64);
      g.act = ACT_RELU;
      g.amax_a = x0_amax; g.amax_c = stem_amax;
      CK(run_gemm(m, "conv.stem", g, GEMM_CONV, s));
    }
    CK(run_other(m, "eltwise.maxpool", 0.0, (double)B * 64 * (H * H + Hp * Hp) * m->esz, s, [&] { return spe_launch_maxpool3s2(P(w.stem), P(pool_at), B, H, H, 64, Hp, Hp, dt, s, uld); }));
  }
  H = Hp;
  size_t cur = pool_at;                                 // (w.pool aliases bufA)
  const float* cur_amax = stem_amax;                    // the max-pool's maximum is the stem's
  const float* xs8_amax = nullptr;
  int cin = 64, cur_ld = uld;
  bool t1_ready = false;                                // this block's conv1 ran in the previous tail
  // conv3 (+ residual) + relu of block bi and the next block's conv1 as one launch (btail.hip)
  // when the next block carries permuted conv1 weights (layer-1 outputs, registry.cpp c1p)
  auto tail = [&](const Block& nb, const void* A, int lda, int k1, const void* R, const Conv& c3, size_t out, int M) {
    BtailArgs t{};
    t.A = A; t.lda = lda; t.k1 = k1; t.R = R; t.ldr = c3.N;
    t.w3 = c3.w; t.ld3 = c3.Kpad; t.b3 = c3.bias; t.y = P(out); t.ldy = c3.N; t.n1 = c3.N;
    t.w1 = nb.c1p.w; t.ld1 = nb.c1p.Kpad; t.b1 = nb.c1p.bias; t.z = P(w.t1); t.ldz = nb.c1.N; t.n2 = nb.c1.N;
    t.M = M;
    const double flops = 2.0 * M * ((double)c3.N * k1 + (double)nb.c1.N * c3.N);
    const double bytes = ((double)M * (k1 + c3.N + nb.c1.N) + (R ? (double)M * c3.N : 0.0)) * m->esz;
    return run_other(m, "conv.1x1", flops, bytes, s, [&] { return spe_launch_btail(t, s); });
  };
  for (size_t bi = 0; bi < m->blocks.size(); ++bi) {
    const Block& blk = m->blocks[bi];
    const bool fused = bi == 0 && fuse0;
    const Block* nb = bi + 1 < m->blocks.size() && m->blocks[bi + 1].c1p.w ? &m->blocks[bi + 1] : nullptr;
    // layer1: blocks 0-2, layer2: 3-6 (its output xs8 is kept for the neck), layer3: 7-12
    const size_t outbuf = (bi == 6) ? w.xs8 : (cur == w.bufA ? w.bufB : w.bufA);
    const int Ho = (H + 2 - 3) / blk.stride + 1;
    float* const t1_amax = slot();
    float* const t2_amax = slot();
    float* const out_amax = slot();
    if (!t1_ready) {  // conv1 1x1 + bn1 + relu
      GemmArgs g = linear_args(blk.c1, P(cur), cur_ld, B * H * H, P(w.t1), blk.c1.N);
      g.act = ACT_RELU;
      g.amax_a = cur_amax; g.amax_c = t1_amax;
      CK(run_gemm(m, "conv.1x1", g, GEMM_LINEAR, s));
    }
    t1_ready = false;
    {  // conv2 3x3 (stride on the 3x3, ResNet v1.5) + bn2 + relu
      GemmArgs g = conv_args(blk.c2, P(w.t1), B, H, H, fused ? P(w.ds) : P(w.t2), fused ? uld : blk.c2.N);
      g.act = ACT_RELU;
      g.amax_a = t1_amax; g.amax_c = t2_amax;
      CK(run_gemm(m, "conv.3x3", g, GEMM_CONV, s));
    }
    if (fused) {  // relu(W3 t2 + Wds x + b3 + bds) over the concatenation
      int rc = 1;
      if (nb && blk.c3ds.N == 256) {
        rc = tail(*nb, P(w.ds), uld, blk.c3ds.K, nullptr, blk.c3ds, outbuf, B * Ho * Ho);
        if (rc != 0 && rc != 1) CK(rc);   // 1 = shapes not served: the GEMM pair below
      }
      if (rc == 1) {
        GemmArgs g = linear_args(blk.c3ds, P(w.ds), uld, B * Ho * Ho, P(outbuf), blk.c3ds.N);
        g.act = ACT_RELU;
        CK(run_gemm(m, "conv.1x1", g, GEMM_LINEAR, s));
      }
      t1_ready = rc == 0;
      cin = cur_ld = blk.c3.N;
      H = Ho;
      cur = outbuf;
      continue;
    }
    size_t res = cur;
    if (blk.has_ds) {
      if (blk.stride == 1) {
        GemmArgs g = linear_args(blk.ds, P(cur), cin, B * H * H, P(w.ds), blk.ds.N);
        g.amax_a = cur_amax;
        CK(run_gemm(m, "conv.1x1", g, GEMM_LINEAR, s));
      } else {
        GemmArgs g = conv_args(blk.ds, P(cur), B, H, H, P(w.ds), blk.ds.N);
        g.amax_a = cur_amax;
        CK(run_gemm(m, "conv.1x1s2", g, GEMM_CONV, s));
      }
      res = w.ds;
    }
    {  // conv3 1x1 + bn3 + residual + relu (+ the next block's conv1, btail.hip)
      int rc = 1;
      if (nb) {
        rc = tail(*nb, P(w.t2), blk.c2.N, blk.c3.K, P(res), blk.c3, outbuf, B * Ho * Ho);
        if (rc != 0 && rc != 1) CK(rc);   // 1 = shapes not served: the GEMM pair below
      }
      if (rc == 1) {
        GemmArgs g = linear_args(blk.c3, P(w.t2), blk.c2.N, B * Ho * Ho, P(outbuf), blk.c3.N);
        g.R = P(res); g.ldr = blk.c3.N; g.act = ACT_RELU;
        g.amax_a = t2_amax; g.amax_c = out_amax;
        CK(run_gemm(m, "conv.1x1", g, GEMM_LINEAR, s));
      }
      t1_ready = rc == 0;
    }
    cur_amax = out_amax;
    if (bi == 6) xs8_amax = out_amax;
    cin = cur_ld = blk.c3.N;
    H = Ho;
    cur = outbuf;
  }
  const size_t xs16 = cur;                              // [B, S/16, S/16, 1024]
  float* const cat_amax = slot();
  {  // s8_latern 1x1 512->256 into channels [0,256) of the concat buffer
    GemmArgs g = linear_args(m->s8, P(w.xs8), 512, B * T, P(w.cat), 512);
    g.bias = nullptr;
    g.amax_a = xs8_amax; g.amax_c = cat_amax;
    CK(run_gemm(m, "conv.neck", g, GEMM_LINEAR, s));
  }
  if (spe_use_upconv(m)) {
    // s16_latern(up16sto8s(xs16)) at the low resolution: Z = xs16 . [W_t]^T for the 9 taps
    // (w.up holds Z [B*(S/16)^2][9*256]), then the bilinear combine into channels [256,512)
    const int h = S / 16, nz = m->s16taps.N;
    GemmArgs g = linear_args(m->s16taps, P(xs16), 1024, B * h * h, P(w.up), nz);
    // the combine sums nine bilinear interpolations of Z (each a convex combination): its output
    // is bounded by 9 max |Z|, published into the concat's slot
    g.amax_a = cur_amax; g.amax_c = cat_amax; g.amax_c_mul = 9.f;
    CK(run_gemm(m, "conv.neck", g, GEMM_LINEAR, s));
    const double by = ((double)B * h * h * nz + (double)B * 4 * h * h * 256) * m->esz;
    CK(run_other(m, "eltwise.upconv", 0.0, by, s, [&] { return spe_launch_upconv_combine(P(w.up), (char*)P(w.cat) + 256 * m->esz, 512, B, h, h, 256, dt, s); }));
  } else {
  CK(run_other(m, "eltwise.upsample", 0.0, (double)B * 1024 * 5 * (S / 16) * (S / 16) * m->esz, s, [&] { return spe_launch_upsample2x(P(xs16), P(w.up), B, S / 16, S / 16, 1024, dt, s); }));
  {  // s16_latern 3x3 1024->256 into channels [256,512)
    GemmArgs g = conv_args(m->s16, P(w.up), B, F, F, (char*)P(w.cat) + 256 * m->esz, 512);
    g.bias = nullptr;
    g.amax_a = cur_amax; g.amax_c = cat_amax;          // (bilinear upsampling keeps max |x|)
    CK(run_gemm(m, "conv.neck", g, GEMM_CONV, s));
  }
  }
  if (spe_use_neckfold(m)) {  // input_proj . output_conv as one 3x3 conv 512->256 -> src [B*T, 256]
    GemmArgs g = conv_args(m->neckip, P(w.cat), B, F, F, P(w.src), d);
    g.amax_a = cat_amax; g.amax_c = src_amax0;
    CK(run_gemm(m, "conv.neck", g, GEMM_CONV, s));
  } else {
  float* const neck_amax = slot();
  {  // output_conv 3x3 512->512 + bias
    GemmArgs g = conv_args(m->outc, P(w.cat), B, F, F, P(w.neck), 512);
    g.amax_a = cat_amax; g.amax_c = neck_amax;
    CK(run_gemm(m, "conv.neck", g, GEMM_CONV, s));
  }
  {  // input_proj 1x1 512->256 + bias -> src [B*T, 256] (token order h*W+w)
    GemmArgs g = linear_args(m->inproj, P(w.neck), 512, B * T, P(w.src), d);
    g.amax_a = neck_amax; g.amax_c = src_amax0;
    CK(run_gemm(m, "gemm.input_proj", g, GEMM_LINEAR, s));
  }
  }
  if (na > SPE_AMAX_BB - 1) return fail(SPE_E_STATE, "fp32h3: backbone slot count out of step with the up-front check");
  }  // SPE_STAGE_BACKBONE
  if (stages & SPE_STAGE_TRANSFORMER) {
  float* const tam = amx ? amx + SPE_AMAX_BB : nullptr;
  if (tam) CK((int)hipMemsetAsync(tam, 0, (SPE_AMAX_DEC - SPE_AMAX_BB) * 4, s));
  if (tam) ledger_scope.ledger.zeroed(SPE_AMAX_BB, SPE_AMAX_DEC - SPE_AMAX_BB);
  const float* src_amax = src_amax0;
  int li = 0;

  // ---------------- encoder (REV/models/transformer.py:154-167)
  // fp16 encoder attention operands (bf16 models, attn_dtype = SPE_DTYPE_F16_): the q/k and V^T
  // projections store fp16, the attention runs fp16 MFMAs; everything else stays bf16
  const int f16attn = c.attn_dtype == SPE_DTYPE_F16_ && dt == SPE_DTYPE_BF16;
  // bf16 models otherwise keep bf16 q/k but store V^T as fp16: the attention's P is then fp16
  // and its row sums packed-fp16 adds (attention.hip, TV).  fp16 has the finer mantissa; V and
  // P stay far inside its range.  SPE_ATTN_F16V=0 keeps V^T and P bf16 (A/B knob).
  static const int f16v_env = [] { const char* e = getenv("SPE_ATTN_F16V"); return e ? atoi(e) : 1; }();
  const int f16v = !f16attn && dt == SPE_DTYPE_BF16 && f16v_env;
  const int attn_dt = f16attn ? SPE_DTYPE_F16 : f16v ? SPE_DTYPE_BF16_F16V : dt;
  // 16-bit encoder attention stages K / V^T by LDS DMA, which needs V^T rows in its key order
  // (vt_pos: the v projection's epilogue writes them so); SPE_ATTN_DMA=0 keeps register staging
  static const int dma_env = [] { const char* e = getenv("SPE_ATTN_DMA"); return e ? atoi(e) : 1; }();
  const int vt_swz = dma_env && dt == SPE_DTYPE_BF16 && T % 16 == 0;
  // fp32x3 / fp32x6 encoder attention: the q/k and v projection epilogues write K and V^T as bf16
  // hi / lo planes (GemmArgs::S) that the attention stages as plain copies (SPE_ATTN_PRESPLIT=0:
  // fp32 K / V^T, split per tile inside the attention)
  static const int ps_env = [] { const char* e = getenv("SPE_ATTN_PRESPLIT"); return e ? atoi(e) : 1; }();
  const bool presplit = ps_env && w.kpl && x3_for(m, "attn.enc") && T % 8 == 0;
  // ... with V^T in the 16-bit key order (T % 16 == 0): the LDS-DMA split kernel (attn_split.hip); the
  // fp32h3 model's V^T planes are then fp16 of V * 2^-ev, ev from max |src| . max_n |Wv[n]|_1 + max |bv|
  const int split_swz = presplit && T % 16 == 0;
  const int split_f16 = split_swz && m->h3 && src_amax0;
  for (const Enc& e : m->enc) {
    {
      GemmArgs g = linear_args(e.qk, P(w.src), d, Mt, P(w.qkv), 3 * d);
      g.out_f16 = f16attn;
      g.amax_a = src_amax;
      if (presplit) { g.S = P(w.kpl); g.s_col0 = d; }
      const int mode = add_pos(m, g, m->pos, d, T, e.pos_qk, 2 * d);
      CK(run_gemm(m, "gemm.enc.qk", g, mode, s));
    }
    {
      GemmArgs g = linear_args(e.v, P(w.src), d, Mt, P(w.vt), 8);
      g.vt_T = T; g.vt_B = B; g.vt_swz = vt_swz;
      // the attention output is a convex combination of V rows: max |V| bounds it
      g.amax_a = src_amax; g.amax_c = tam ? tam + 2 * li : nullptr;
      g.out_f16 = f16attn || f16v;
      if (presplit) g.S = P(w.vt);               // hi plane then lo plane, in the fp32 V^T's bytes
      if (split_swz) g.vt_swz = 1;
      if (split_f16) { g.s_f16 = 1; g.s_l1 = e.v.l1max; g.s_bmax = e.v.bmax; }
      CK(run_gemm(m, "gemm.enc.v", g, GEMM_LINEAR, s));
    }
    {
      AttnArgs a{};
      a.q = P(w.qkv); a.ldq = 3 * d;
      a.k = presplit ? P(w.kpl) : (char*)P(w.qkv) + d * m->esz; a.ldk = presplit ? d : 3 * d;
      a.presplit = presplit;
      a.vt = P(w.vt); a.vt_swz = vt_swz || split_swz;
      if (split_f16) { a.v_f16 = 1; a.v_amax = src_amax; a.v_l1 = e.v.l1max; a.v_bmax = e.v.bmax; }
      a.o = P(w.ao); a.ldo = d;
      a.B = B; a.H = c.nheads; a.Tq = T; a.Tk = T; a.scale = scale;
      CK(run_attn(m, "attn.enc", a, attn_dt, s));
    }
    {
      // out-proj + residual; bf16 large batches fuse norm1 into the GEMM epilogue, in place over src
      GemmArgs g = linear_args(e.o, P(w.ao), d, Mt, P(w.tmp), d);
      g.R = P(w.src); g.ldr = d;
      g.amax_a = tam ? tam + 2 * li : nullptr;
      GemmArgs gf = g;
      gf.C = P(w.src); gf.ln_g = e.n1g; gf.ln_b = e.n1b;
      // (fp32h3 runs the persistent GEMM + the LayerNorm kernel: 0.15 + 0.06 ms a layer against 0.31 ms
      // for the fused 256-wide h3 tile with a LayerNorm epilogue, which ended every tile cold; removed)
      if (m->esz == 2 && spe_ln_fusable(gf)) {
        CK(run_gemm(m, "gemm.enc.o", gf, GEMM_LINEAR, s));
      } else {
        CK(run_gemm(m, "gemm.enc.o", g, GEMM_LINEAR, s));
        CK(run_other(m, "ln.enc", 0.0, (double)Mt * d * 2 * m->esz, s, [&] { return spe_launch_layernorm(P(w.tmp), e.n1g, e.n1b, P(w.src), nullptr, Mt, d, dt, s); }));
      }
      src_amax = e.n1_bound;
    }
    if (use_fused_ffn(m)) {
      // the last layer also emits memory + pos for the cross-K projection (xattn adds pos itself)
      const bool last = &e == &m->enc.back();
      CK(run_ffn(m, "ffn.enc", e.l1, e.l2, e.n2g, e.n2b, P(w.src), Mt, s, last ? m->pos : nullptr,
                 last ? P(w.srcpos) : nullptr, T, nullptr, e.ffn_w2c));
    } else if (m->h3 && e.ffn_w2p && src_amax && m->wh3.count(e.l1.w)) {
      // fp32h3: linear1 + ReLU + linear2 + residual + norm2 in one pass, in place over src
      FfnH3Args a{};
      a.x = (const float*)P(w.src); a.ldx = d; a.y = (float*)P(w.src); a.ldy = d;
      a.M = Mt; a.D = d; a.F = ff;
      a.w1 = m->wh3.at(e.l1.w).planes; a.ld1 = e.l1.Kpad; a.meta1 = e.ffn_meta1;
      a.w2 = e.ffn_w2p; a.ld2 = ff; a.sinv2 = m->wh3.at(e.l2.w).sinv; a.b2 = e.l2.bias;
      a.gamma = e.n2g; a.beta = e.n2b;
      a.amax_x = src_amax; a.sh = e.ffn_sh;
      const double fl = 4.0 * Mt * (double)d * ff, by = 2.0 * Mt * d * 4.0 + 2.0 * 2.0 * 2.0 * d * ff;
      CK(ledger_use(a.amax_x, nullptr, "ffn.enc"));
      CK(run_other(m, "ffn.enc", fl, by, s, [&] { return spe_launch_ffn_h3(a, s); }));
    } else {
      {
        GemmArgs g = linear_args(e.l1, P(w.src), d, Mt, P(w.ffn), ff);
        g.act = ACT_RELU;
        g.amax_a = src_amax; g.amax_c = tam ? tam + 2 * li + 1 : nullptr;
        CK(run_gemm(m, "gemm.enc.ffn1", g, GEMM_LINEAR, s));
      }
      {
        GemmArgs g = linear_args(e.l2, P(w.ffn), ff, Mt, P(w.tmp), d);
        g.R = P(w.src); g.ldr = d;
        g.amax_a = tam ? tam + 2 * li + 1 : nullptr;
        // (fp32h3 likewise: the persistent GEMM + LayerNorm, 0.65 + 0.06 against 0.85 ms fused)
        CK(run_gemm(m, "gemm.enc.ffn2", g, GEMM_LINEAR, s));
        CK(run_other(m, "ln.enc", 0.0, (double)Mt * d * 2 * m->esz, s, [&] { return spe_launch_layernorm(P(w.tmp), e.n2g, e.n2b, P(w.src), nullptr, Mt, d, dt, s); }));
      }
    }
    src_amax = e.n2_bound;
    ++li;
  }
  if (tam && 2 * li > SPE_AMAX_DEC - SPE_AMAX_BB - 1) return fail(SPE_E_STATE, "fp32h3: encoder activation-scale slots exhausted");
  // memory = src.  Unless the layers attend to memory + pos / memory directly (xattn path),
  // project the cross-attention K (memory + pos) and V^T (memory) for all decoder layers.
  if (xa && m->h3) {
    // fp32h3: the memory once as fp16 planes for all decoder layers (xattn_h3.hip): key planes of
    // memory + pos into srcpos, value planes into xvp
    CK(ledger_use(src_amax, nullptr, "eltwise.xsplit"));
    CK(run_other(m, "eltwise.xsplit", 0.0, (double)Mt * d * (4 + 4 + 4) + (double)T * d * 4, s, [&] {
      return spe_launch_xattn_h3_split((const float*)P(w.src), (const float*)m->pos, src_amax, P(w.srcpos), P(w.xvp), B, T, s);
    }));
  }
  if (!xa) {
  {
    // bf16 fused path: the last FFN wrote memory + pos (rounded once, like the reference's
    // fp32 add) -> plain GEMM; its 8 MB pos.W^T table would not stay L2-resident
    const bool have_srcpos = use_fused_ffn(m) && !m->enc.empty();
    GemmArgs g = linear_args(m->crossK, P(have_srcpos ? w.srcpos : w.src), d, Mt, P(w.ck), L * d);
    const int mode = have_srcpos ? GEMM_LINEAR : add_pos(m, g, m->pos, d, T, m->pos_crossK, L * d);
    if (!have_srcpos) g.amax_a = src_amax;
    CK(run_gemm(m, "gemm.cross_kv", g, mode, s));
  }
  {
    GemmArgs g = linear_args(m->crossV, P(w.src), d, Mt, P(w.cvt), 8);
    g.vt_T = T; g.vt_B = B;
    g.amax_a = src_amax; g.amax_c = amx ? amx + SPE_AMAX_DEC - 1 : nullptr;   // bounds every cross-attention output
    CK(run_gemm(m, "gemm.cross_kv", g, GEMM_LINEAR, s));
  }
  }

  }  // SPE_STAGE_TRANSFORMER
  if (!(stages & SPE_STAGE_DECODE)) return 0;

  // ---------------- decoder (REV/models/transformer.py:100-129,218-239)
  // (reads only the memory -- src, srcpos, or ck / cvt -- that the encode stage left in the
  // workspace, so the two stages may run on different streams, e.g. batch i's decoder beside
  // batch i+1's backbone with two workspaces)
  const int Mq = B * Q;
  CK((int)hipMemsetAsync(P(w.tgt), 0, (size_t)Mq * d * m->esz, s));
  // fp32h3 decoder scales: tgt's from its LayerNorm bounds (zeros before the first layer: any scale
  // serves), the attention outputs' from their V (self: the sv GEMM's published maximum; cross: the
  // crossV GEMM's, transformer stage), the FFN hidden's from the linear1 GEMM
  float* const dam = amx ? amx + SPE_AMAX_DEC : nullptr;
  if (dam) CK((int)hipMemsetAsync(dam, 0, (SPE_AMAX_SLOTS - SPE_AMAX_DEC) * 4, s));
  if (dam) ledger_scope.ledger.zeroed(SPE_AMAX_DEC, SPE_AMAX_SLOTS - SPE_AMAX_DEC);
  if (dam && 3 * L > SPE_AMAX_SLOTS - SPE_AMAX_DEC) return fail(SPE_E_STATE, "fp32h3: decoder activation-scale slots exhausted");
  // fp32h3 cross-attention against the memory: the memory's bound (the last encoder norm2's) scales
  // its planes; layer l's output raises slot dam + 2L + l
  const float* const mem_bound = m->h3 && xa && !m->enc.empty() ? m->enc.back().n2_bound : nullptr;
  const float* tgt_amax = m->h3 && L > 0 ? m->dec[0].n1_bound : nullptr;
  const float* const cross_v_amax = amx ? amx + SPE_AMAX_DEC - 1 : nullptr;
  // tgt = LayerNorm(tgt + dao . W^T + b) (REV/models/transformer.py:227-228, 233-234) as GEMM +
  // LayerNorm: at these few rows (B.Q) lnproj's one-workgroup-per-8-tiles form measured slower
  // (24 vs 18 us a layer: 6 workgroups each staging all of W)
  static const bool decproj_on = [] { const char* e = getenv("SPE_DECPROJ"); return e ? atoi(e) != 0 : true; }();
  auto dec_proj_ln = [&](const Conv& wo, const void* fwo, const float* lg, const float* lb, const float* x_amax) -> int {
    if (decproj_on && fwo && Q <= 64) {
      // bf16: one workgroup per image, the rows in LDS from the GEMM to the LayerNorm (decsa.hip)
      DecProjArgs pa{};
      pa.tgt = P(w.tgt); pa.ldt = d; pa.x = P(w.dao); pa.ldx = d; pa.B = B; pa.Q = Q;
      pa.wo = fwo; pa.bo = wo.bias; pa.g = lg; pa.b = lb;
      CK(run_other(m, "dec.proj", 2.0 * Mq * d * d, 3.0 * Mq * d * m->esz + (double)d * d * m->esz, s,
                   [&] { return spe_launch_decproj(pa, s); }));
      return 0;
    }
    GemmArgs g = linear_args(wo, P(w.dao), d, Mq, P(w.dtmp), d);
    g.R = P(w.tgt); g.ldr = d;
    g.amax_a = x_amax;
    CK(run_gemm(m, "gemm.dec", g, GEMM_LINEAR, s));
    CK(run_other(m, "ln.dec", 0.0, (double)Mq * d * 2 * m->esz, s, [&] { return spe_launch_layernorm(P(w.dtmp), lg, lb, P(w.tgt), nullptr, Mq, d, dt, s); }));
    return 0;
  };
  // bf16: the self-attention block (projections, attention, out-projection, norm1) as one
  // launch per layer (decsa.hip); SPE_DECSA=0 runs the separate launches for A/B runs
  static const bool decsa_on = [] { const char* e = getenv("SPE_DECSA"); return e ? atoi(e) != 0 : true; }();
  // bf16: the decoder FFN and the cross-attention's query projection as decsa.hip's 16-row kernels;
  // SPE_DECFFN=0 runs ffn.hip's FFN and the GEMM for A/B runs
  static const bool decffn_on = [] { const char* e = getenv("SPE_DECFFN"); return e ? atoi(e) != 0 : true; }();
  for (int l = 0; l < L; ++l) {
    const Dec& e = m->dec[l];
    const bool sa_fused = decsa_on && e.fsqk && c.nheads == 8 && Q <= 64 && e.qpos_sqk;
    if (sa_fused) {
      DecSaArgs sa{};
      sa.tgt = P(w.tgt); sa.ldt = d; sa.B = B; sa.Q = Q;
      sa.wqk = e.fsqk; sa.bqk = e.sqk.bias;
      sa.wv = e.fsv; sa.bv = e.sv.bias;
      sa.qpos = e.qpos_sqk;
      sa.wo = e.fso; sa.bo = e.so.bias;
      sa.g = e.n1g; sa.b = e.n1b; sa.scale = scale;
      const double fl = 2.0 * Mq * d * (4.0 * d) + 4.0 * B * 8.0 * Q * Q * 32;
      const double by = 2.0 * Mq * d * m->esz + 4.0 * d * d * m->esz;
      CK(run_other(m, "dec.self", fl, by, s, [&] { return spe_launch_decsa(sa, s); }));
    } else {
    {
      GemmArgs g = linear_args(e.sqk, P(w.tgt), d, Mq, P(w.dqkv), 3 * d);
      const int mode = add_pos(m, g, m->qpos, d, Q, e.qpos_sqk, 2 * d);
      g.amax_a = tgt_amax;
      CK(run_gemm(m, "gemm.dec", g, mode, s));
    }
    {
      GemmArgs g = linear_args(e.sv, P(w.tgt), d, Mq, P(w.dvt), 8);
      g.vt_T = Q; g.vt_B = B;
      g.amax_a = tgt_amax; g.amax_c = dam ? dam + 2 * l : nullptr;
      CK(run_gemm(m, "gemm.dec", g, GEMM_LINEAR, s));
    }
    {
      AttnArgs a{};
      a.q = P(w.dqkv); a.ldq = 3 * d;
      a.k = (char*)P(w.dqkv) + d * m->esz; a.ldk = 3 * d;
      a.vt = P(w.dvt);
      a.o = P(w.dao); a.ldo = d;
      a.B = B; a.H = c.nheads; a.Tq = Q; a.Tk = Q; a.scale = scale;
      CK(run_attn(m, "attn.dec_self", a, dt, s));
    }
    CK(dec_proj_ln(e.so, e.fso, e.n1g, e.n1b, dam ? dam + 2 * l : nullptr));
    }
    if (m->h3) tgt_amax = e.n1_bound;
    bool xtail = false;                         // the merge + value + out-projection + norm2 ran in one launch
    const float* cross_o_amax = cross_v_amax;   // fp32h3: the out-projection's scale input
    if (xa) {
      // q' = (tgt + query_pos) . Wqk^T + bqk: the query-side fold of Wq and Wk (xattn.hip)
      if (e.fxq && decffn_on) {
        // (16 rows, 256 columns) workgroups over the packed weights (decsa.hip)
        DecQArgs qa{};
        qa.x = P(w.tgt); qa.ldx = d; qa.M = Mq; qa.N = 8 * d;
        qa.w = e.fxq; qa.bias = e.xq.bias; qa.R = e.xq_r; qa.ldr = 8 * d; qa.period = Q;
        qa.y = P(w.xq); qa.ldy = 8 * d;
        CK(run_other(m, "gemm.dec", 2.0 * Mq * d * 8.0 * d, 2.0 * Mq * (d + 8.0 * d) * m->esz + 2.0 * 8 * d * d * m->esz, s,
                     [&] { return spe_launch_decq(qa, s); }));
      } else {
        GemmArgs g = linear_args(e.xq, P(w.tgt), d, Mq, P(w.xq), 8 * d);
        g.R = e.xq_r; g.ldr = 8 * d; g.r_period = Q;
        g.amax_a = tgt_amax;                    // fp32h3: the h3 GEMM's scale input
        CK(run_gemm(m, "gemm.dec", g, GEMM_LINEAR, s));
      }
      if (m->h3) {
        // fp32h3: scores and value sums against the memory's fp16 planes, three products each; the
        // merge applies Wv / bv in fp32 and raises max |o| for the out-projection
        XattnArgs x{};
        x.q = P(w.xq); x.ldq = 8 * d;
        x.k = P(w.srcpos); x.ldk = 2 * d;
        x.v = P(w.xvp); x.ldv = 2 * d;
        x.wv = e.xv.w; x.bv = e.xv.bias;
        x.o = P(w.dao); x.ldo = d;
        x.B = B; x.Q = Q; x.T = T; x.splits = spe_xattn_splits(B, Q, T);
        x.pm = (float*)P(w.xpm); x.pl = (float*)P(w.xpl); x.pu = (float*)P(w.xpu);
        x.mem_amax = mem_bound; x.o_amax = dam ? dam + 2 * L + l : nullptr;
        const double fl = 4.0 * B * 8.0 * Q * (double)T * d + 2.0 * Mq * 8.0 * d * 32;
        const double by = 2.0 * B * (double)T * 2 * d * 2 + 2.0 * Mq * 8.0 * d * 4;
        CK(ledger_use(x.mem_amax, x.o_amax, "attn.dec_cross"));
        CK(run_other(m, "attn.dec_cross", fl, by, s, [&] { return spe_launch_xattn_h3(x, s); }));
        cross_o_amax = x.o_amax;
      } else {
        XattnArgs x{};
        x.q = P(w.xq); x.ldq = 8 * d;
        x.k = P(w.srcpos); x.ldk = d;
        x.v = P(w.src); x.ldv = d;
        x.wv = e.xv.w; x.bv = e.xv.bias;
        x.o = P(w.dao); x.ldo = d;
        x.B = B; x.Q = Q; x.T = T; x.splits = spe_xattn_splits(B, Q, T);
        x.pm = (float*)P(w.xpm); x.pl = (float*)P(w.xpl); x.pu = (float*)P(w.xpu);
        // Q <= 48: the split merge and the value projection move into the out-projection + norm2
        // launch (decsa.hip decxproj_kernel), the per-split partials its only input
        xtail = decproj_on && e.fxv && Q <= 48;
        x.partials_only = xtail;
        const double fl = 4.0 * B * 8.0 * Q * (double)T * d + (xtail ? 0.0 : 2.0 * Mq * 8.0 * d * 32);
        const double by = 2.0 * B * (double)T * d * m->esz + 2.0 * Mq * 8.0 * d * m->esz;
        CK(run_other(m, "attn.dec_cross", fl, by, s, [&] { return spe_launch_xattn(x, s); }));
        if (xtail) {
          DecProjArgs pa{};
          pa.tgt = P(w.tgt); pa.ldt = d; pa.B = B; pa.Q = Q;
          pa.wo = e.fco; pa.bo = e.co.bias; pa.g = e.n2g; pa.b = e.n2b;
          pa.pm = x.pm; pa.pl = x.pl; pa.pu = x.pu; pa.splits = spe_xattn_launch_splits(T, x.splits);
          pa.wv = e.fxv; pa.bv = e.xv.bias;
          const double pfl = 2.0 * Mq * 8.0 * d * 32 + 2.0 * Mq * d * d;
          const double pby = (double)pa.splits * B * 8.0 * Q * (d + 2) * 4 + 2.0 * Mq * d * m->esz + 2.0 * d * d * m->esz;
          CK(run_other(m, "dec.xproj", pfl, pby, s, [&] { return spe_launch_decproj(pa, s); }));
        }
      }
    } else {
    {
      GemmArgs g = linear_args(e.cq, P(w.tgt), d, Mq, P(w.dqc), d);
      const int mode = add_pos(m, g, m->qpos, d, Q, e.qpos_cq, d);
      g.amax_a = tgt_amax;
      CK(run_gemm(m, "gemm.dec", g, mode, s));
    }
    {
      AttnArgs a{};
      a.q = P(w.dqc); a.ldq = d;
      a.k = (char*)P(w.ck) + (size_t)l * d * m->esz; a.ldk = L * d;
      a.vt = (char*)P(w.cvt) + (size_t)l * B * d * T * m->esz;
      a.o = P(w.dao); a.ldo = d;
      a.B = B; a.H = c.nheads; a.Tq = Q; a.Tk = T; a.scale = scale;
      CK(run_attn(m, "attn.dec_cross", a, dt, s));
    }
    }
    if (!xtail) CK(dec_proj_ln(e.co, e.fco, e.n2g, e.n2b, cross_o_amax));
    if (m->h3) tgt_amax = e.n2_bound;
    if (e.fl1 && decffn_on) {
      // bf16: one workgroup per (16 rows, 256 hidden units), all of its weight fragments in flight
      // from the start (decsa.hip), then ffn.hip's split-F reduce + norm3
      DecFfnArgs fa{};
      fa.x = P(w.tgt); fa.ldx = d; fa.M = Mq; fa.F = ff;
      fa.w1 = e.fl1; fa.b1 = e.l1.bias; fa.w2 = e.fl2; fa.partial = (float*)P(w.dffnpart);
      FfnArgs ra{};
      ra.x = P(w.tgt); ra.ldx = d; ra.y = P(w.tgt); ra.ldy = d; ra.M = Mq; ra.D = d; ra.F = ff;
      ra.b2 = e.l2.bias; ra.gamma = e.n3g; ra.beta = e.n3b; ra.splits = ff / 256; ra.partial = fa.partial;
      const double fl = 4.0 * Mq * (double)d * ff;
      const double by = 2.0 * Mq * d * m->esz + 2.0 * (double)d * ff * m->esz + 2.0 * ra.splits * Mq * d * 4;
      CK(run_other(m, "ffn.dec", fl, by, s, [&] {
        const int rc = spe_launch_decffn(fa, s);
        return rc ? rc : spe_launch_ffn_reduce_ln(ra, s);
      }));
    } else if (use_fused_ffn(m)) {
      CK(run_ffn(m, "ffn.dec", e.l1, e.l2, e.n3g, e.n3b, P(w.tgt), Mq, s, nullptr, nullptr, 0,
                 (float*)P(w.dffnpart)));
    } else {
      {
        GemmArgs g = linear_args(e.l1, P(w.tgt), d, Mq, P(w.dffn), ff);
        g.act = ACT_RELU;
        g.amax_a = tgt_amax; g.amax_c = dam ? dam + 2 * l + 1 : nullptr;
        CK(run_gemm(m, "gemm.dec", g, GEMM_LINEAR, s));
      }
      {
        GemmArgs g = linear_args(e.l2, P(w.dffn), ff, Mq, P(w.dtmp), d);
        g.R = P(w.tgt); g.ldr = d;
        g.amax_a = dam ? dam + 2 * l + 1 : nullptr;
        CK(run_gemm(m, "gemm.dec", g, GEMM_LINEAR, s));
      }
      CK(run_other(m, "ln.dec", 0.0, (double)Mq * d * 2 * m->esz, s, [&] { return spe_launch_layernorm(P(w.dtmp), e.n3g, e.n3b, P(w.tgt), nullptr, Mq, d, dt, s); }));
    }
    if (m->h3) tgt_amax = e.n3_bound;
    if (out->aux_logits && out->aux_points && l + 1 < L) {
      // aux output of layer l: the shared decoder_norm (REV/models/transformer.py:117-124) and
      // the same heads (REV/models/detr_speed.py:83-99), into the aux slices
      float* hs_aux = (float*)P(w.hs);
      CK(run_other(m, "ln.dec", 0.0, (double)Mq * d * (m->esz + 4), s, [&] { return spe_launch_layernorm(P(w.tgt), m->dng, m->dnb, nullptr, hs_aux, Mq, d, dt, s); }));
      HeadArgs ha = m->head;
      ha.hs = hs_aux; ha.B = B; ha.Q = Q;
      ha.clip_bbox = nullptr; ha.probs = nullptr; ha.points_px = nullptr;
      ha.log_sigmas = nullptr; ha.sigmas = nullptr;
      ha.logits = out->aux_logits + (size_t)l * Mq * 12;
      ha.points = out->aux_points + (size_t)l * Mq * 2;
      CK(run_other(m, "heads", 0.0, (double)Mq * d * 4, s, [&] { return spe_launch_heads(ha, s); }));
    }
  }
  float* hs = out->hs ? out->hs : (float*)P(w.hs);
  CK(run_other(m, "ln.dec", 0.0, (double)Mq * d * (m->esz + 4), s, [&] { return spe_launch_layernorm(P(w.tgt), m->dng, m->dnb, nullptr, hs, Mq, d, dt, s); }));

  // ---------------- heads + PostProcess (REV/models/detr_speed.py:83-92,266-293)
  HeadArgs h = m->head;
  h.hs = hs; h.B = B; h.Q = Q;
  h.clip_bbox = out->clip_bbox;
  h.logits = out->logits; h.points = out->points;
  h.probs = out->clip_bbox ? out->probs : nullptr;
  h.points_px = out->clip_bbox ? out->points_px : nullptr;
  h.log_sigmas = out->log_sigmas; h.sigmas = out->sigmas;
  if (!c.sigma_head) { h.log_sigmas = nullptr; h.sigmas = nullptr; }
  CK(run_other(m, "heads", 0.0, (double)Mq * d * 4, s, [&] { return spe_launch_heads(h, s); }));
  return 0;
}

// Device scratch of the solver's RANSAC hypothesis records and the criterion's per-image partial
// sums: one buffer per (device, stream, kind), grown on demand and kept for the process lifetime,
// so steady-state calls allocate nothing (a first call with a larger batch allocates and must
// therefore happen outside graph capture).  Keying by stream is what makes concurrent calls safe:
// calls on one stream are ordered by the stream, calls on different streams never share records.
// A stream handle that is destroyed while its work is pending and then reissued by the runtime
// would inherit the buffer; callers keep solver streams alive for as long as they use them.
static void* stream_scratch(hipStream_t stream, int kind, size_t bytes) {
  static std::mutex mu;
  static std::map<std::tuple<int, hipStream_t, int>, std::pair<void*, size_t>> bufs;
  int dev = 0;
  if (hipGetDevice(&dev) != hipSuccess) return nullptr;
  std::lock_guard<std::mutex> g(mu);
  auto& e = bufs[std::make_tuple(dev, stream, kind)];
  if (e.second < bytes) {
    // the old buffer may still be read by work queued on this stream: free it in stream order
    if (e.first) {
      if (hipStreamSynchronize(stream) != hipSuccess) return nullptr;
      (void)hipFree(e.first);
    }
    e.first = nullptr;
    e.second = 0;
    if (hipMalloc(&e.first, bytes) != hipSuccess) return nullptr;
    e.second = bytes;
  }
  return e.first;
}
enum { SCRATCH_CRITERION = 0, SCRATCH_HYP = 1 };

int spe_criterion(void* stream, const float* logits, const float* points, const int32_t* tgt_labels,
                  const float* tgt_points, int layers, int batch, int num_queries, int num_classes, int num_targets,
                  float cost_class, float cost_pts, float eos_coef, double num_points, int32_t* match, double* losses) {
  if (!logits || !points || !tgt_labels || !tgt_points || !match || !losses || layers < 1 || batch < 0 ||
      num_queries < 1 || num_queries > 64 || num_targets < 1 || num_targets > 32 || num_targets > num_queries ||
      num_classes < 2 || num_classes > 32 || !(num_points > 0))
    return fail(SPE_E_ARG, "bad argument");
  CritArgs a{logits, points, tgt_labels, tgt_points, layers, batch, num_queries, num_classes, num_targets,
             cost_class, cost_pts, eos_coef, num_points, match, nullptr, losses};
  if (batch > 0) {
    a.partial = (double*)stream_scratch((hipStream_t)stream, SCRATCH_CRITERION, (size_t)layers * batch * 5 * sizeof(double));
    if (!a.partial) return fail(SPE_E_LAUNCH, "criterion scratch allocation failed");
  }
  CK(spe_launch_criterion(a, (hipStream_t)stream));
  return 0;
}

int spe_ensemble_fuse(void* stream, const float* points_px, const float* probs, int models, int batch,
                      int num_queries, int num_classes, float* fused_points, float* fused_probs) {
  if (!points_px || !probs || !fused_points || !fused_probs || models < 1 || batch < 0 || num_queries < 1 ||
      num_classes < 2 || num_classes > 17 || (int64_t)models * num_queries > 256)
    return fail(SPE_E_ARG, "bad argument");
  EnsembleArgs a{points_px, probs, models, batch, num_queries, num_classes, fused_points, fused_probs};
  CK(spe_launch_ensemble_fuse(a, (hipStream_t)stream));
  return 0;
}

int spe_preprocess(void* stream, const uint8_t* frames, int batch, int height, int width, int channels,
                   const double* bbox_xxyy, int size, float* images, float* clip_bbox, int32_t* status) {
  if (!frames || !bbox_xxyy || !images || !clip_bbox || batch < 0 || height <= 0 || width <= 0 || size <= 0 ||
      (channels != 1 && channels != 3))
    return fail(SPE_E_ARG, "bad argument");
  CK(spe_launch_preprocess(frames, batch, height, width, channels, bbox_xxyy, size, images, clip_bbox, status,
                           (hipStream_t)stream));
  return 0;
}

int spe_postprocess(void* stream, const float* logits, const float* points, const float* clip_bbox, int B, int Q,
                    float* probs, float* points_px) {
  if (!logits || !points || !clip_bbox || !probs || !points_px || B < 0 || Q <= 0) return fail(SPE_E_ARG, "bad argument");
  CK(spe_launch_postprocess(logits, points, clip_bbox, B, Q, probs, points_px, (hipStream_t)stream));
  return 0;
}

int spe_pnp_batch(void* stream, const float* points_px, const float* probs, const float* sigmas, int B, int Q, int C,
                  const double* K, const double* world, int mode, float repro, int ransac_iters, double confidence,
                  float* quat, double* tvec, double* rvec, int32_t* status, int32_t* n_corr, int32_t* corr_label,
                  uint32_t* inlier_mask, const float* repro_per_image) {
  if (!points_px || !probs || !K || !world || !quat || !tvec || B < 0 || Q <= 0 || Q > 64 || C < 2 || C > 17)
    return fail(SPE_E_ARG, "bad argument");
  if (mode < SPE_PNP_EPNP || mode > SPE_PNP_EPNP_CERES) return fail(SPE_E_ARG, "bad solver mode");
  if (ransac_iters < 1 || ransac_iters > 255 || !(confidence > 0 && confidence < 1))
    return fail(SPE_E_ARG, "ransac_iters must be in [1,255], confidence in (0,1)");
  PnpArgs a{};
  a.points = points_px; a.probs = probs; a.sigmas = sigmas;
  a.B = B; a.Q = Q; a.C = C; a.K = K; a.world = world; a.mode = mode; a.repro = repro;
  a.repro_img = repro_per_image;
  a.ransac_iters = ransac_iters; a.confidence = confidence;
  a.quat = quat; a.tvec = tvec; a.rvec = rvec; a.status = status; a.n_corr = n_corr;
  a.corr_label = corr_label; a.inlier_mask = inlier_mask;
  if (mode == SPE_PNP_EPNP_RANSAC_SIGMA && B > 0) {
    a.hyp = (HypRec*)stream_scratch((hipStream_t)stream, SCRATCH_HYP, (size_t)B * ransac_iters * sizeof(HypRec));
    a.hyp_stride = ransac_iters;
    if (!a.hyp) return fail(SPE_E_LAUNCH, "hypothesis scratch allocation failed");
  }
  CK(spe_launch_pnp(a, (hipStream_t)stream));
  return 0;
}

int spe_self_assess(void* stream, const float* probs, const float* sigmas, const int32_t* status,
                    const int32_t* corr_label, const uint32_t* inlier_mask, int B, int Q, int C, float score_th,
                    float sigma_th, int min_inliers, float* mean_sigma, int32_t* n_confident, uint8_t* reliable) {
  if (!probs || !sigmas || !status || !corr_label || !inlier_mask || !mean_sigma || !n_confident || !reliable || B < 0 ||
      Q <= 0 || Q > 64 || C < 2 || C > 17 || min_inliers < 0)
    return fail(SPE_E_ARG, "bad argument");
  SelfAssessArgs a{probs, sigmas, status, corr_label, inlier_mask, B, Q, C, score_th, sigma_th, min_inliers,
                   mean_sigma, n_confident, reliable};
  CK(spe_launch_self_assess(a, (hipStream_t)stream));
  return 0;
}

int spe_speed_score(void* stream, const float* quat, const double* tvec, const double* q_gt, const double* t_gt, int B,
                    double* s_t, double* s_q) {
  if (!quat || !tvec || !q_gt || !t_gt || !s_t || !s_q || B < 0) return fail(SPE_E_ARG, "bad argument");
  CK(spe_launch_score(quat, tvec, q_gt, t_gt, B, s_t, s_q, (hipStream_t)stream));
  return 0;
}

int spe_model_profile_begin(spe_model* m, const char* kind_prefix) {
  if (!m) return fail(SPE_E_ARG, "null model");
  m->prof.on = true;
  m->prof.filter = kind_prefix ? kind_prefix : "";
  m->prof.recs.clear();
  m->prof.next_event = 0;
  return 0;
}

int spe_model_profile_end(spe_model* m) {
  if (!m) return fail(SPE_E_ARG, "null model");
  m->prof.on = false;
  for (auto& r : m->prof.recs) {
    hipError_t e = hipEventSynchronize(r.end);
    if (e != hipSuccess) return fail((int)e, "profile event sync failed");
  }
  return (int)m->prof.recs.size();
}

int spe_model_profile_get(const spe_model* m, int i, char* kind, int kind_len, double* ms, double* flops,
                          double* bytes) {
  if (!m || i < 0 || i >= (int)m->prof.recs.size()) return fail(SPE_E_ARG, "bad profile record index");
  const ProfRecord& r = m->prof.recs[i];
  if (kind && kind_len > 0) {
    std::strncpy(kind, r.kind.c_str(), kind_len - 1);
    kind[kind_len - 1] = 0;
  }
  float t = 0.f;
  hipError_t e = hipEventElapsedTime(&t, r.beg, r.end);
  if (e != hipSuccess) return fail((int)e, "hipEventElapsedTime failed");
  if (ms) *ms = t;
  if (flops) *flops = r.flops;
  if (bytes) *bytes = r.bytes;
  return 0;
}

}  // extern "C"
