// Kernel-level test hooks (declared in include/spe.h, "kernel test hooks"): thin C entry points
// that launch one kernel family on caller-provided device buffers, so tests/ can check each
// kernel against a plain torch reference of the same op at awkward shapes (edges, ragged
// tiles, strides) — the forward pass alone would hide a wrong-but-normalised intermediate.
#include <hip/hip_runtime.h>

#include "../../include/spe.h"
#include "model_state.h"

namespace {
thread_local const void* g_planes = nullptr;   // spe_debug_gemm_planes -> spe_debug_gemm
thread_local int g_plane_rows = 0;
}  // namespace

extern "C" {

int spe_debug_gemm(void* stream, int dtype, int mode, const void* A, int lda, const void* P, int ldp, int prow,
                   int H, int W, int Cin, int KH, int KW, int stride, int pad, const void* Bw, int ldb, int M, int N,
                   int K, const float* bias, const void* R, int ldr, int act_code, void* C, int ldc, int out_f32, int vt_T,
                   int vt_B, int r_period, const float* ln_g, const float* ln_b, int out_f16) {
  GemmArgs g{};
  g.A = A; g.lda = lda; g.P = P; g.ldp = ldp; g.prow = prow;
  g.H = H; g.W = W; g.Cin = Cin; g.KH = KH; g.KW = KW; g.stride = stride; g.pad = pad;
  g.Ho = mode == GEMM_CONV ? (H + 2 * pad - KH) / stride + 1 : 0;
  g.Wo = mode == GEMM_CONV ? (W + 2 * pad - KW) / stride + 1 : 0;
  g.B = Bw; g.ldb = ldb; g.M = M; g.N = N; g.K = K;
  g.bias = bias; g.R = R; g.ldr = ldr; g.act = act_code & 255; g.res_post = (act_code >> 8) & 1; g.C = C; g.ldc = ldc; g.out_f32 = out_f32;
  g.vt_swz = (act_code >> 9) & 1;
  g.vt_T = vt_T; g.vt_B = vt_B;
  g.r_period = r_period;
  g.ln_g = ln_g; g.ln_b = ln_b;
  g.out_f16 = out_f16;
  g.B6 = g_planes;
  g.b6_rows = g_plane_rows;
  int rc = spe_launch_gemm(g, dtype, mode, (hipStream_t)stream);
  return rc < 0 ? spe_fail(SPE_E_LAUNCH, "gemm launch rejected its arguments") : rc;
}

int spe_debug_gemm_planes(void* stream, int dtype, int mode, const void* A, int lda, const void* P, int ldp, int prow,
                          int H, int W, int Cin, int KH, int KW, int stride, int pad, const void* Bw, int ldb, int M,
                          int N, int K, const float* bias, const void* R, int ldr, int act_code, void* C, int ldc,
                          const void* planes, int plane_rows) {
  g_planes = planes;
  g_plane_rows = plane_rows;
  const int rc = spe_debug_gemm(stream, dtype, mode, A, lda, P, ldp, prow, H, W, Cin, KH, KW, stride, pad, Bw, ldb, M, N,
                                K, bias, R, ldr, act_code, C, ldc, 0, 0, 0, 0, nullptr, nullptr, 0);
  g_planes = nullptr;
  g_plane_rows = 0;
  return rc;
}

int spe_debug_gemm_h3(void* stream, int mode, const void* A, int lda, int H, int W, int Cin, int KH, int KW, int stride,
                      int pad, int ldb, int M, int N, int K, const float* bias, const void* R, int ldr, int act_code,
                      void* C, int ldc, const void* planes, int plane_rows, const float* sinv, const float* amax_a,
                      float* amax_c, float amax_c_mul) {
  if (!A || !C || !planes || !sinv || M < 0 || N <= 0 || K <= 0) return spe_fail(SPE_E_ARG, "bad argument");
  GemmArgs g{};
  g.A = A; g.lda = lda;
  g.H = H; g.W = W; g.Cin = Cin; g.KH = KH; g.KW = KW; g.stride = stride; g.pad = pad;
  g.Ho = mode == GEMM_CONV ? (H + 2 * pad - KH) / stride + 1 : 0;
  g.Wo = mode == GEMM_CONV ? (W + 2 * pad - KW) / stride + 1 : 0;
  g.B = planes; g.ldb = ldb; g.M = M; g.N = N; g.K = K;
  g.bias = bias; g.R = R; g.ldr = ldr; g.act = act_code & 255; g.C = C; g.ldc = ldc;
  g.H3 = planes; g.h3_rows = plane_rows; g.h3_sinv = sinv; g.amax_a = amax_a; g.amax_c = amax_c;
  g.amax_c_mul = amax_c_mul;
  // (the h3 kernels only: through spe_launch_gemm an unserved shape would run the x6 kernel, which
  // reads the fp16 planes as fp32 weights)
  const int rc = spe_launch_gemm_h3(g, mode, (hipStream_t)stream);
  if (rc == 1) return spe_fail(SPE_E_LAUNCH, "shape not served by the fp32h3 kernel");
  return rc < 0 ? spe_fail(SPE_E_LAUNCH, "gemm launch rejected its arguments") : rc;
}

int spe_debug_gemm_path(void) { return spe_gemm_last_path; }

int spe_debug_ffn_h3(void* stream, const float* x, int ldx, float* y, int ldy, int M, int F, const void* w1, int ld1,
                     const float* meta1, const void* w2, int ld2, const float* sinv2, const float* b2,
                     const float* gamma, const float* beta, const float* amax_x, float sh) {
  FfnH3Args a{};
  a.x = x; a.ldx = ldx; a.y = y; a.ldy = ldy; a.M = M; a.D = 256; a.F = F;
  a.w1 = w1; a.ld1 = ld1; a.meta1 = meta1; a.w2 = w2; a.ld2 = ld2; a.sinv2 = sinv2; a.b2 = b2;
  a.gamma = gamma; a.beta = beta; a.amax_x = amax_x; a.sh = sh;
  const int rc = spe_launch_ffn_h3(a, (hipStream_t)stream);
  return rc < 0 ? spe_fail(SPE_E_ARG, "ffn_h3 launch rejected its arguments") : rc;
}

int spe_debug_ffn_h3_perm(int p) { return p >= 0 && p < 32 ? spe_ffn_h3_perm(p) : -1; }

int spe_debug_attention(void* stream, int dtype, const void* q, int ldq, const void* k, int ldk, const void* vt,
                        void* o, int ldo, int B, int H, int Tq, int Tk, float scale) {
  AttnArgs a{};
  a.q = q; a.ldq = ldq; a.k = k; a.ldk = ldk; a.vt = vt; a.o = o; a.ldo = ldo;
  a.B = B; a.H = H; a.Tq = Tq; a.Tk = Tk; a.scale = scale;
  a.vt_swz = (dtype >> 8) & 1;
  a.presplit = (dtype >> 9) & 1;
  a.v_f16 = (dtype >> 10) & 1;                     // (unscaled fp16 V^T planes: v_amax null)
  int rc = spe_launch_attention(a, dtype & 255, (hipStream_t)stream);
  return rc < 0 ? spe_fail(SPE_E_LAUNCH, "attention launch rejected its arguments") : rc;
}

int spe_debug_layernorm(void* stream, int dtype, const void* x, const float* gamma, const float* beta, void* out,
                        float* out_f32, int M, int D) {
  int rc = spe_launch_layernorm(x, gamma, beta, out, out_f32, M, D, dtype, (hipStream_t)stream);
  return rc < 0 ? spe_fail(SPE_E_LAUNCH, "layernorm launch rejected its arguments") : rc;
}

int spe_debug_ffn(void* stream, const void* x, int ldx, const void* w1, int ld1, const float* b1, const void* w2,
                  int ld2, const float* b2, const float* gamma, const float* beta, void* y, int ldy, int M, int D,
                  int F, float* partial, int splits) {
  FfnArgs a{};
  a.x = x; a.ldx = ldx; a.w1 = w1; a.ld1 = ld1; a.b1 = b1; a.w2 = w2; a.ld2 = ld2; a.b2 = b2;
  a.gamma = gamma; a.beta = beta; a.y = y; a.ldy = ldy; a.M = M; a.D = D; a.F = F;
  if (ld2 == 0) {                               // w2 chunk-packed [F/32][256][32] (the model's bf16 encoder form)
    a.w2_chunked = 1;
    a.ld2 = F;
  }
  a.partial = partial; a.splits = splits;
  int rc = spe_launch_ffn_ln(a, (hipStream_t)stream);
  return rc < 0 ? spe_fail(SPE_E_LAUNCH, "ffn launch rejected its arguments") : rc;
}

int spe_debug_upconv(void* stream, int dtype, const void* z, void* out, int ldo, int B, int H, int W, int C) {
  if (!z || !out || B < 0 || H < 1 || W < 1 || C < 1) return spe_fail(SPE_E_ARG, "bad argument");
  int rc = spe_launch_upconv_combine(z, out, ldo, B, H, W, C, dtype, (hipStream_t)stream);
  return rc < 0 ? spe_fail(SPE_E_LAUNCH, "upconv launch rejected its arguments") : rc;
}

int spe_debug_xattn(void* stream, const void* q, int ldq, const void* k, int ldk, const void* v, int ldv, void* u,
                    int ldu, const void* wv, const float* bv, void* o, int ldo, int B, int Q, int T, int splits,
                    float* partial_scratch) {
  XattnArgs a{};
  a.q = q; a.ldq = ldq; a.k = k; a.ldk = ldk; a.v = v; a.ldv = ldv; a.u = u; a.ldu = ldu;
  a.wv = wv; a.bv = bv; a.o = o; a.ldo = ldo;
  a.B = B; a.Q = Q; a.T = T; a.splits = splits > 0 ? splits : spe_xattn_splits(B, Q, T);
  const size_t rows = (size_t)a.splits * B * 8 * Q;
  a.pm = partial_scratch; a.pl = partial_scratch ? partial_scratch + rows : nullptr;
  a.pu = partial_scratch ? partial_scratch + 2 * rows : nullptr;
  const int rc = spe_launch_xattn(a, (hipStream_t)stream);
  return rc < 0 ? spe_fail(SPE_E_LAUNCH, "xattn launch rejected its arguments") : rc;
}

int spe_debug_xattn_h3(void* stream, const float* q, int ldq, const float* mem, const float* pos, const float* mem_amax,
                       const float* wv, const float* bv, float* o, int ldo, float* o_amax, int B, int Q, int T,
                       int splits, float* partial_scratch, void* plane_scratch) {
  if (!q || !mem || !pos || !mem_amax || !wv || !bv || !o || !partial_scratch || !plane_scratch || B < 0 || Q < 1 ||
      T < 1)
    return spe_fail(SPE_E_ARG, "bad argument");
  hipStream_t s = (hipStream_t)stream;
  char* kp = (char*)plane_scratch;
  char* vp = kp + (size_t)B * T * 1024;
  if (spe_launch_xattn_h3_split(mem, pos, mem_amax, kp, vp, B, T, s) != 0)
    return spe_fail(SPE_E_LAUNCH, "xattn_h3 split launch failed");
  XattnArgs a{};
  a.q = q; a.ldq = ldq; a.k = kp; a.ldk = 512; a.v = vp; a.ldv = 512;
  a.wv = wv; a.bv = bv; a.o = o; a.ldo = ldo;
  a.B = B; a.Q = Q; a.T = T; a.splits = splits > 0 ? splits : spe_xattn_splits(B, Q, T);
  const size_t rows = (size_t)a.splits * B * 8 * Q;
  a.pm = partial_scratch; a.pl = partial_scratch + rows; a.pu = partial_scratch + 2 * rows;
  a.mem_amax = mem_amax; a.o_amax = o_amax;
  const int rc = spe_launch_xattn_h3(a, s);
  return rc != 0 ? spe_fail(SPE_E_LAUNCH, "xattn_h3 launch rejected its arguments") : 0;
}

int spe_debug_btail(void* stream, const void* a, int lda, int k1, const void* r, const void* w3, int ld3,
                    const float* b3, void* y, const void* w1p, int ld1, const float* b1, void* z, int n2, int M) {
  if (!a || !w3 || !b3 || !y || !w1p || !b1 || !z || M < 0) return spe_fail(SPE_E_ARG, "bad argument");
  BtailArgs t{};
  t.A = a; t.lda = lda; t.k1 = k1; t.R = r; t.ldr = 256;
  t.w3 = w3; t.ld3 = ld3; t.b3 = b3; t.y = y; t.ldy = 256; t.n1 = 256;
  t.w1 = w1p; t.ld1 = ld1; t.b1 = b1; t.z = z; t.ldz = n2; t.n2 = n2; t.M = M;
  const int rc = spe_launch_btail(t, (hipStream_t)stream);
  return rc != 0 ? spe_fail(SPE_E_LAUNCH, "btail launch rejected its arguments") : 0;
}

// The decoder kernels read fragment-packed weights (spe_launch_wfrag_pack).  The hooks take
// row-major rows (ld > 0) and pack them into scratch of their own, released after the launch has
// completed, or already-packed weights (ld == 0, spe_debug_wfrag_pack: timing loops).
namespace {
struct Frags {
  std::vector<void*> bufs;
  hipStream_t s;
  int err = 0;
  explicit Frags(hipStream_t st) : s(st) {}
  const void* get(const void* w, int ld, int N) {
    if (ld == 0 || !w) return w;
    void* p = nullptr;
    if (hipMalloc(&p, (size_t)N * 256 * 2) != hipSuccess) { err = 1; return nullptr; }
    bufs.push_back(p);
    if (spe_launch_wfrag_pack(w, ld, N, p, s) != 0) err = 1;
    return p;
  }
  ~Frags() {
    if (bufs.empty()) return;
    (void)hipStreamSynchronize(s);
    for (void* p : bufs) (void)hipFree(p);
  }
};
}  // namespace

int spe_debug_wfrag_pack(void* stream, const void* w, int ld, int N, void* dst) {
  const int rc = spe_launch_wfrag_pack(w, ld, N, dst, (hipStream_t)stream);
  return rc != 0 ? spe_fail(SPE_E_ARG, "wfrag_pack: bad argument") : 0;
}

int spe_debug_decsa(void* stream, void* tgt, int ldt, int B, int Q, const void* wqk, int ldqk, const float* bqk,
                    const void* wv, int ldv, const float* bv, const void* qpos, const void* wo, int ldo,
                    const float* bo, const float* g, const float* b, float scale) {
  Frags f((hipStream_t)stream);
  DecSaArgs a{};
  a.tgt = tgt; a.ldt = ldt; a.B = B; a.Q = Q;
  a.wqk = f.get(wqk, ldqk, 512); a.bqk = bqk; a.wv = f.get(wv, ldv, 256); a.bv = bv; a.qpos = qpos;
  a.wo = f.get(wo, ldo, 256); a.bo = bo; a.g = g; a.b = b; a.scale = scale;
  if (f.err) return spe_fail(SPE_E_ARG, "decsa: weight packing failed");
  const int rc = spe_launch_decsa(a, (hipStream_t)stream);
  return rc != 0 ? spe_fail(SPE_E_LAUNCH, "decsa launch rejected its arguments") : 0;
}

int spe_debug_decproj(void* stream, void* tgt, int ldt, const void* x, int ldx, int B, int Q, const void* wo, int ldo,
                      const float* bo, const float* g, const float* b) {
  Frags f((hipStream_t)stream);
  DecProjArgs a{};
  a.tgt = tgt; a.ldt = ldt; a.x = x; a.ldx = ldx; a.B = B; a.Q = Q; a.wo = f.get(wo, ldo, 256); a.bo = bo;
  a.g = g; a.b = b;
  if (f.err) return spe_fail(SPE_E_ARG, "decproj: weight packing failed");
  const int rc = spe_launch_decproj(a, (hipStream_t)stream);
  return rc != 0 ? spe_fail(SPE_E_LAUNCH, "decproj launch rejected its arguments") : 0;
}

int spe_debug_decxproj(void* stream, void* tgt, int ldt, float* partial_scratch, int splits, int T, int B, int Q,
                       const void* wv, int ldwv, const float* bv, const void* wo, int ldo, const float* bo,
                       const float* g, const float* b) {
  if (!partial_scratch || T < 1 || B < 0 || Q < 1) return spe_fail(SPE_E_ARG, "bad argument");
  Frags f((hipStream_t)stream);
  DecProjArgs a{};
  a.tgt = tgt; a.ldt = ldt; a.B = B; a.Q = Q; a.wo = f.get(wo, ldo, 256); a.bo = bo; a.g = g; a.b = b;
  const int req = splits > 0 ? splits : spe_xattn_splits(B, Q, T);
  const size_t rows = (size_t)req * B * 8 * Q;  // spe_debug_xattn's scratch layout
  a.pm = partial_scratch; a.pl = partial_scratch + rows; a.pu = partial_scratch + 2 * rows;
  a.splits = spe_xattn_launch_splits(T, req);
  a.wv = f.get(wv, ldwv, 256); a.bv = bv;
  if (f.err) return spe_fail(SPE_E_ARG, "decxproj: weight packing failed");
  const int rc = spe_launch_decproj(a, (hipStream_t)stream);
  return rc != 0 ? spe_fail(SPE_E_LAUNCH, "decxproj launch rejected its arguments") : 0;
}

int spe_debug_decffn(void* stream, const void* x, int ldx, int M, int F, const void* w1, int ld1, const float* b1,
                     const void* w2, int ld2, const float* b2, const float* gamma, const float* beta, void* y, int ldy,
                     float* partial) {
  if (!x || !w1 || !w2 || !y || !partial || M < 0 || F < 256 || F % 256) return spe_fail(SPE_E_ARG, "bad argument");
  Frags f((hipStream_t)stream);
  DecFfnArgs a{};
  a.x = x; a.ldx = ldx; a.M = M; a.F = F; a.b1 = b1; a.partial = partial;
  a.w1 = f.get(w1, ld1, F);
  if (ld2 == 0) {
    a.w2 = w2;
  } else {                                      // W2 packed per 256-wide hidden chunk
    void* p = nullptr;
    if (hipMalloc(&p, (size_t)256 * F * 2) != hipSuccess) return spe_fail(SPE_E_ARG, "decffn: scratch");
    f.bufs.push_back(p);
    for (int c0 = 0; c0 < F; c0 += 256)
      if (spe_launch_wfrag_pack((const char*)w2 + (size_t)c0 * 2, ld2, 256, (char*)p + (size_t)c0 * 256 * 2,
                                (hipStream_t)stream))
        f.err = 1;
    a.w2 = p;
  }
  if (f.err) return spe_fail(SPE_E_ARG, "decffn: weight packing failed");
  FfnArgs r{};
  r.x = x; r.ldx = ldx; r.y = y; r.ldy = ldy; r.M = M; r.D = 256; r.F = F;
  r.b2 = b2; r.gamma = gamma; r.beta = beta; r.splits = F / 256; r.partial = partial;
  int rc = spe_launch_decffn(a, (hipStream_t)stream);
  if (!rc) rc = spe_launch_ffn_reduce_ln(r, (hipStream_t)stream);
  return rc != 0 ? spe_fail(SPE_E_LAUNCH, "decffn launch rejected its arguments") : 0;
}

int spe_debug_decq(void* stream, const void* x, int ldx, int M, int N, const void* w, int ldw, const float* bias,
                   const void* r, int ldr, int period, void* y, int ldy) {
  if (!x || !w || !y || M < 0 || N < 256 || N % 256) return spe_fail(SPE_E_ARG, "bad argument");
  Frags f((hipStream_t)stream);
  DecQArgs a{};
  a.x = x; a.ldx = ldx; a.M = M; a.N = N; a.w = f.get(w, ldw, N); a.bias = bias;
  a.R = r; a.ldr = ldr; a.period = period; a.y = y; a.ldy = ldy;
  if (f.err) return spe_fail(SPE_E_ARG, "decq: weight packing failed");
  const int rc = spe_launch_decq(a, (hipStream_t)stream);
  return rc != 0 ? spe_fail(SPE_E_LAUNCH, "decq launch rejected its arguments") : 0;
}

int spe_debug_btail_perm(int k) { return spe_btail_perm(k); }

int spe_debug_stempool(void* stream, const void* x, const void* w, int ldw, const float* bias, void* out, int ldo,
                       int B, int S) {
  if (!x || !w || !bias || !out || B < 0) return spe_fail(SPE_E_ARG, "bad argument");
  const int rc = spe_launch_stempool(x, w, ldw, bias, out, ldo, B, S, (hipStream_t)stream);
  return rc != 0 ? spe_fail(SPE_E_LAUNCH, "stempool launch rejected its arguments") : 0;
}

}  // extern "C"
