// Persistent weight-stationary streaming GEMM for the short-K bf16 linear problems of the
// forward pass: the 1x1 convs of ResNet-50 layer1-3 (REV/models/backbone.py:114-125), the
// neck's s8_latern and input_proj (:138, detr_speed.py:54-55) and the encoder's q/k, v and
// out projections (REV/models/transformer.py:154-167).  These read an activation once and write
// one back with only K <= 512 multiply-adds per output, so they are HBM-bound; the tile-per-
// workgroup kernel (gemm2.hip) loses much of the bandwidth to its per-tile prologue (the first
// K-step's round trip) and to its epilogue, during which the workgroup has nothing in flight.
//
//   C[M,N] = act(A[M,K] . W[N,K]^T + bias (+ R)) | LayerNorm(A . W^T + bias + R) | V^T store
//
// * One persistent workgroup (8 waves) per CU owns one BN-wide slice of W for its whole life:
//   the slice is copied into LDS once (XOR-swizzled 16-byte chunks, conflict-free fragment
//   reads) and never re-read from memory.
// * Each wave streams its own row tiles (RF x 16 rows x all K) from HBM straight into
//   registers as MFMA fragments -- one 16-byte load per lane per fragment, a row's K extent in
//   contiguous 64-byte pieces -- and computes the tile's whole BN-wide output row block against
//   the LDS-resident W.  The next row tile's fragments (and residual) are loaded before the
//   current tile is multiplied, so every wave always has a tile in flight, epilogue included.
//   No barrier after the prologue: W is read-only, the waves run independently.
// * Epilogue straight from the accumulators.  Row-major outputs use MFMA(W, A) so a lane owns 4
//   consecutive columns of one row (8-byte stores, residual read the same way); a row's BN
//   columns live in one wave, so the fused post-norm LayerNorm (encoder norm1) is two
//   shuffle reductions.  The head-transposed V^T store uses MFMA(A, W): 4 consecutive tokens of
//   one column per lane.
// N > BN: the NS slices of W go to NS adjacent workgroups of the XCD-remapped grid (same XCD),
// which walk the same row tiles in step, so A comes from HBM once and from L2 for the others.
#include <cstdlib>
#include <type_traits>

#include "spe_common.h"
#include "spe_kernels.h"

namespace {

typedef __attribute__((address_space(3))) void* lds_ptr_t;

enum { EPI_ROW = 0, EPI_LN = 1, EPI_VT = 2 };

// Every wave issues the same memory instructions on every path (prefetches past the last tile
// re-load the last tile, rows past M store to this sink line): the compiler's s_waitcnt vmcnt
// counts are exact only when no path skips a load or a store, and a conservative count would
// drain the prefetched tiles before every multiply.
__device__ __attribute__((aligned(256))) uint32_t g_sg_sink[64];

// CP: the pair-packed stem (forward.cpp, registry.cpp) as a streaming GEMM.  Its K order
// k = (kh*8 + kw)*4 + ci makes fragment kf (32 elements = 64 bytes) the kh = kf row of the
// 7x8 window: 8 adjacent 4-channel pixels of the zero-bordered input, contiguous.  So A row m
// (output pixel b, oh, ow) is 8 pieces of 64 B at a stride of one input row; piece 7 (kh = 7,
// zero weights) stays inside the bordered image.
template <int K, int BN, int RF, int OCC, int NB, bool HAS_R, int EPI, bool CP = false>
__global__ __launch_bounds__(256, OCC) void sgemm_kernel(GemmArgs g, int ns_count, int row_tiles) {
  constexpr int KB = K * 2;                          // bytes of one W / A row
  constexpr int KF = K / 32, JF = BN / 16;           // K fragments, 16-column fragments
  constexpr int TR = RF * 16;                        // rows per wave tile
  constexpr bool SWAP = EPI != EPI_VT;               // MFMA(W, A): lanes own row segments
  constexpr int JGMAX = (OCC >= 2 || (HAS_R && EPI == EPI_LN)) ? 4 : 8;   // W fragments per LDS read group
  constexpr int NW = 4, NT = 256;                    // 4 waves; OCC workgroups per CU: 512/OCC registers per wave
  static_assert(!HAS_R || NB % 2 == 0, "residual buffers alternate with the A buffers");
  // EXACT: identical memory instructions on every path (see g_sg_sink).  The residual variants
  // skip instead: the always-live buffers would not fit their registers.
  constexpr bool EXACT = !HAS_R;
  __shared__ __attribute__((aligned(1024))) char wl[BN * KB];
  // bias and LayerNorm affine of the slice (fp32), read in the epilogue instead of being held
  // in registers for the kernel's life
  __shared__ __attribute__((aligned(16))) float sb[BN], slg[EPI == EPI_LN ? BN : 1], slb[EPI == EPI_LN ? BN : 1];

  const int tid = threadIdx.x, lane = tid & 63, wid = __builtin_amdgcn_readfirstlane(tid >> 6);
  const int fg = lane >> 4, fr = lane & 15;
  const int G = gridDim.x;
  const int gid = xcd_remap(blockIdx.x, G);
  const int ns = gid % ns_count;
  const int n0 = ns * BN;
  const int wstride = (G / ns_count) * NW;           // row tiles advanced per step of one wave
  int rt = (gid / ns_count) * NW + wid;               // this wave's first row tile

  // ---- W slice -> LDS.  Row n, 16-byte chunk c (of K/8) at n*KB + (c ^ (n & wkey_mask(KB)))*16.
  // One direct-to-LDS wave instruction fills 1 KB linearly; the swizzle is applied on the source.
  {
    constexpr int INS = BN * KB / 1024;
    for (int q = wid; q < INS; q += NW) {
      const int o = q * 1024 + lane * 16;
      const int n = o / KB, within = o - n * KB;
      const int chunk = (within >> 4) ^ (n & wkey_mask(KB));
      const int nn = n0 + n < g.N ? n0 + n : g.N - 1;     // (N % BN == 0 on every launch)
      const char* src = (const char*)g.B + (size_t)nn * g.ldb * 2 + chunk * 16;
      __builtin_amdgcn_global_load_lds((const void*)src, (lds_ptr_t)(wl + q * 1024), 16, 0, 0);
    }
    for (int i = tid; i < BN; i += NT) {
      sb[i] = g.bias ? g.bias[n0 + i] : 0.f;
      if constexpr (EPI == EPI_LN) {
        slg[i] = g.ln_g[n0 + i];
        slb[i] = g.ln_b[n0 + i];
      }
    }
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    __syncthreads();
  }
  auto w_addr = [&](int n, int chunk) { return wkey_addr(n, chunk, KB); };

  // first row of row tile t.  (An image-interleaved tile order that kept a row-periodic
  // residual's table rows hot in L2 measured neutral-to-slower on the q/k projection and was
  // removed)
  auto row0 = [&](int t) { return t * TR; };

  // A fragments of one row tile: lane (fg, fr) holds row fr of fragment rf, K chunk 4kf + fg
  auto load_a = [&](int t, u32x4 (&a)[RF][KF]) {
    if constexpr (!EXACT) {
      if (t >= row_tiles) return;
    }
    t = t < row_tiles ? t : row_tiles - 1;
#pragma unroll
    for (int rf = 0; rf < RF; ++rf) {
      int m = row0(t) + 16 * rf + fr;
      m = m < g.M ? m : g.M - 1;                    // clamp: rows past M are computed, not stored
      if constexpr (CP) {
        const int hw = g.Ho * g.Wo, b = m / hw, r = m - b * hw, oh = r / g.Wo, ow = r - oh * g.Wo;
        const char* p = (const char*)g.A + (((size_t)b * g.H + oh * g.stride) * g.W + ow * g.stride) * 8 + fg * 16;
        const int rs = g.W * 8;
#pragma unroll
        for (int kf = 0; kf < KF; ++kf) a[rf][kf] = ld16(p + kf * rs);
      } else {
        const char* p = (const char*)g.A + (size_t)m * g.lda * 2 + fg * 16;
#pragma unroll
        for (int kf = 0; kf < KF; ++kf) a[rf][kf] = ld16(p + kf * 64);
      }
    }
  };
  auto load_r = [&](int t, u32x2 (&r)[RF][JF]) {
    if constexpr (HAS_R) {
      if (t >= row_tiles) return;
#pragma unroll
      for (int rf = 0; rf < RF; ++rf) {
        int m = row0(t) + 16 * rf + fr;
        m = m < g.M ? m : g.M - 1;
        const int rm = g.r_period > 0 ? m % g.r_period : m;
        const char* p = (const char*)g.R + ((size_t)rm * g.ldr + n0 + 4 * fg) * 2;
#pragma unroll
        for (int j = 0; j < JF; ++j) r[rf][j] = ld8(p + j * 32);
      }
    }
  };

  auto tile = [&](int t, const u32x4 (&a)[RF][KF], const u32x2 (&r)[RF][JF]) {
    // (a compiler-only fence: W, bias and the LayerNorm affine are loop-invariant LDS reads, and
    // hoisting all of them out of the tile loop would pin hundreds of registers)
    asm volatile("" ::: "memory");
    f32x4 acc[RF][JF];
#pragma unroll
    for (int rf = 0; rf < RF; ++rf)
#pragma unroll
      for (int j = 0; j < JF; ++j) acc[rf][j] = f32x4{0.f, 0.f, 0.f, 0.f};
    // W fragments are read from LDS in groups of JG (one K step, JG column fragments), group
    // i+1 while group i multiplies (two register sets); the scheduling fences keep the compiler
    // from hoisting every group's reads to the top of the tile
    constexpr int JG = JF < JGMAX ? JF : JGMAX, NGR = KF * (JF / JG);
    u32x4 wb[2][JG];
    auto read_w = [&](int gi, u32x4 (&w)[JG]) {
      const int kf = gi / (JF / JG), j0 = (gi % (JF / JG)) * JG;
#pragma unroll
      for (int j = 0; j < JG; ++j) w[j] = ld16(wl + w_addr(16 * (j0 + j) + fr, 4 * kf + fg));
    };
    read_w(0, wb[0]);
#pragma unroll
    for (int gi = 0; gi < NGR; ++gi) {
      if (gi + 1 < NGR) read_w(gi + 1, wb[(gi + 1) & 1]);
      const int kf = gi / (JF / JG), j0 = (gi % (JF / JG)) * JG;
#pragma unroll
      for (int j = 0; j < JG; ++j) {
        const bf16x8 w = __builtin_bit_cast(bf16x8, wb[gi & 1][j]);
#pragma unroll
        for (int rf = 0; rf < RF; ++rf) {
          const bf16x8 av = __builtin_bit_cast(bf16x8, a[rf][kf]);
          acc[rf][j0 + j] = SWAP ? __builtin_amdgcn_mfma_f32_16x16x32_bf16(w, av, acc[rf][j0 + j], 0, 0, 0)
                                 : __builtin_amdgcn_mfma_f32_16x16x32_bf16(av, w, acc[rf][j0 + j], 0, 0, 0);
        }
      }
      __builtin_amdgcn_sched_barrier(0);
    }
    // epilogue, specialised on the output type and the ReLU (uniform branches, once per tile)
    auto epi = [&](auto f16c, auto reluc) {
      constexpr bool F16 = decltype(f16c)::value, RELU = decltype(reluc)::value;
      if constexpr (EPI == EPI_VT) {
        // lane: C[t*TR + 16rf + 4fg + r][n0 + 16j + fr], 4 consecutive tokens of one column
  #pragma unroll
        for (int rf = 0; rf < RF; ++rf) {
          const int m = row0(t) + 16 * rf + 4 * fg;
          const bool ok = m < g.M;
          const int b = m / g.vt_T, tok = m - b * g.vt_T;
  #pragma unroll
          for (int j = 0; j < JF; ++j) {
            const int n = n0 + 16 * j + fr;
            const float bv = sb[16 * j + fr];
            const uint32_t lo = pack_out2(acc[rf][j][0] + bv, acc[rf][j][1] + bv, F16);
            const uint32_t hi = pack_out2(acc[rf][j][2] + bv, acc[rf][j][3] + bv, F16);
            const int pos = g.vt_swz ? vt_pos(tok) : tok;   // (a 4-token quad moves as a whole)
            char* cp = (char*)g.C + (((size_t)((n >> 8) * g.vt_B + b) * 256 + (n & 255)) * g.vt_T + pos) * 2;
            st8(ok ? cp : (char*)g_sg_sink, u32x2{lo, hi});
          }
        }
      } else {
  #pragma unroll
        for (int rf = 0; rf < RF; ++rf) {
          const int m = row0(t) + 16 * rf + fr;
          float v[JF][4];
  #pragma unroll
          for (int j = 0; j < JF; ++j) {
            float rv[4] = {0.f, 0.f, 0.f, 0.f};
            if constexpr (HAS_R) {
              rv[0] = __uint_as_float(r[rf][j].x << 16);
              rv[1] = __uint_as_float(r[rf][j].x & 0xffff0000u);
              rv[2] = __uint_as_float(r[rf][j].y << 16);
              rv[3] = __uint_as_float(r[rf][j].y & 0xffff0000u);
            }
            const f32x4 bv = *reinterpret_cast<const f32x4*>(sb + 16 * j + 4 * fg);
  #pragma unroll
            for (int e = 0; e < 4; ++e) v[j][e] = acc[rf][j][e] + bv[e] + rv[e];
          }
          if constexpr (EPI == EPI_LN) {
            // the row's 256 columns: 16 fragments x 4 values here, x 4 lanes (fg) -- two xor steps
            float s = 0.f;
  #pragma unroll
            for (int j = 0; j < JF; ++j)
  #pragma unroll
              for (int e = 0; e < 4; ++e) s += v[j][e];
            s += __shfl_xor(s, 16, 64);
            s += __shfl_xor(s, 32, 64);
            const float mean = s * (1.f / 256);
            float q = 0.f;
  #pragma unroll
            for (int j = 0; j < JF; ++j)
  #pragma unroll
              for (int e = 0; e < 4; ++e) q += (v[j][e] - mean) * (v[j][e] - mean);
            q += __shfl_xor(q, 16, 64);
            q += __shfl_xor(q, 32, 64);
            const float rs = rsqrtf(q * (1.f / 256) + 1e-5f);
  #pragma unroll
            for (int j = 0; j < JF; ++j) {
              const f32x4 gm = *reinterpret_cast<const f32x4*>(slg + 16 * j + 4 * fg);
              const f32x4 bt = *reinterpret_cast<const f32x4*>(slb + 16 * j + 4 * fg);
  #pragma unroll
              for (int e = 0; e < 4; ++e) v[j][e] = (v[j][e] - mean) * rs * gm[e] + bt[e];
            }
          } else if (RELU) {
  #pragma unroll
            for (int j = 0; j < JF; ++j)
  #pragma unroll
              for (int e = 0; e < 4; ++e) v[j][e] = fmaxf(v[j][e], 0.f);
          }
          const bool ok = m < g.M;
          if (!EXACT && !ok) continue;
          char* cp = ok ? (char*)g.C + ((size_t)m * g.ldc + n0 + 4 * fg) * 2 : (char*)g_sg_sink;
          const int cstep = ok ? 32 : 0;
  #pragma unroll
          for (int j = 0; j < JF; ++j)
            st8(cp + j * cstep, u32x2{pack_out2(v[j][0], v[j][1], F16), pack_out2(v[j][2], v[j][3], F16)});
        }
      }
    };
    using T_ = std::true_type;
    using F_ = std::false_type;
    if (g.out_f16) {
      if (g.act) epi(T_{}, T_{}); else epi(T_{}, F_{});
    } else {
      if (g.act) epi(F_{}, T_{}); else epi(F_{}, F_{});
    }
  };

  // NB A register sets in rotation: tiles i+1 .. i+NB-1 are in flight while tile i is
  // multiplied and stored; the residual of tile i+1 is requested as tile i starts (two sets).
  u32x4 ab[NB][RF][KF];
  u32x2 rb[HAS_R ? 2 : 1][RF][JF];
  const int rt0 = rt;
  if (rt0 >= row_tiles) return;
#pragma unroll
  for (int u = 0; u < NB - 1; ++u) load_a(rt0 + u * wstride, ab[u]);
  load_r(rt0, rb[0]);
  for (int base = 0;; base += NB) {
    bool done = false;
#pragma unroll
    for (int u = 0; u < NB; ++u) {
      const int t = rt0 + (base + u) * wstride;
      if (t >= row_tiles) {
        done = true;
        break;
      }
      load_a(t + (NB - 1) * wstride, ab[(u + NB - 1) % NB]);
      load_r(t + wstride, rb[HAS_R ? (u + 1) % 2 : 0]);
      tile(t, ab[u], rb[HAS_R ? u % 2 : 0]);
    }
    if (done) break;
  }
}

}  // namespace

int spe_cu_count() {
  static const int n = [] {
    int dev = 0, c = 0;
    if (hipGetDevice(&dev) != hipSuccess ||
        hipDeviceGetAttribute(&c, hipDeviceAttributeMultiprocessorCount, dev) != hipSuccess || c <= 0)
      c = 256;
    return c;
  }();
  return n;
}

namespace {

bool sgemm_enabled() {
  static const bool on = [] { const char* e = getenv("SPE_SGEMM"); return !e || atoi(e) != 0; }();
  return on;
}

template <int K, int BN, int RF, int OCC, int NB, bool HAS_R, int EPI, bool CP = false>
int launch_k(const GemmArgs& g, hipStream_t s) {
  const int row_tiles = (g.M + RF * 16 - 1) / (RF * 16), nsc = g.N / BN;
  const int G = (spe_cu_count() * OCC / nsc) * nsc;
  if ((long)row_tiles < 2L * (G / nsc) * 4) return 1;    // fewer than two tiles per wave
  hipLaunchKernelGGL((sgemm_kernel<K, BN, RF, OCC, NB, HAS_R, EPI, CP>), dim3(G), dim3(256), 0, s, g, nsc, row_tiles);
  spe_gemm_last_path = 2;
  return (int)hipGetLastError();
}

// Per (K, BN): row fragments per wave tile RF, workgroups per CU OCC (LDS: BN*K*2 bytes each;
// registers: 512/OCC per wave), A register sets NB -- for the plain (0) and the residual (1)
// epilogues.  Registers per wave ~ RF*BN/4 accumulators + NB*RF*K/4 A + 2*JG*4 W + RF*BN/4 R.
template <int K, int BN, int RF0, int OCC0, int NB0, int RF1, int OCC1, int NB1>
int launch_kbn(const GemmArgs& g, hipStream_t s) {
  if (g.N % BN) return 1;
  if (g.vt_T > 0) return g.R ? 1 : launch_k<K, BN, RF0, OCC0, NB0, false, EPI_VT>(g, s);
  if (g.ln_g) {                                   // encoder norm1 (K = N = 256): two A sets, the
    if constexpr (K == 256 && BN == 256)           // LayerNorm epilogue needs the registers
      return g.R ? launch_k<K, BN, 1, 1, 2, true, EPI_LN>(g, s) : 1;
    return 1;
  }
  return g.R ? launch_k<K, BN, RF1, OCC1, NB1, true, EPI_ROW>(g, s) : launch_k<K, BN, RF0, OCC0, NB0, false, EPI_ROW>(g, s);
}

}  // namespace

// Returns 1 when the problem is not for this kernel (the caller takes gemm2 / gemm).
int spe_launch_sgemm(const GemmArgs& g, int mode, hipStream_t s) {
  if (mode == GEMM_CONV && sgemm_enabled()) {
    // the pair-packed stem (see CP): 7x8 window, 4 channels, pre-bordered input, N = 64
    static const int on = [] { const char* e = getenv("SPE_SG_STEM"); return e ? atoi(e) : 1; }();
    if (on && g.Cin == 4 && g.KH == 7 && g.KW == 8 && g.pad == 0 && g.K == 224 && g.ldb == 256 && g.N == 64 &&
        !g.R && !g.ln_g && g.vt_T == 0 && g.act <= ACT_RELU && !g.res_post && !g.out_f32 && g.ldc % 4 == 0 &&
        (g.Ho - 1) * g.stride + 8 <= g.H && (g.Wo - 1) * g.stride + 8 <= g.W)
      return launch_k<256, 64, 1, 2, 4, false, EPI_ROW, true>(g, s);
    return 1;
  }
  if (!sgemm_enabled() || mode != GEMM_LINEAR || g.M <= 0) return 1;
  if (g.act > ACT_RELU || g.res_post || g.out_f32) return 1;
  if (g.ldb < g.K || g.ldb % 8 || g.lda % 8 || g.ldc % 4 || (g.R && g.ldr % 4)) return 1;
  if (g.ln_g && (g.N != 256 || g.act)) return 1;
  if (g.vt_T > 0 && (g.vt_T % 4 || g.M % 4 || g.N % 256 || g.act || (g.vt_swz && g.vt_T % 16))) return 1;
  switch (g.K) {
    case 64:
      if (g.N == 64) return launch_kbn<64, 64, 2, 2, 4, 2, 2, 4>(g, s);
      if (g.N == 128) return launch_kbn<64, 128, 1, 2, 4, 1, 2, 4>(g, s);
      return 1;                                    // (N >= 256: the 256-row tiles of gemm2 measured faster)
    case 128:
      if (g.N == 64) return launch_kbn<128, 64, 1, 2, 4, 1, 2, 4>(g, s);
      if (g.N == 128) return launch_kbn<128, 128, 1, 2, 4, 1, 2, 2>(g, s);
      // the layer-2 conv3 + identity (N = 512): 0.126 -> 0.115 ms per launch at B = 64 against
      // gemm2's 256-row tiles (kbench); without a residual gemm2 stays faster
      if (g.N % 256 == 0 && g.R) return launch_kbn<128, 256, 1, 2, 2, 1, 2, 2>(g, s);
      return 1;
    case 256:
      if (g.N == 64) return launch_kbn<256, 64, 1, 2, 4, 1, 2, 4>(g, s);
      if (g.N == 128) return launch_kbn<256, 128, 1, 2, 4, 1, 2, 2>(g, s);
      return launch_kbn<256, 256, 1, 1, 4, 1, 1, 2>(g, s);
    case 512:
      if (g.N == 64) return launch_kbn<512, 64, 1, 2, 2, 1, 2, 2>(g, s);
      return launch_kbn<512, 128, 1, 1, 4, 1, 1, 4>(g, s);
    default: return 1;
  }
}
