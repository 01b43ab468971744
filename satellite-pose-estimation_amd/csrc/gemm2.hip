// Large-tile bf16 GEMM / implicit-GEMM convolution for gfx950 with direct-to-LDS staging.
//
// Serves the bf16 throughput path of every big contraction (ResNet-50 convs, neck convs,
// transformer projections; REV/models/backbone.py:114-149, REV/models/transformer.py:137-191)
// when the problem fills the chip with 256-row tiles; small or fp32 problems stay on gemm.hip.
//
//   C[M,N] = A[M,K] . W[N,K]^T  (+bias[n]) (+R[m or m % r_period, n]) (ReLU)
//
// * Tile 256 x BN (BN = 256 / 128 / 64 by N), 512 threads = 8 waves, wave tile
//   (256/WM) x (BN/WN) of 16x16x32 bf16 MFMA fragments.  K-step = 64 bf16 = one 128-byte line
//   per row.
// * Staging: __builtin_amdgcn_global_load_lds (16 B per lane) straight into LDS, no VGPR
//   round trip and no ds_write.  One wave-instruction fills 8 rows x 128 B linearly, so the
//   XOR swizzle (16-byte chunk c of row r at slot c ^ (r & 7), conflict-free fragment reads)
//   is applied on the SOURCE address (lane slot s loads global chunk s ^ (r & 7)) and again on
//   the read.  Rows past M / N, columns past K and conv padding taps load from a zero line.
// * Pipeline: two LDS stages; stage k+1's loads are issued before stage k is consumed and
//   retired with a counted `s_waitcnt vmcnt(loads per stage)` + raw s_barrier (never
//   __syncthreads, whose fence would drain the in-flight stage).  All LDS is one array.
// * The `+ pos` of the attention projections is NOT applied to A here: by linearity
//   (x + pos) W^T = x W^T + (pos W^T), the runtime precomputes pos W^T once per model and the
//   epilogue adds it as a row-periodic residual (r_period = tokens per image).
// * The residual tile is fetched into registers before the K loop (it is independent of the
//   contraction), so the epilogue never waits on HBM.
// * Epilogue: accumulators -> fp32 LDS tile in 64-row passes -> bias / residual / ReLU ->
//   16-byte row stores (or the head-transposed V^T store).
#include "spe_common.h"
#include "spe_kernels.h"

#include <cstdlib>

namespace {

constexpr int BM = 256, BK = 64, NT = 512;
__device__ __attribute__((aligned(64))) uint32_t g_zero_line[16];   // zero-filled source line

SPE_DEV int swz(int row, int chunk) { return row * 128 + ((chunk ^ (row & 7)) << 4); }

template <int BN> struct Cfg;
template <> struct Cfg<256> { static constexpr int WM = 2, WN = 4; };
template <> struct Cfg<128> { static constexpr int WM = 4, WN = 2; };
template <> struct Cfg<64> { static constexpr int WM = 4, WN = 2; };

typedef __attribute__((address_space(3))) void* lds_ptr_t;

template <int N>
SPE_DEV void wait_vmcnt() { asm volatile("s_waitcnt vmcnt(%0)" ::"n"(N) : "memory"); }

// raw workgroup barrier (no vmcnt drain) that LDS reads / DMA issues are not moved across
SPE_DEV void bar_raw() {
  asm volatile("" ::: "memory");
  __builtin_amdgcn_s_barrier();
  asm volatile("" ::: "memory");
}

// K from which a 256-wide linear GEMM takes the 4-phase half-tile schedule (P8 below).  Measured
// (B=64 bench shapes): +10-12 % on long-K linear problems (8192^3, K = 9216); slower for K <= 256
// (the deeper prologue) and for the implicit-GEMM convolutions, which keep the 2-stage loop.
constexpr int P8_MIN_K = 1024;

// LN: fused post-norm LayerNorm epilogue (a separate instantiation: its 16 extra live
// registers would push the plain 256-wide kernel into spills)
// NST = LDS stages: 2 (double-buffered K loop, one workgroup per CU) or 1 (load, wait,
// multiply per K-step, LDS and registers sized for two resident workgroups per CU, so one
// workgroup's epilogue and load latency overlap the other's work: short-K linear problems)
// XA: extended epilogue (SiLU / GELU, residual after the activation) for the RT-DETR encoder.
// A separate instantiation: the extra live state made the ReLU-only tiles spill (272 B/lane).
// PIN: no residual (g.R must be null: the residual prefetch registers are compiled out) and a
// pinned fragment schedule in the 2-stage loop -- the reads of the next fragment group are
// issued ahead of the current group's MFMAs and the order is fixed with sched_barrier, where
// the compiler's schedule waits on lgkmcnt(0) before every 8 MFMAs.
// BUF: stage through buffer_load ... lds (see PIN) without the pinned schedule.
template <int BN, int MODE, bool LN, bool P8K = false, int NST = 2, bool XA = false, bool PIN = false, bool BUF = false>
__global__ __launch_bounds__(NT, NST == 1 ? 4 : 1) void gemm2_kernel(GemmArgs g) {
  constexpr int WM = Cfg<BN>::WM, WN = Cfg<BN>::WN;
  constexpr int TM = BM / WM, TN = BN / WN, FM = TM / 16, FN = TN / 16;
  constexpr int A_BYTES = BM * 128, STAGE = (BM + BN) * 128;
  constexpr int IA = BM / 64, IB = BN / 64;            // glds instructions per wave per stage
  constexpr int LOADS = IA + IB;
  constexpr int EPI_ROWS = 64, EPI_LD = BN + 4;
  constexpr int SMEM = (NST * STAGE > EPI_ROWS * EPI_LD * 4) ? NST * STAGE : EPI_ROWS * EPI_LD * 4;
  __shared__ __attribute__((aligned(1024))) char smem[SMEM];

  const int tid = threadIdx.x, lane = tid & 63, wid = __builtin_amdgcn_readfirstlane(tid >> 6);
  const int wr = wid / WN, wc = wid % WN;
  const int tilesN = (g.N + BN - 1) / BN;
  const int t = xcd_remap(blockIdx.x, gridDim.x);
  const int m0 = (t / tilesN) * BM, n0 = (t % tilesN) * BN;
  const int nk = (g.K + BK - 1) / BK;

  // P8 (256x256 tiles): the K-step is split into 4 phases over half-tiles (A rows 0-127 / 128-255,
  // W rows 0-127 / 128-255).  A wave's 128x64 output is then two 64-row halves (one in each A
  // half-tile) x two 32-column halves, so every phase multiplies one A half by one W half and a
  // half-tile's buffer can be refilled as soon as its phase has been read.
  constexpr bool P8 = BN == 256 && P8K;
  // first row of load instruction i (IA = IB = 4 when P8) and of fragment i / j
  auto ld_row = [&](int i, int I) { return P8 ? (i >> 1) * 128 + wid * 16 + (i & 1) * 8 : (wid * I + i) * 8; };
  auto frag_row = [&](int i) { return P8 ? (i >> 2) * 128 + wr * 64 + (i & 3) * 16 : wr * TM + i * 16; };
  auto frag_col = [&](int j) { return P8 ? (j >> 1) * 128 + wc * 32 + (j & 1) * 16 : wc * TN + j * 16; };

  // ---- per-lane load descriptors.  Instruction i of wave w fills rows ld_row(i) + lane/8.
  const int lrow = lane >> 3;                    // row within the 8-row group
  const int chunk = (lane & 7) ^ lrow;           // global 16-byte chunk this lane fetches
  const char* zero = reinterpret_cast<const char*>(g_zero_line);
  const char* abase[IA];
  int aih[IA], aiw[IA];
  bool arow[IA];
#pragma unroll
  for (int i = 0; i < IA; ++i) {
    const int m = m0 + ld_row(i, IA) + lrow;
    arow[i] = m < g.M;
    const int mm = arow[i] ? m : 0;
    if constexpr (MODE == GEMM_CONV) {
      const int hw = g.Ho * g.Wo;
      const int b = mm / hw, r = mm - b * hw;
      const int oh = r / g.Wo, ow = r - oh * g.Wo;
      aih[i] = oh * g.stride - g.pad;
      aiw[i] = ow * g.stride - g.pad;
      abase[i] = (const char*)g.A + (size_t)b * g.H * g.W * g.Cin * 2;
    } else {
      abase[i] = (const char*)g.A + (size_t)mm * g.lda * 2;
      aih[i] = aiw[i] = 0;
    }
  }
  const char* bbase[IB];
#pragma unroll
  for (int i = 0; i < IB; ++i) {
    const int n = n0 + ld_row(i, IB) + lrow;
    bbase[i] = n < g.N ? (const char*)g.B + ((size_t)n * g.ldb + chunk * 8) * 2 : nullptr;
  }

  // Convolution K position of a K-step.  Channel-blocked order (Cin % 64 == 0, see
  // conv_k_decode) makes a whole K-step one (channel block, tap): it is tracked incrementally in
  // scalar registers instead of being divided out per lane.
  const int taps = g.KH * g.KW;
  const bool kblocked = MODE == GEMM_CONV && conv_channel_blocked(g.Cin, taps);
  struct KPos { int cb, kh, kw; };
  auto kadv = [&](KPos p) {
    if (++p.kw == g.KW) {
      p.kw = 0;
      if (++p.kh == g.KH) { p.kh = 0; ++p.cb; }
    }
    return p;
  };
  // PIN: the same loads as buffer_load ... lds (MUBUF: the compiler then counts only the LDS
  // fragment reads on lgkmcnt -- pending FLAT-encoded global_load_lds make it wait lgkmcnt(0)
  // before every fragment group).  32-bit byte offsets; out-of-range offsets read zeros.
  constexpr int BAD = 0x7ffffff0;
  const long long abytes = !(PIN || BUF) ? 0
                           : MODE == GEMM_CONV ? (long long)((g.M + g.Ho * g.Wo - 1) / (g.Ho * g.Wo)) * g.H * g.W * g.Cin * 2
                                               : (long long)g.M * g.lda * 2;
  const __amdgpu_buffer_rsrc_t rsa =
      __builtin_amdgcn_make_buffer_rsrc((void*)g.A, (short)0, (int)(abytes < BAD ? abytes : BAD), 0x00020000);
  const __amdgpu_buffer_rsrc_t rsb = __builtin_amdgcn_make_buffer_rsrc((void*)g.B, (short)0, g.N * g.ldb * 2, 0x00020000);
  int aoff[(PIN || BUF) ? IA : 1], boff[(PIN || BUF) ? IB : 1];
  if constexpr (PIN || BUF) {
#pragma unroll
    for (int i = 0; i < IA; ++i) aoff[i] = (int)(abase[i] - (const char*)g.A);
#pragma unroll
    for (int i = 0; i < IB; ++i) boff[i] = bbase[i] ? (int)(bbase[i] - (const char*)g.B) : BAD;
  }
  auto issue_buf = [&](int ks, const KPos& kp, int buf, int ia0, int ia1, int ib0, int ib1) {
    char* st = smem + buf * STAGE;
    const int k = ks * BK + chunk * 8;
    const bool kv = k < g.K;
#pragma unroll
    for (int i = 0; i < IA; ++i) {
      if (i < ia0 || i >= ia1) continue;
      int off;
      if constexpr (MODE == GEMM_CONV) {
        int kh, kw, ci;
        if (kblocked) {
          kh = kp.kh; kw = kp.kw; ci = kp.cb * 64 + chunk * 8;
        } else if (taps == 1) {
          kh = kw = 0; ci = k;
        } else {
          conv_k_decode(k, g.Cin, g.KW, taps, kh, kw, ci);
        }
        const int ih = aih[i] + kh, iw = aiw[i] + kw;
        const bool v = kv && arow[i] && ih >= 0 && ih < g.H && iw >= 0 && iw < g.W;
        off = v ? aoff[i] + ((ih * g.W + iw) * g.Cin + ci) * 2 : BAD;
      } else {
        off = (kv && arow[i]) ? aoff[i] + k * 2 : BAD;
      }
      __builtin_amdgcn_raw_ptr_buffer_load_lds(rsa, (lds_ptr_t)(st + ld_row(i, IA) * 128), 16, off, 0, 0, 0);
    }
#pragma unroll
    for (int i = 0; i < IB; ++i) {
      if (i < ib0 || i >= ib1) continue;
      const int off = (boff[i] != BAD && ks * BK < g.K) ? boff[i] + ks * BK * 2 : BAD;
      __builtin_amdgcn_raw_ptr_buffer_load_lds(rsb, (lds_ptr_t)(st + A_BYTES + ld_row(i, IB) * 128), 16, off, 0, 0, 0);
    }
  };
  // issue A instructions [ia0, ia1) and W instructions [ib0, ib1) of K-step ks (K position kp)
  // into stage buf (constant ranges after inlining; K-steps past the end load the zero line)
  auto issue_rng =[&](int ks, const KPos& kp, int buf, int ia0, int ia1, int ib0, int ib1) {
    if constexpr (PIN || BUF) {
      issue_buf(ks, kp, buf, ia0, ia1, ib0, ib1);
      return;
    }
    char* st = smem + buf * STAGE;
    const int k = ks * BK + chunk * 8;
    const bool kv = k < g.K;
    if constexpr (MODE == GEMM_CONV) {
      int kh, kw, ci;
      if (kblocked) {
        kh = kp.kh; kw = kp.kw; ci = kp.cb * 64 + chunk * 8;
      } else if (taps == 1) {
        kh = kw = 0; ci = k;
      } else {
        conv_k_decode(k, g.Cin, g.KW, taps, kh, kw, ci);
      }
#pragma unroll
      for (int i = 0; i < IA; ++i) {
        if (i < ia0 || i >= ia1) continue;
        const int ih = aih[i] + kh, iw = aiw[i] + kw;
        const bool v = kv && arow[i] && ih >= 0 && ih < g.H && iw >= 0 && iw < g.W;
        const char* src = v ? abase[i] + ((size_t)(ih * g.W + iw) * g.Cin + ci) * 2 : zero;
        __builtin_amdgcn_global_load_lds((const void*)src, (lds_ptr_t)(st + ld_row(i, IA) * 128), 16, 0, 0);
      }
    } else {
#pragma unroll
      for (int i = 0; i < IA; ++i) {
        if (i < ia0 || i >= ia1) continue;
        const char* src = (kv && arow[i]) ? abase[i] + (size_t)k * 2 : zero;
        __builtin_amdgcn_global_load_lds((const void*)src, (lds_ptr_t)(st + ld_row(i, IA) * 128), 16, 0, 0);
      }
    }
#pragma unroll
    for (int i = 0; i < IB; ++i) {
      if (i < ib0 || i >= ib1) continue;
      const char* src = (bbase[i] && ks * BK < g.K) ? bbase[i] + (size_t)ks * BK * 2 : zero;
      __builtin_amdgcn_global_load_lds((const void*)src, (lds_ptr_t)(st + A_BYTES + ld_row(i, IB) * 128), 16, 0, 0);
    }
  };
  auto issue = [&](int ks, const KPos& kp, int buf) { issue_rng(ks, kp, buf, 0, IA, 0, IB); };
  const KPos kp0{0, 0, 0};

  f32x4 acc[FM][FN];
#pragma unroll
  for (int i = 0; i < FM; ++i)
#pragma unroll
    for (int j = 0; j < FN; ++j) acc[i][j] = f32x4{0.f, 0.f, 0.f, 0.f};

  // BN = 64 tiles store straight from the accumulators (see the direct epilogue below); the
  // wider tiles stage their output through LDS for 16-byte row stores, which measured faster
  // for the store-heavy 256-wide shapes.
  constexpr bool DIRECT = BN == 64;
  const int fg = lane >> 4, fr = lane & 15;
  u32x2 dres[DIRECT ? FM : 1][FN];
  f32x4 dbias[DIRECT ? FN : 1];
  if constexpr (DIRECT) {
#pragma unroll
    for (int j = 0; j < FN; ++j) {
      const int n = n0 + wc * TN + 16 * j + 4 * fg;
      dbias[j] = f32x4{0.f, 0.f, 0.f, 0.f};
      if (g.bias && n + 4 <= g.N) dbias[j] = *reinterpret_cast<const f32x4*>(g.bias + n);
      else if (g.bias)
        for (int r = 0; r < 4; ++r) dbias[j][r] = n + r < g.N ? g.bias[n + r] : 0.f;
    }
#pragma unroll
    for (int i = 0; i < FM; ++i)
#pragma unroll
      for (int j = 0; j < FN; ++j) {
        dres[i][j] = u32x2{0, 0};
        const int m = m0 + wr * TM + 16 * i + fr, n = n0 + wc * TN + 16 * j + 4 * fg;
        if (!PIN && g.R && m < g.M && n + 4 <= g.N) {
          const int rm = g.r_period > 0 ? m % g.r_period : m;
          dres[i][j] = ld8((const bf16*)g.R + (size_t)rm * g.ldr + n);
        }
      }
  }

  // ---- residual tile prefetch: this thread's epilogue rows x 8 columns, in registers
  constexpr int TPR = BN / 8;                   // epilogue threads per row (8 columns each)
  constexpr int RSTEP = NT / TPR, RPT = EPI_ROWS / RSTEP, NPASS = BM / EPI_ROWS;
  const int ecg = (tid % TPR) * 8, en = n0 + ecg, ert = tid / TPR;
  const bool efull = en + 8 <= g.N;
  // (BN = 256: only the first half here, the rest after the K loop, or the K loop would spill)
  // (P8: none before the loop, its phases hold more fragments live)
  constexpr int NPRE = (P8 || NST == 1 || PIN) ? 0 : BN == 256 ? NPASS / 2 : NPASS;
  u32x4 rres[NPASS][RPT];
  auto fetch_res = [&](int pp) {
#pragma unroll
    for (int q = 0; q < RPT; ++q) {
      rres[pp][q] = u32x4{0, 0, 0, 0};
      const int m = m0 + pp * EPI_ROWS + ert + q * RSTEP;
      if (!PIN && !DIRECT && g.R && g.vt_T == 0 && efull && m < g.M) {
        const int rm = g.r_period > 0 ? m % g.r_period : m;
        rres[pp][q] = ld16((const bf16*)g.R + (size_t)rm * g.ldr + en);
      }
    }
  };
#pragma unroll
  for (int pp = 0; pp < NPRE; ++pp) fetch_res(pp);
  // the bias too: a load in the epilogue would cost one more HBM round trip per tile
  float ebias[8];
  if (!DIRECT && g.bias && efull) {
    const f32x4 b0 = *reinterpret_cast<const f32x4*>(g.bias + en), b1 = *reinterpret_cast<const f32x4*>(g.bias + en + 4);
#pragma unroll
    for (int e = 0; e < 4; ++e) { ebias[e] = b0[e]; ebias[4 + e] = b1[e]; }
  } else {
#pragma unroll
    for (int e = 0; e < 8; ++e) ebias[e] = (!DIRECT && g.bias && en + e < g.N) ? g.bias[en + e] : 0.f;
  }
  float elg[LN ? 8 : 1], elb[LN ? 8 : 1];        // fused LayerNorm affine (this thread's 8 columns)
  if constexpr (LN) {
#pragma unroll
    for (int e = 0; e < 8; ++e) {
      elg[e] = en + e < g.N ? g.ln_g[en + e] : 0.f;
      elb[e] = en + e < g.N ? g.ln_b[en + e] : 0.f;
    }
  }

  if constexpr (P8) {
    // Half-tile stream, 2 glds per half per wave.  Issue order per K-step: A0 W0 W1 A1; the
    // halves of K-step t+2 go into the stage t is using two phases after t read them, and each
    // K-step's wait leaves 3 halves (6 loads) in flight.
    //   phase 1: read W0, A0 | issue A1(t+1)          | A0 x W0
    //   phase 2: read W1     |                        | A0 x W1
    //   phase 3: read A1     | issue A0, W0 (t+2)     | A1 x W1
    //   phase 4:             | issue W1(t+2), vmcnt(6) retires all of t+1 | A1 x W0
    KPos kp1 = kadv(kp0), kp2 = kadv(kp1);       // K positions of steps ks+1, ks+2
    issue(0, kp0, 0);
    issue_rng(1, kp1, 1, 0, 2, 0, 4);
    wait_vmcnt<6>();
    bar_raw();
    u32x4 fa[8][2], fb[4][2];                    // [fragment][kk]
    auto read_a = [&](const char* st, int i0) {
#pragma unroll
      for (int i = i0; i < i0 + 4; ++i)
#pragma unroll
        for (int kk = 0; kk < 2; ++kk) fa[i][kk] = ld16(st + swz(frag_row(i) + fr, 4 * kk + fg));
    };
    auto read_b = [&](const char* st, int j0) {
#pragma unroll
      for (int j = j0; j < j0 + 2; ++j)
#pragma unroll
        for (int kk = 0; kk < 2; ++kk) fb[j][kk] = ld16(st + A_BYTES + swz(frag_col(j) + fr, 4 * kk + fg));
    };
    auto mma = [&](int i0, int j0) {
      asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
      __builtin_amdgcn_sched_barrier(0);
      __builtin_amdgcn_s_setprio(1);
#pragma unroll
      for (int kk = 0; kk < 2; ++kk)
#pragma unroll
        for (int i = i0; i < i0 + 4; ++i)
#pragma unroll
          for (int j = j0; j < j0 + 2; ++j)
            acc[i][j] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(__builtin_bit_cast(bf16x8, fa[i][kk]),
                                                                __builtin_bit_cast(bf16x8, fb[j][kk]), acc[i][j], 0, 0, 0);
      __builtin_amdgcn_s_setprio(0);
      __builtin_amdgcn_sched_barrier(0);
      bar_raw();
    };
    // The waves of row group 1 (one per SIMD) run one barrier behind group 0, so on every SIMD
    // one wave reads fragments while the other multiplies.  Under that stagger a barrier orders
    // the two groups only one phase apart, hence: a half is restaged >= 2 phases after the phase
    // that read it, and read >= 1 phase after the phase whose vmcnt retired it.
    if (wr == 1) bar_raw();
    for (int ks = 0; ks < nk; ++ks) {
      const int cur = ks & 1;
      const char* st = smem + cur * STAGE;
      // phase 1
      read_b(st, 0);
      __builtin_amdgcn_sched_barrier(0);
      read_a(st, 0);
      issue_rng(ks + 1, kp1, cur ^ 1, 2, 4, 0, 0);
      bar_raw();
      mma(0, 0);
      // phase 2
      read_b(st, 2);
      bar_raw();
      mma(0, 2);
      // phase 3
      read_a(st, 4);
      issue_rng(ks + 2, kp2, cur, 0, 2, 0, 2);
      bar_raw();
      mma(4, 2);
      // phase 4
      issue_rng(ks + 2, kp2, cur, 0, 0, 2, 4);
      wait_vmcnt<6>();
      bar_raw();
      mma(4, 0);
      kp1 = kp2;
      kp2 = kadv(kp2);
    }
    if (wr == 0) bar_raw();                      // close the stagger
    wait_vmcnt<0>();                             // the zero-line loads past the end, before the
    bar_raw();                                   // epilogue reuses the LDS
  } else if constexpr (NST == 1) {
    KPos kpc = kp0;
    for (int ks = 0; ks < nk; ++ks) {
      issue(ks, kpc, 0);
      kpc = kadv(kpc);
      wait_vmcnt<0>();
      __builtin_amdgcn_s_barrier();             // every wave's stage-ks lines have landed
#pragma unroll
      for (int kk = 0; kk < 2; ++kk) {
        u32x4 af[FM], bfr[FN];
#pragma unroll
        for (int i = 0; i < FM; ++i) af[i] = ld16(smem + swz(wr * TM + i * 16 + fr, 4 * kk + fg));
#pragma unroll
        for (int j = 0; j < FN; ++j) bfr[j] = ld16(smem + A_BYTES + swz(wc * TN + j * 16 + fr, 4 * kk + fg));
#pragma unroll
        for (int i = 0; i < FM; ++i)
#pragma unroll
          for (int j = 0; j < FN; ++j)
            acc[i][j] = DIRECT ? __builtin_amdgcn_mfma_f32_16x16x32_bf16(__builtin_bit_cast(bf16x8, bfr[j]),
                                                                        __builtin_bit_cast(bf16x8, af[i]), acc[i][j], 0, 0, 0)
                               : __builtin_amdgcn_mfma_f32_16x16x32_bf16(__builtin_bit_cast(bf16x8, af[i]),
                                                                        __builtin_bit_cast(bf16x8, bfr[j]), acc[i][j], 0, 0, 0);
      }
      asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
      __builtin_amdgcn_s_barrier();             // stage read: the next K-step may refill it
    }
  } else if constexpr (PIN) {
    issue(0, kp0, 0);
    KPos kpn = kadv(kp0);
    constexpr int NP = FM / 2;                   // A-fragment pairs per kk
    for (int ks = 0; ks < nk; ++ks) {
      // unconditional (past the end: zero lines into the free stage) -- a branch here leaves
      // the compiler unsure of the outstanding LDS counts and every fragment group then waits
      // on lgkmcnt(0)
      issue(ks + 1, kpn, (ks + 1) & 1);
      kpn = kadv(kpn);
      wait_vmcnt<LOADS>();
      __builtin_amdgcn_s_barrier();
      const char* st = smem + (ks & 1) * STAGE;
      u32x4 bfr[2][FN], af[2][2];                // [kk][j], [pair parity][2 rows]
      auto rd_b = [&](int kk) {
#pragma unroll
        for (int j = 0; j < FN; ++j) bfr[kk][j] = ld16(st + A_BYTES + swz(wc * TN + j * 16 + fr, 4 * kk + fg));
      };
      auto rd_a = [&](int kk, int p) {
#pragma unroll
        for (int u = 0; u < 2; ++u) af[p & 1][u] = ld16(st + swz(wr * TM + (2 * p + u) * 16 + fr, 4 * kk + fg));
      };
      rd_b(0);
      rd_a(0, 0);
      __builtin_amdgcn_sched_barrier(0);
#pragma unroll
      for (int sidx = 0; sidx < 2 * NP; ++sidx) {
        const int kk = sidx / NP, p = sidx % NP;
        int nrd = 0;
        if (sidx + 1 < 2 * NP) {                 // next group's fragments, ahead of this one's MFMAs
          const int kn = (sidx + 1) / NP, pn = (sidx + 1) % NP;
          if (kn != kk) { rd_b(kn); nrd += FN; }
          rd_a(kn, pn);
          nrd += 2;
        }
#pragma unroll
        for (int u = 0; u < 2; ++u)
#pragma unroll
          for (int j = 0; j < FN; ++j) {
            const int i = 2 * p + u;
            acc[i][j] = DIRECT ? __builtin_amdgcn_mfma_f32_16x16x32_bf16(__builtin_bit_cast(bf16x8, bfr[kk][j]),
                                                                        __builtin_bit_cast(bf16x8, af[p & 1][u]), acc[i][j], 0, 0, 0)
                               : __builtin_amdgcn_mfma_f32_16x16x32_bf16(__builtin_bit_cast(bf16x8, af[p & 1][u]),
                                                                        __builtin_bit_cast(bf16x8, bfr[kk][j]), acc[i][j], 0, 0, 0);
          }
        // the reads first, then the MFMAs (else the scheduler sinks the reads between the MFMAs
        // that free their registers, and each group waits on lgkmcnt(0))
        if (nrd == 2) __builtin_amdgcn_sched_group_barrier(0x100, 2, 0);
        else if (nrd == FN + 2) __builtin_amdgcn_sched_group_barrier(0x100, FN + 2, 0);
        __builtin_amdgcn_sched_group_barrier(0x008, 2 * FN, 0);
        __builtin_amdgcn_sched_barrier(0);
      }
      asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
      __builtin_amdgcn_s_barrier();
    }
    wait_vmcnt<0>();                             // the zero-line stage, before the epilogue
    bar_raw();                                   // reuses the LDS
  } else {
  issue(0, kp0, 0);
  KPos kpn = kadv(kp0);                          // K position of step ks+1
  for (int ks = 0; ks < nk; ++ks) {
    if (ks + 1 < nk) {
      issue(ks + 1, kpn, (ks + 1) & 1);
      kpn = kadv(kpn);
      wait_vmcnt<LOADS>();                      // retire stage ks, keep ks+1 in flight
    } else {
      wait_vmcnt<0>();
    }
    __builtin_amdgcn_s_barrier();               // every wave's stage-ks lines have landed
    const char* st = smem + (ks & 1) * STAGE;
#pragma unroll
    for (int kk = 0; kk < 2; ++kk) {
      u32x4 af[FM], bfr[FN];
#pragma unroll
      for (int i = 0; i < FM; ++i) af[i] = ld16(st + swz(wr * TM + i * 16 + fr, 4 * kk + fg));
#pragma unroll
      for (int j = 0; j < FN; ++j) bfr[j] = ld16(st + A_BYTES + swz(wc * TN + j * 16 + fr, 4 * kk + fg));
#pragma unroll
      for (int i = 0; i < FM; ++i)
#pragma unroll
        for (int j = 0; j < FN; ++j)
          // DIRECT: MFMA(W, A) = C^T fragments -> a lane owns 4 consecutive columns of one row
          acc[i][j] = DIRECT ? __builtin_amdgcn_mfma_f32_16x16x32_bf16(__builtin_bit_cast(bf16x8, bfr[j]),
                                                                      __builtin_bit_cast(bf16x8, af[i]), acc[i][j], 0, 0, 0)
                             : __builtin_amdgcn_mfma_f32_16x16x32_bf16(__builtin_bit_cast(bf16x8, af[i]),
                                                                      __builtin_bit_cast(bf16x8, bfr[j]), acc[i][j], 0, 0, 0);
    }
    asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
    __builtin_amdgcn_s_barrier();               // stage ks fully read: its buffer may be refilled
  }
  }

  if constexpr (DIRECT) {
    // lane holds C[m = 16i + fr][n = 16j + 4fg + r], r = 0..3 -> 8-byte stores
#pragma unroll
    for (int j = 0; j < FN; ++j) {
      const int n = n0 + wc * TN + 16 * j + 4 * fg;
      if (n >= g.N) continue;
      const bool full = n + 4 <= g.N;
      const f32x4 bv = dbias[j];                  // loaded before the K loop
#pragma unroll
      for (int i = 0; i < FM; ++i) {
        const int m = m0 + wr * TM + 16 * i + fr;
        if (m >= g.M) continue;
        float v[4];
#pragma unroll
        for (int r = 0; r < 4; ++r) v[r] = acc[i][j][r] + bv[r];
        auto add_res = [&]() {
          if (full) {
            v[0] += __uint_as_float(dres[i][j].x << 16);
            v[1] += __uint_as_float(dres[i][j].x & 0xffff0000u);
            v[2] += __uint_as_float(dres[i][j].y << 16);
            v[3] += __uint_as_float(dres[i][j].y & 0xffff0000u);
          } else {
            const bf16* rp = (const bf16*)g.R + (size_t)(g.r_period > 0 ? m % g.r_period : m) * g.ldr + n;
            for (int r = 0; r < 4 && n + r < g.N; ++r) v[r] += to_f32(rp[r]);
          }
        };
        const bool rpost = XA && g.res_post;
        if (!PIN && g.R && !rpost) add_res();
        if constexpr (XA) {
          if (g.act) {
#pragma unroll
            for (int r = 0; r < 4; ++r) v[r] = apply_act(v[r], g.act);
          }
        } else if (g.act) {
#pragma unroll
          for (int r = 0; r < 4; ++r) v[r] = fmaxf(v[r], 0.f);
        }
        if (!PIN && g.R && rpost) add_res();
        if (g.out_f32) {
          float* cp = (float*)g.C + (size_t)m * g.ldc + n;
          if (full) st16(cp, pack16<float>(v));
          else for (int r = 0; r < 4 && n + r < g.N; ++r) cp[r] = v[r];
        } else {
          bf16* cp = (bf16*)g.C + (size_t)m * g.ldc + n;
          if (full) st8(cp, u32x2{pack_out2(v[0], v[1], g.out_f16), pack_out2(v[2], v[3], g.out_f16)});
          else for (int r = 0; r < 4 && n + r < g.N; ++r) store_out1(cp, r, v[r], g.out_f16);
        }
      }
    }
    return;
  }

  // ---- epilogue in 64-row passes through an fp32 LDS tile
#pragma unroll
  for (int pp = NPRE; pp < NPASS; ++pp) fetch_res(pp);
  float* ct = reinterpret_cast<float*>(smem);
#pragma unroll
  for (int pass = 0; pass < NPASS; ++pass) {
    const int r0 = pass * EPI_ROWS;
#pragma unroll
    for (int i = 0; i < FM; ++i) {
      const int rb = frag_row(i);                 // fragment rows [rb, rb+16)
      if (rb >= r0 && rb < r0 + EPI_ROWS) {
#pragma unroll
        for (int j = 0; j < FN; ++j)
#pragma unroll
          for (int r = 0; r < 4; ++r)
            ct[(rb - r0 + fg * 4 + r) * EPI_LD + frag_col(j) + fr] = acc[i][j][r];
      }
    }
    __syncthreads();
    if (g.vt_T > 0) {
      // head-transposed store: column n = grp*256 + hd -> C[((grp*vt_B + b)*256 + hd)*T + tok]
      for (int it = tid; it < (EPI_ROWS / 8) * BN; it += NT) {
        const int col = it % BN, rg = (it / BN) * 8, n = n0 + col, m = m0 + r0 + rg;
        if (n >= g.N || m >= g.M) continue;
        float bv = g.bias ? g.bias[n] : 0.f;
        float v[8];
#pragma unroll
        for (int e = 0; e < 8; ++e) v[e] = ct[(rg + e) * EPI_LD + col] + bv;
        const int grp = n >> 8, hd = n & 255;
        const int b = m / g.vt_T, tok = m - b * g.vt_T;
        if ((g.vt_T & 7) == 0 && m + 8 <= g.M) {
          bf16* row = (bf16*)g.C + ((size_t)(grp * g.vt_B + b) * 256 + hd) * g.vt_T;
          const u32x4 pk = pack_out8(v, g.out_f16);
          if (g.vt_swz) {                        // the two quads land apart (vt_pos)
            st8(row + vt_pos(tok), u32x2{pk.x, pk.y});
            st8(row + vt_pos(tok + 4), u32x2{pk.z, pk.w});
          } else {
            st16(row + tok, pk);
          }
        } else {
          for (int e = 0; e < 8 && m + e < g.M; ++e) {
            const int me = m + e, be = me / g.vt_T, te = me - be * g.vt_T;
            store_out1(g.C, ((size_t)(grp * g.vt_B + be) * 256 + hd) * g.vt_T + (g.vt_swz ? vt_pos(te) : te), v[e],
                       g.out_f16);
          }
        }
      }
    } else {
      const int cg = ecg, n = en;
      if (n < g.N) {
        const bool full = efull;
        const float* bv = ebias;
#pragma unroll
        for (int q = 0; q < RPT; ++q) {
          const int rr = ert + q * RSTEP, m = m0 + r0 + rr;
          if (m >= g.M) continue;
          float v[8];
#pragma unroll
          for (int e = 0; e < 8; ++e) v[e] = ct[rr * EPI_LD + cg + e] + bv[e];
          auto add_res = [&]() {
            if (full) {
              float f[8];
              unpack16<bf16>(rres[pass][q], f);
#pragma unroll
              for (int e = 0; e < 8; ++e) v[e] += f[e];
            } else {
              const bf16* rp = (const bf16*)g.R + (size_t)(g.r_period > 0 ? m % g.r_period : m) * g.ldr + n;
              for (int e = 0; e < 8 && n + e < g.N; ++e) v[e] += to_f32(rp[e]);
            }
          };
          const bool rpost = XA && g.res_post;
          if (!PIN && g.R && !rpost) add_res();
          if constexpr (LN) {
            // fused post-norm LayerNorm (N == BN == 256): a row's 32 column groups are the 32
            // lanes of one half-wave, so the row statistics are five xor-shuffles away
            float sm = 0.f;
#pragma unroll
            for (int e = 0; e < 8; ++e) sm += v[e];
#pragma unroll
            for (int o = 1; o < 32; o <<= 1) sm += __shfl_xor(sm, o, 64);
            const float mean = sm * (1.f / 256);
            float sq = 0.f;
#pragma unroll
            for (int e = 0; e < 8; ++e) sq += (v[e] - mean) * (v[e] - mean);
#pragma unroll
            for (int o = 1; o < 32; o <<= 1) sq += __shfl_xor(sq, o, 64);
            const float rs = rsqrtf(sq * (1.f / 256) + 1e-5f);
#pragma unroll
            for (int e = 0; e < 8; ++e) v[e] = (v[e] - mean) * rs * elg[e] + elb[e];
          }
          if constexpr (XA) {
            if (g.act) {
#pragma unroll
              for (int e = 0; e < 8; ++e) v[e] = apply_act(v[e], g.act);
            }
          } else if (g.act) {
#pragma unroll
            for (int e = 0; e < 8; ++e) v[e] = fmaxf(v[e], 0.f);
          }
          if (!PIN && g.R && rpost) add_res();
          if (g.out_f32) {
            float* cp = (float*)g.C + (size_t)m * g.ldc + n;
            if (full) {
              st16(cp, pack16<float>(v));
              st16(cp + 4, pack16<float>(v + 4));
            } else {
              for (int e = 0; e < 8 && n + e < g.N; ++e) cp[e] = v[e];
            }
          } else {
            bf16* cp = (bf16*)g.C + (size_t)m * g.ldc + n;
            if (full) {
              st16(cp, pack_out8(v, g.out_f16));
            } else {
              for (int e = 0; e < 8 && n + e < g.N; ++e) store_out1(cp, e, v[e], g.out_f16);
            }
          }
        }
      }
    }
    __syncthreads();
  }
}

template <int BN>
int launch_bn(const GemmArgs& g, int mode, hipStream_t s) {
  const int tiles = ((g.M + BM - 1) / BM) * ((g.N + BN - 1) / BN);
  dim3 grid(tiles), block(NT);
  if (g.act > ACT_RELU || g.res_post) {
    if (g.ln_g) return -1;
    if (mode == GEMM_CONV)
      hipLaunchKernelGGL((gemm2_kernel<BN, GEMM_CONV, false, false, 2, true>), grid, block, 0, s, g);
    else
      hipLaunchKernelGGL((gemm2_kernel<BN, GEMM_LINEAR, false, false, 2, true>), grid, block, 0, s, g);
    return (int)hipGetLastError();
  }
  // SPE_GEMM2_PIN=0: residual-free convs on the compiler-scheduled loop (A/B knob).  The other
  // convs and linear problems stage with global_load_lds (buffer-load staging without the pinned
  // schedule measured neutral, 4806 vs 4786 img/s, and was removed)
  static const int pin = [] { const char* e = getenv("SPE_GEMM2_PIN"); return e ? atoi(e) : 1; }();
  constexpr long long LIM = (1ll << 31) - (1 << 20);          // 32-bit buffer offsets
  const bool bfits = (long long)g.N * g.ldb * 2 < LIM;
  if (mode == GEMM_CONV) {
    const long long abytes = (long long)((g.M + g.Ho * g.Wo - 1) / (g.Ho * g.Wo)) * g.H * g.W * g.Cin * 2;
    // (the stem's tap-major K, Cin = 8, measured slower pinned: 0.33 -> 0.40 ms)
    const bool kpos_scalar = conv_channel_blocked(g.Cin, g.KH * g.KW) || g.KH * g.KW == 1;
    const bool fits = abytes < LIM && bfits;
    if (pin && !g.R && kpos_scalar && fits)
      hipLaunchKernelGGL((gemm2_kernel<BN, GEMM_CONV, false, false, 2, false, true>), grid, block, 0, s, g);
    else
      hipLaunchKernelGGL((gemm2_kernel<BN, GEMM_CONV, false>), grid, block, 0, s, g);
  } else {
    if constexpr (BN == 256) {
      if (g.ln_g) {
        hipLaunchKernelGGL((gemm2_kernel<BN, GEMM_LINEAR, true>), grid, block, 0, s, g);
        return (int)hipGetLastError();
      }
    }
    if constexpr (BN == 256) {
      if (g.K >= P8_MIN_K) {
        hipLaunchKernelGGL((gemm2_kernel<BN, GEMM_LINEAR, false, true>), grid, block, 0, s, g);
        return (int)hipGetLastError();
      }
    }
    hipLaunchKernelGGL((gemm2_kernel<BN, GEMM_LINEAR, false>), grid, block, 0, s, g);
  }
  return (int)hipGetLastError();
}

// one-stage 256x128 tiles, two workgroups per CU (see NST above)
int launch_st1(const GemmArgs& g, hipStream_t s) {
  const int tiles = ((g.M + BM - 1) / BM) * ((g.N + 127) / 128);
  hipLaunchKernelGGL((gemm2_kernel<128, GEMM_LINEAR, false, false, 1>), dim3(tiles), dim3(NT), 0, s, g);
  return (int)hipGetLastError();
}
// Short-K linear problems take the one-stage kernel when the grid holds >= 2 tiles per
// workgroup slot.  Measured at the B = 64 bench shapes (kbench): 256x128 + residual 0.118 ->
// 0.097 ms, 256x256 + residual (K = 64) 0.194 -> 0.182, q/k projection + pos.W^T 0.121 ->
// 0.113, layer2/3 conv3 + residual -7 / -8 %; a plain K = 64, N = 256 store got slower
// (0.129 -> 0.138) and stays on the two-stage kernel.  SPE_GEMM_ST1_K overrides the K bound
// (0 disables) for A/B runs.
int st1_max_k() {
  static const int v = [] { const char* e = getenv("SPE_GEMM_ST1_K"); return e ? atoi(e) : 256; }();
  return v;
}
bool use_st1(const GemmArgs& g, int mode) {
  if (mode != GEMM_LINEAR || g.K > st1_max_k() || g.N < 128 || g.ln_g) return false;
  if (!g.R && g.vt_T == 0 && g.N >= 256) return false;
  return ((g.M + BM - 1) / BM) * ((g.N + 127) / 128) >= 512;
}

}  // namespace

namespace {

// ---------------------------------------------------------------- few-row GEMM (decoder, M = B*Q)
// 64x64 tile, 4 waves (2x2, 32x32 each), the WHOLE K extent (<= 256) staged by one round of
// global_load_lds: a single memory round trip per tile instead of one per 64-deep K-step, which
// is what bounds these latency-limited problems.  Stores straight from the accumulators (C^T
// fragments for row-major output, C fragments for the head-transposed V^T store).
constexpr int SM_T = 64, SM_NT = 256, SM_KMAX = 256;

template <bool VT>
__global__ __launch_bounds__(SM_NT) void gemm_small_kernel(GemmArgs g) {
  constexpr int ROWB = SM_KMAX * 2;                  // 512 B LDS row (K = 256 bf16)
  __shared__ __attribute__((aligned(1024))) char lds[2 * SM_T * ROWB];   // A tile | W tile
  const int tid = threadIdx.x, lane = tid & 63, wid = __builtin_amdgcn_readfirstlane(tid >> 6);
  const int tilesN = (g.N + SM_T - 1) / SM_T;
  const int m0 = (blockIdx.x / tilesN) * SM_T, n0 = (blockIdx.x % tilesN) * SM_T;
  const char* zero = reinterpret_cast<const char*>(g_zero_line);
  // 64 wave-instructions of 1 KB (2 rows x 512 B); wave w issues 8 for A then 8 for W.  LDS row
  // r, 16-byte chunk c lives at slot c ^ (r & 15) (conflict-free fragment reads): lane slot s
  // fetches source chunk s ^ (r & 15).
#pragma unroll
  for (int i = 0; i < 16; ++i) {
    const int ins = wid * 16 + i, isB = ins >= 32, r = 2 * (ins & 31) + (lane >> 5);
    const int c = (lane & 31) ^ (r & 15), k = c * 8;
    const char* src = zero;
    if (!isB) {
      const int m = m0 + r;
      if (m < g.M && k < g.K) src = (const char*)g.A + ((size_t)m * g.lda + k) * 2;
    } else {
      const int n = n0 + r;
      if (n < g.N && k < g.K) src = (const char*)g.B + ((size_t)n * g.ldb + k) * 2;
    }
    __builtin_amdgcn_global_load_lds((const void*)src, (lds_ptr_t)(lds + ins * 1024), 16, 0, 0);
  }
  const int fg = lane >> 4, fr = lane & 15, wr = wid >> 1, wc = wid & 1;
  // epilogue operands fetched while the tile is in flight
  f32x4 bias[2];
  u32x2 res[2][2];
#pragma unroll
  for (int j = 0; j < 2; ++j) {
    bias[j] = f32x4{0.f, 0.f, 0.f, 0.f};
#pragma unroll
    for (int i = 0; i < 2; ++i) res[i][j] = u32x2{0, 0};
    if constexpr (!VT) {
      const int n = n0 + wc * 32 + 16 * j + 4 * fg;
      if (g.bias && n + 4 <= g.N) bias[j] = *reinterpret_cast<const f32x4*>(g.bias + n);
      else if (g.bias)
        for (int r = 0; r < 4; ++r) bias[j][r] = n + r < g.N ? g.bias[n + r] : 0.f;
#pragma unroll
      for (int i = 0; i < 2; ++i) {
        const int m = m0 + wr * 32 + 16 * i + fr;
        if (g.R && m < g.M && n + 4 <= g.N)
          res[i][j] = ld8((const bf16*)g.R + (size_t)(g.r_period > 0 ? m % g.r_period : m) * g.ldr + n);
      }
    }
  }
  wait_vmcnt<0>();
  __syncthreads();
  f32x4 acc[2][2];
#pragma unroll
  for (int i = 0; i < 2; ++i)
#pragma unroll
    for (int j = 0; j < 2; ++j) acc[i][j] = f32x4{0.f, 0.f, 0.f, 0.f};
  const int nks = (g.K + 31) / 32;
  for (int kk = 0; kk < nks; ++kk) {
    u32x4 af[2], wf[2];
#pragma unroll
    for (int i = 0; i < 2; ++i) {
      const int ra = wr * 32 + 16 * i + fr, rb = wc * 32 + 16 * i + fr, c = 4 * kk + fg;
      af[i] = ld16(lds + ra * ROWB + ((c ^ (ra & 15)) << 4));
      wf[i] = ld16(lds + SM_T * ROWB + rb * ROWB + ((c ^ (rb & 15)) << 4));
    }
#pragma unroll
    for (int i = 0; i < 2; ++i)
#pragma unroll
      for (int j = 0; j < 2; ++j) {
        const bf16x8 a = __builtin_bit_cast(bf16x8, af[i]), b = __builtin_bit_cast(bf16x8, wf[j]);
        acc[i][j] = VT ? __builtin_amdgcn_mfma_f32_16x16x32_bf16(a, b, acc[i][j], 0, 0, 0)
                       : __builtin_amdgcn_mfma_f32_16x16x32_bf16(b, a, acc[i][j], 0, 0, 0);
      }
  }
#pragma unroll
  for (int i = 0; i < 2; ++i)
#pragma unroll
    for (int j = 0; j < 2; ++j) {
      if constexpr (VT) {
        // C fragment: 4 consecutive tokens m = .. + 4fg + r of column n
        const int n = n0 + wc * 32 + 16 * j + fr, m = m0 + wr * 32 + 16 * i + 4 * fg;
        if (n >= g.N) continue;
        const float bv = g.bias ? g.bias[n] : 0.f;
        const int grp = n >> 8, hd = n & 255;
        for (int r = 0; r < 4 && m + r < g.M; ++r) {
          const int me = m + r, be = me / g.vt_T, te = me - be * g.vt_T;
          store_out1(g.C, ((size_t)(grp * g.vt_B + be) * 256 + hd) * g.vt_T + (g.vt_swz ? vt_pos(te) : te),
                     acc[i][j][r] + bv, g.out_f16);
        }
      } else {
        // C^T fragment: 4 consecutive columns n = .. + 4fg + r of row m
        const int m = m0 + wr * 32 + 16 * i + fr, n = n0 + wc * 32 + 16 * j + 4 * fg;
        if (m >= g.M || n >= g.N) continue;
        const bool full = n + 4 <= g.N;
        float v[4];
#pragma unroll
        for (int r = 0; r < 4; ++r) v[r] = acc[i][j][r] + bias[j][r];
        auto add_res = [&]() {
          if (full) {
            v[0] += __uint_as_float(res[i][j].x << 16);
            v[1] += __uint_as_float(res[i][j].x & 0xffff0000u);
            v[2] += __uint_as_float(res[i][j].y << 16);
            v[3] += __uint_as_float(res[i][j].y & 0xffff0000u);
          } else {
            const bf16* rp = (const bf16*)g.R + (size_t)(g.r_period > 0 ? m % g.r_period : m) * g.ldr + n;
            for (int r = 0; r < 4 && n + r < g.N; ++r) v[r] += to_f32(rp[r]);
          }
        };
        if (g.R && !g.res_post) add_res();
        if (g.act)
          for (int r = 0; r < 4; ++r) v[r] = apply_act(v[r], g.act);
        if (g.R && g.res_post) add_res();
        if (g.out_f32) {
          float* cp = (float*)g.C + (size_t)m * g.ldc + n;
          if (full) st16(cp, pack16<float>(v));
          else for (int r = 0; r < 4 && n + r < g.N; ++r) cp[r] = v[r];
        } else {
          bf16* cp = (bf16*)g.C + (size_t)m * g.ldc + n;
          if (full) st8(cp, u32x2{pack_out2(v[0], v[1], g.out_f16), pack_out2(v[2], v[3], g.out_f16)});
          else for (int r = 0; r < 4 && n + r < g.N; ++r) store_out1(cp, r, v[r], g.out_f16);
        }
      }
    }
}

}  // namespace

bool spe_gemm_ln_fusable(const GemmArgs& g) {
  const int tiles = (g.M + BM - 1) / BM;
  return g.N == 256 && g.vt_T == 0 && tiles >= 256 && g.K % 8 == 0 && g.ldb % 64 == 0 && g.lda % 8 == 0 &&
         g.ldc % 8 == 0 && (!g.R || g.ldr % 8 == 0);
}

// Returns 1 when the problem is not for this kernel (caller falls back to gemm.hip).
int spe_launch_gemm2(const GemmArgs& g, int mode, hipStream_t s) {
  if (mode != GEMM_LINEAR && mode != GEMM_CONV) return 1;
  if (g.M <= 0 || g.N <= 0) return 0;
  // conv chunks are 16 bytes of one pixel (Cin % 8 == 0), or two horizontally adjacent pixels
  // (Cin == 4: the pair-packed stem, pre-padded input, even KW, every tap in range)
  const bool pairs = mode == GEMM_CONV && g.Cin == 4 && g.pad == 0 && g.KW % 2 == 0 &&
                     (g.Wo - 1) * g.stride + g.KW <= g.W && (g.Ho - 1) * g.stride + g.KH <= g.H;
  if (g.K % 8 || g.ldb % 64 || g.lda % 8 || (mode == GEMM_CONV && g.Cin % 8 && !pairs)) return 1;
  if (g.out_f32 ? (g.ldc % 4) : (g.ldc % 8)) return 1;
  if (g.R && g.ldr % 8) return 1;
  if (mode == GEMM_CONV) {
    const int rc = spe_launch_pconv(g, s);         // 3x3 stride-1 convs: patch-staged kernel (pconv.hip)
    if (rc != 1) return rc;
  }
  if (mode == GEMM_LINEAR && g.ln_g) {
    const int rc = spe_launch_lnproj(g, s);       // out-projection + residual + LayerNorm (lnproj.hip)
    if (rc != 1) return rc;
  }
  {
    const int rc = spe_launch_sgemm(g, mode, s);   // short-K streaming kernel (gemm_stream.hip)
    if (rc != 1) return rc;
  }
  if (g.ln_g) {                                  // fused LayerNorm needs whole rows in one 256-wide tile
    if (g.N != 256 || g.vt_T > 0 || mode != GEMM_LINEAR || !spe_gemm_ln_fusable(g)) return -5;
    return launch_bn<256>(g, mode, s);
  }
  if (mode == GEMM_LINEAR && g.M <= 4096 && g.K <= SM_KMAX) {   // few rows: one-shot K, 64x64 tiles
    const int tiles = ((g.M + SM_T - 1) / SM_T) * ((g.N + SM_T - 1) / SM_T);
    if (g.vt_T > 0) hipLaunchKernelGGL(gemm_small_kernel<true>, dim3(tiles), dim3(SM_NT), 0, s, g);
    else hipLaunchKernelGGL(gemm_small_kernel<false>, dim3(tiles), dim3(SM_NT), 0, s, g);
    return (int)hipGetLastError();
  }
  if (use_st1(g, mode) && g.act <= ACT_RELU && !g.res_post) return launch_st1(g, s);
  int bn = (g.N <= 64 && g.vt_T == 0) ? 64 : g.N <= 128 ? 128 : 256;   // BN 64 has no V^T store
  // (128-wide tiles for the under-filled 256-wide conv grids measured neutral in the pipelined
  // bench -- the other streams fill the idle CUs -- and were removed)
  const int tiles = ((g.M + BM - 1) / BM) * ((g.N + bn - 1) / bn);
  // too few tiles for the large-tile kernel: the 128x128 kernel.  (169 tiles of 256x256 on the
  // layer3 convs, M = B*26*26, still beat 676 tiles of the 128x128 kernel by 12-18 %.)
  if (tiles < 128) return 1;
  return bn == 64 ? launch_bn<64>(g, mode, s) : bn == 128 ? launch_bn<128>(g, mode, s) : launch_bn<256>(g, mode, s);
}
