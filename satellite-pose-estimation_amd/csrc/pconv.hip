// Patch-staged implicit-GEMM 3x3 convolution (stride 1, pad 1) for bf16 NHWC activations:
// the ResNet-50 bottleneck conv2 of layers 1-3 and the neck's 3x3 (REV/models/backbone.py:114-125,
// torchvision Bottleneck.conv2; K order channel-block-major, spe_kernels.h conv_k_decode).
//
// gemm2.hip streams the A operand of an implicit-GEMM conv once per tap: every K-step
// (64 channels x one tap) re-fetches a 256-row im2col slice through L2, so the input window is
// read 9 times, and every lane decodes its own (ih, iw) bounds per step.  Here a workgroup owns a
// TH x TW block of output pixels of one image and stages the block's input patch
// ((TH+2) x (TW+2) pixels x 64 channels, zero padding included) into LDS ONCE per channel block;
// the 9 taps then read their A fragments from the patch at a scalar row shift
// (kh * (TW+2) + kw).  Per K-step only the weight slice (BN rows x 128 B) is staged.
//
// * Tile: BM output pixels (capacity; the block has TH*TW <= BM of them) x BN output channels,
//   8 waves, wave tile (BM/WM) x (BN/WN) of 16x16x32 bf16 MFMA fragments computed in the
//   transposed form (MFMA(W, A) = C^T fragments), so a lane owns 4 consecutive channels of one
//   pixel and stores them as one 8-byte write (no LDS epilogue).
// * LDS: NPB patch buffers of PCAP 128-byte rows (the next channel block's patch is fetched piece
//   by piece during the current block's first taps) + 2 weight stages.  Every 128-byte row holds
//   one pixel's 64-channel slice with the 16-byte chunk c of row q at slot c ^ (q & 7) -- applied
//   on the DMA source address -- so the 16 rows of a fragment read hit distinct banks whatever
//   the tap shift.
// * Staging: buffer_load ... lds (16 B per lane, 8 rows per wave-instruction); out-of-image taps
//   and rows past N use an out-of-range offset, which the buffer descriptor returns as zeros.
// * One barrier per K-step: wait for this wave's loads of step s, barrier (every wave's loads
//   landed and every wave finished reading step s-1's buffers), then issue step s+1's weights
//   into the freed stage and multiply step s.
// NPB = 1 (Cin = 64, the layer-1 conv2: one channel block, nothing to prefetch) sizes LDS and
// registers for two workgroups per CU, so one workgroup's patch fetch overlaps the other's work.
#include "spe_common.h"
#include "spe_kernels.h"

#include <algorithm>
#include <cstdlib>

namespace {

constexpr int PNT = 512;
constexpr int PCAP = 320;                   // patch capacity: (TH+2)*(TW+2) 128-byte rows
constexpr int PBAD = 0x7ffffff0;            // out-of-range buffer offset -> reads zeros
typedef __attribute__((address_space(3))) void* lds_ptr_t;

struct PcGeom {
  int TH, TW, nbh, nbw;                     // output block and block counts per image
  int tilesN;                               // N / BN
  int PW, PR;                               // patch row pitch (TW+2) and rows (TH+2)*(TW+2)
};

template <int N>
SPE_DEV void wait_vm() { asm volatile("s_waitcnt vmcnt(%0)" ::"n"(N) : "memory"); }

template <int BM, int BN, int NPB>
__global__ __launch_bounds__(PNT, NPB == 1 ? 2 : 1) void pconv_kernel(GemmArgs g, PcGeom p) {
  constexpr int WN = BN == 64 ? 1 : BN == 128 ? 2 : 4;
  constexpr int WM = 8 / WN;
  constexpr int TMw = BM / WM, TNw = BN / WN, FM = TMw / 16, FN = TNw / 16;
  static_assert(TMw % 16 == 0 && TNw % 16 == 0, "wave tile");
  constexpr int PBYTES = PCAP * 128, WBYTES = BN * 128;
  constexpr int PPW = (PCAP / 8 + 7) / 8;   // patch pieces per wave (upper bound)
  constexpr int WPW = BN / 64;              // weight pieces per wave per K-step
  __shared__ __attribute__((aligned(1024))) char smem[NPB * PBYTES + 2 * WBYTES];
  char* const wst = smem + NPB * PBYTES;

  const int tid = threadIdx.x, lane = tid & 63;
  const int wid = __builtin_amdgcn_readfirstlane(tid >> 6);
  const int wr = wid / WN, wc = wid % WN;
  const int t = xcd_remap(blockIdx.x, gridDim.x);
  const int nt = t % p.tilesN, st = t / p.tilesN;
  const int per_img = p.nbh * p.nbw;
  const int b = st / per_img, rblk = st - b * per_img;
  const int bh = rblk / p.nbw, bw = rblk - bh * p.nbw;
  const int oh0 = bh * p.TH, ow0 = bw * p.TW, n0 = nt * BN;
  const int the = min(p.TH, g.Ho - oh0), twe = min(p.TW, g.Wo - ow0);
  const int H = g.H, W = g.W, Cin = g.Cin;

  const __amdgpu_buffer_rsrc_t rsa = __builtin_amdgcn_make_buffer_rsrc(
      (void*)g.A, (short)0, (int)std::min<long long>((long long)(b + 1) * H * W * Cin * 2, PBAD), 0x00020000);
  const __amdgpu_buffer_rsrc_t rsb = __builtin_amdgcn_make_buffer_rsrc((void*)g.B, (short)0, g.N * g.ldb * 2, 0x00020000);

  // ---- DMA descriptors.  Wave-instruction (piece) i fills LDS rows 8i..8i+7; lane l writes row
  // 8i + l/8, slot l & 7, and so fetches chunk (l & 7) ^ (row & 7) of that row's source.
  const int lrow = lane >> 3;
  const int npieces = (p.PR + 7) >> 3;
  int poff[PPW];
#pragma unroll
  for (int j = 0; j < PPW; ++j) {
    const int q = (wid + 8 * j) * 8 + lrow;
    const int pr = q / p.PW, pc = q - pr * p.PW;
    const int ih = oh0 - 1 + pr, iw = ow0 - 1 + pc;
    const bool v = q < p.PR && ih >= 0 && ih < H && iw >= 0 && iw < W;
    poff[j] = v ? (((b * H + ih) * W + iw) * Cin + (((lane & 7) ^ (q & 7)) << 3)) * 2 : PBAD;
  }
  int boff[WPW];
#pragma unroll
  for (int j = 0; j < WPW; ++j) {
    const int row = (wid * WPW + j) * 8 + lrow, n = n0 + row;
    boff[j] = n < g.N ? (n * g.ldb + (((lane & 7) ^ (row & 7)) << 3)) * 2 : PBAD;
  }
  auto issue_patch = [&](int cb, int pbuf, int j) {
    if (wid + 8 * j < npieces) {
      const int off = poff[j] == PBAD ? PBAD : poff[j] + cb * 128;
      __builtin_amdgcn_raw_ptr_buffer_load_lds(rsa, (lds_ptr_t)(smem + pbuf * PBYTES + (wid + 8 * j) * 1024), 16, off,
                                               0, 0, 0);
    }
  };
  auto issue_w = [&](int s, int wbuf) {
#pragma unroll
    for (int j = 0; j < WPW; ++j) {
      const int off = boff[j] == PBAD ? PBAD : boff[j] + s * 128;
      __builtin_amdgcn_raw_ptr_buffer_load_lds(rsb, (lds_ptr_t)(wst + wbuf * WBYTES + (wid * WPW + j) * 1024), 16, off,
                                               0, 0, 0);
    }
  };

  // ---- fragment read addresses.  A fragment i row fr = tile pixel m -> patch row of tap (0, 0).
  const int fg = lane >> 4, fr = lane & 15;
  int pbase[FM];
#pragma unroll
  for (int i = 0; i < FM; ++i) {
    const int m = wr * TMw + 16 * i + fr;
    const int th = m / p.TW, tw = m - th * p.TW;
    pbase[i] = (th < p.TH) ? th * p.PW + tw : 0;          // rows past the block read row 0 (discarded)
  }
  int brd[FN];                                            // weight fragment byte offsets, kk = 0
#pragma unroll
  for (int j = 0; j < FN; ++j) {
    const int row = wc * TNw + 16 * j + fr;
    brd[j] = row * 128 + ((fg ^ (row & 7)) << 4);
  }

  f32x4 acc[FM][FN];
#pragma unroll
  for (int i = 0; i < FM; ++i)
#pragma unroll
    for (int j = 0; j < FN; ++j) acc[i][j] = f32x4{0.f, 0.f, 0.f, 0.f};

  const int cbs = Cin >> 6, steps = 9 * cbs;
#pragma unroll
  for (int j = 0; j < PPW; ++j) issue_patch(0, 0, j);
  issue_w(0, 0);
  int cb = 0, tap = 0;
  for (int s = 0; s < steps; ++s) {
    wait_vm<0>();
    asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
    __builtin_amdgcn_s_barrier();
    if (s + 1 < steps) issue_w(s + 1, (s + 1) & 1);
    if constexpr (NPB == 2) {
      // next channel block's patch, one piece per wave per tap (PPW <= 9 taps)
      if (cb + 1 < cbs) {
#pragma unroll
        for (int j = 0; j < PPW; ++j)
          if (j == tap) issue_patch(cb + 1, (cb + 1) & 1, j);
      }
    }
    const int kh = tap / 3, kw = tap - 3 * (tap / 3);
    const int toff = kh * p.PW + kw;
    const char* pst = smem + (NPB == 2 ? (cb & 1) * PBYTES : 0);
    const char* wcur = wst + (s & 1) * WBYTES;
    u32x4 af[2][FM], bfr[2][FN];
#pragma unroll
    for (int kk = 0; kk < 2; ++kk) {
#pragma unroll
      for (int j = 0; j < FN; ++j) bfr[kk][j] = ld16(wcur + (brd[j] ^ (kk << 6)));
#pragma unroll
      for (int i = 0; i < FM; ++i) {
        const int q = pbase[i] + toff;
        af[kk][i] = ld16(pst + ((q * 128 + ((fg ^ (q & 7)) << 4)) ^ (kk << 6)));
      }
    }
#pragma unroll
    for (int kk = 0; kk < 2; ++kk)
#pragma unroll
      for (int i = 0; i < FM; ++i)
#pragma unroll
        for (int j = 0; j < FN; ++j)
          acc[i][j] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(__builtin_bit_cast(bf16x8, bfr[kk][j]),
                                                              __builtin_bit_cast(bf16x8, af[kk][i]), acc[i][j], 0, 0, 0);
    if constexpr (NPB == 1) {
      if (tap == 8 && cb + 1 < cbs) {
        asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
        __builtin_amdgcn_s_barrier();                      // every wave done with this patch
#pragma unroll
        for (int j = 0; j < PPW; ++j) issue_patch(cb + 1, 0, j);
      }
    }
    if (++tap == 9) { tap = 0; ++cb; }
  }

  // ---- epilogue: lane owns C[pixel m = 16i + fr][channels 16j + 4fg .. +3] of its wave tile
#pragma unroll
  for (int j = 0; j < FN; ++j) {
    const int n = n0 + wc * TNw + 16 * j + 4 * fg;
    if (n >= g.N) continue;
    const f32x4 bv = g.bias ? *reinterpret_cast<const f32x4*>(g.bias + n) : f32x4{0.f, 0.f, 0.f, 0.f};
#pragma unroll
    for (int i = 0; i < FM; ++i) {
      const int m = wr * TMw + 16 * i + fr;
      const int th = m / p.TW, tw = m - th * p.TW;
      if (th >= the || tw >= twe) continue;
      const long long row = ((long long)b * g.Ho + oh0 + th) * g.Wo + ow0 + tw;
      float v[4];
#pragma unroll
      for (int r = 0; r < 4; ++r) {
        v[r] = acc[i][j][r] + bv[r];
        if (g.act) v[r] = fmaxf(v[r], 0.f);
      }
      st8((bf16*)g.C + row * g.ldc + n, u32x2{pack_out2(v[0], v[1], g.out_f16), pack_out2(v[2], v[3], g.out_f16)});
    }
  }
}

struct PcChoice {
  PcGeom geo;
  int rounds;
  double halo;
};

// Output block for a BM-pixel tile: the fewest rounds of workgroups over the chip, then the
// smallest patch per output pixel.
bool choose_block(const GemmArgs& g, int BM, int BN, int slots, PcChoice& best) {
  const int B = g.M / (g.Ho * g.Wo);
  bool found = false;
  for (int TW = std::min(g.Wo, BM); TW >= 1; --TW) {
    const int TH = std::min(g.Ho, BM / TW);
    if (TH < 1 || (TH + 2) * (TW + 2) > PCAP) continue;
    const int nbh = (g.Ho + TH - 1) / TH, nbw = (g.Wo + TW - 1) / TW;
    const long long tiles = (long long)B * nbh * nbw * (g.N / BN);
    const int rounds = (int)((tiles + slots - 1) / slots);
    const double halo = (double)(TH + 2) * (TW + 2) / ((double)g.Ho * g.Wo / (nbh * nbw));
    if (!found || rounds < best.rounds || (rounds == best.rounds && halo < best.halo)) {
      best.geo = PcGeom{TH, TW, nbh, nbw, g.N / BN, TW + 2, (TH + 2) * (TW + 2)};
      best.rounds = rounds;
      best.halo = halo;
      found = true;
    }
  }
  return found;
}

template <int BM, int BN, int NPB>
int launch_pc(const GemmArgs& g, const PcGeom& geo, hipStream_t s) {
  const int B = g.M / (g.Ho * g.Wo);
  const long long tiles = (long long)B * geo.nbh * geo.nbw * geo.tilesN;
  hipLaunchKernelGGL((pconv_kernel<BM, BN, NPB>), dim3((unsigned)tiles), dim3(PNT), 0, s, g, geo);
  spe_gemm_last_path = 3;
  return (int)hipGetLastError();
}

}  // namespace

// 1 = not a problem for this kernel (the caller takes gemm2 / gemm)
int spe_launch_pconv(const GemmArgs& g, hipStream_t s) {
  static const int en = [] { const char* e = getenv("SPE_PCONV"); return e ? atoi(e) : 1; }();
  if (!en) return 1;
  if (g.KH != 3 || g.KW != 3 || g.stride != 1 || g.pad != 1 || g.Ho != g.H || g.Wo != g.W) return 1;
  if (g.Cin % 64 || g.N % 64 || g.R || g.act > ACT_RELU || g.res_post || g.out_f32 || g.vt_T > 0 || g.ln_g) return 1;
  if (g.K != 9 * g.Cin || g.ldc % 4 || g.M % (g.Ho * g.Wo)) return 1;
  const long long abytes = (long long)g.M * g.Cin * 2;
  if (abytes >= PBAD || (long long)g.N * g.ldb * 2 >= PBAD) return 1;   // 32-bit buffer offsets
  if (g.bias && (reinterpret_cast<uintptr_t>(g.bias) & 15)) return 1;
  const int cus = spe_cu_count();
  PcChoice c{};
  if (g.N == 64) {
    if (!choose_block(g, 256, 64, 2 * cus, c)) return 1;
    return launch_pc<256, 64, 1>(g, c.geo, s);
  }
  if (g.N % 256 == 0) {
    PcChoice c2{};
    const bool a = choose_block(g, 192, 256, cus, c), bq = choose_block(g, 256, 256, cus, c2);
    if (!a && !bq) return 1;
    // per-tile time ~ BM: compare rounds x BM
    if (bq && (!a || (long long)c2.rounds * 256 <= (long long)c.rounds * 192)) return launch_pc<256, 256, 2>(g, c2.geo, s);
    return launch_pc<192, 256, 2>(g, c.geo, s);
  }
  if (g.N % 128 == 0) {
    if (!choose_block(g, 256, 128, cus, c)) return 1;
    return launch_pc<256, 128, 2>(g, c.geo, s);
  }
  return 1;
}
