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
//   one pixel's 64-channel slice, the 16-byte chunk c of patch pixel (pr, pc) at slot
//   c ^ ((pr * TW + pc) & 7) -- applied on the DMA source address.  The swizzle key is the pixel's
//   index in a TW-wide grid, not its LDS row (pitch TW + 2): a fragment's 16 consecutive output
//   pixels m then read keys (m + kh*TW + kw) & 7, consecutive for every tap even where the
//   fragment wraps to the next block row, so its reads hit distinct banks (keyed by the LDS row,
//   each wrap repeated two keys: 14-38 % of LDS cycles were bank conflicts).
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
  int abl;                                  // ablation bits (SPE_PCONV_ABL, timing only; 0 in the product)
};

template <int N>
SPE_DEV void wait_vm() { asm volatile("s_waitcnt vmcnt(%0)" ::"n"(N) : "memory"); }

template <int BM, int BN, int NPB>
__global__ __launch_bounds__(PNT, NPB == 1 ? 2 : 1) void pconv_kernel(GemmArgs g, PcGeom p) {
  constexpr int WN = BN == 64 ? 1 : BN == 128 ? 2 : 4;
  constexpr int WM = 8 / WN;
  constexpr int TMw = BM / WM, TNw = BN / WN, FM = TMw / 16, FN = TNw / 16;
  constexpr bool PF = FM <= 6;              // next-tap A prefetch (registers: the 8-fragment tile would spill)
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
    poff[j] = v ? (((b * H + ih) * W + iw) * Cin + (((lane & 7) ^ ((pr * p.TW + pc) & 7)) << 3)) * 2 : PBAD;
  }
  int boff[WPW];
#pragma unroll
  for (int j = 0; j < WPW; ++j) {
    const int row = (wid * WPW + j) * 8 + lrow, n = n0 + row;
    boff[j] = n < g.N ? (n * g.ldb + (((lane & 7) ^ ((((row >> 4) & 1) << 2) | (row & 3))) << 3)) * 2 : PBAD;
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
  int pbase[FM], pswz[FM];
#pragma unroll
  for (int i = 0; i < FM; ++i) {
    const int m = wr * TMw + 16 * i + fr;
    const int th = m / p.TW, tw = m - th * p.TW;
    const bool in = th < p.TH;                            // rows past the block read row 0 (discarded)
    pbase[i] = in ? th * p.PW + tw : 0;
    pswz[i] = in ? m : 0;
  }
  // Weight fragment j, lane row t = fr reads channel 16 * (t >> 2) + 4j + (t & 3) of the wave's
  // 64: the C^T fragment's lane (fg, fr) then holds channels 16 fg + 4j + r, i.e. over its four
  // j fragments 16 consecutive channels -- two 16-byte stores, 128 contiguous bytes per pixel
  // row across the four fg lanes (4-channel fragments stored 32 B at a time made the 256-wide
  // tiles write 2.4x their output bytes).  The weight rows' swizzle key keeps these reads
  // conflict-free: wkey(row) = bit 4 of the row : its low two bits.
  static_assert(TNw == 64, "epilogue packs 64 channels per wave");
  auto wkey = [](int row) { return (((row >> 4) & 1) << 2) | (row & 3); };
  int brd[FN];                                            // weight fragment byte offsets, kk = 0
#pragma unroll
  for (int j = 0; j < FN; ++j) {
    const int row = wc * TNw + 16 * (fr >> 2) + 4 * j + (fr & 3);
    brd[j] = row * 128 + ((fg ^ wkey(row)) << 4);
  }

  f32x4 acc[FM][FN];
#pragma unroll
  for (int i = 0; i < FM; ++i)
#pragma unroll
    for (int j = 0; j < FN; ++j) acc[i][j] = f32x4{0.f, 0.f, 0.f, 0.f};

  auto read_a = [&](u32x4* dst, const char* pst, int tap, int kk) {
    const int kh = tap / 3, kw = tap - 3 * (tap / 3);
    const int toff = kh * p.PW + kw, tswz = kh * p.TW + kw;
#pragma unroll
    for (int i = 0; i < FM; ++i) {
      const int q = pbase[i] + toff;
      dst[i] = ld16(pst + ((q * 128 + ((fg ^ ((pswz[i] + tswz) & 7)) << 4)) ^ (kk << 6)));
    }
  };
  auto mma = [&](const u32x4* af, const u32x4* bf) {
#pragma unroll
    for (int i = 0; i < FM; ++i)
#pragma unroll
      for (int j = 0; j < FN; ++j)
        acc[i][j] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(__builtin_bit_cast(bf16x8, bf[j]),
                                                            __builtin_bit_cast(bf16x8, af[i]), acc[i][j], 0, 0, 0);
  };

  const int cbs = Cin >> 6, steps = 9 * cbs;
#pragma unroll
  for (int j = 0; j < PPW; ++j) issue_patch(0, 0, j);
  issue_w(0, 0);
  int cb = 0, tap = 0;
  u32x4 a0[FM], a1[FM], an[PF ? FM : 1], b0[FN], b1[FN];
  bool pre = false;                                       // an holds this step's kk = 0 A fragments
  for (int s = 0; s < steps; ++s) {
    wait_vm<0>();
    asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
    if (!(p.abl & 1)) __builtin_amdgcn_s_barrier();
    const char* pst = smem + (NPB == 2 ? (cb & 1) * PBYTES : 0);
    const char* wcur = wst + (s & 1) * WBYTES;
#pragma unroll
    for (int j = 0; j < FN; ++j) b0[j] = ld16(wcur + brd[j]);
    if (PF && pre) {
#pragma unroll
      for (int i = 0; i < FM; ++i) a0[i] = an[i];
    } else {
      read_a(a0, pst, tap, 0);
    }
#pragma unroll
    for (int j = 0; j < FN; ++j) b1[j] = ld16(wcur + (brd[j] ^ 64));
    read_a(a1, pst, tap, 1);
    mma(a0, b0);
    __builtin_amdgcn_sched_barrier(0);
    // the next step's weights into the stage every wave finished reading before the barrier,
    // issued once this step's first MFMA group is queued
    if (s + 1 < steps && !(p.abl & 2)) issue_w(s + 1, (s + 1) & 1);
    if constexpr (NPB == 2) {
      if (cb + 1 < cbs) {                                 // next channel block's patch, a piece per tap
#pragma unroll
        for (int j = 0; j < PPW; ++j)
          if (j == tap) issue_patch(cb + 1, (cb + 1) & 1, j);
      }
    }
    // the next tap of the same channel block reads the same (complete) patch: its first A
    // fragments need no barrier
    pre = PF && tap < 8;
    if (PF && pre) read_a(an, pst, tap + 1, 0);
    mma(a1, b1);
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

  // ---- epilogue: lane owns C[pixel m = 16i + fr][channels nb .. nb + 15] of its wave tile
  const int nb = n0 + wc * TNw + 16 * fg;
  if (nb < g.N) {
    float bv[16];
#pragma unroll
    for (int q = 0; q < 4; ++q) {
      const f32x4 b4 = g.bias ? *reinterpret_cast<const f32x4*>(g.bias + nb + 4 * q) : f32x4{0.f, 0.f, 0.f, 0.f};
#pragma unroll
      for (int r = 0; r < 4; ++r) bv[4 * q + r] = b4[r];
    }
#pragma unroll
    for (int i = 0; i < FM; ++i) {
      const int m = wr * TMw + 16 * i + fr;
      const int th = m / p.TW, tw = m - th * p.TW;
      if (th >= the || tw >= twe) continue;
      const long long row = ((long long)b * g.Ho + oh0 + th) * g.Wo + ow0 + tw;
      float v[16];
#pragma unroll
      for (int j = 0; j < FN; ++j)
#pragma unroll
        for (int r = 0; r < 4; ++r) {
          const float x = acc[i][j][r] + bv[4 * j + r];
          v[4 * j + r] = g.act ? fmaxf(x, 0.f) : x;
        }
      bf16* cp = (bf16*)g.C + row * g.ldc + nb;
      st16(cp, pack_out8(v, g.out_f16));
      st16(cp + 8, pack_out8(v + 8, g.out_f16));
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
      best.geo = PcGeom{TH, TW, nbh, nbw, g.N / BN, TW + 2, (TH + 2) * (TW + 2), 0};
      best.rounds = rounds;
      best.halo = halo;
      found = true;
    }
  }
  return found;
}

template <int BM, int BN, int NPB>
int launch_pc(const GemmArgs& g, const PcGeom& geo, int abl, hipStream_t s) {
  const int B = g.M / (g.Ho * g.Wo);
  const long long tiles = (long long)B * geo.nbh * geo.nbw * geo.tilesN;
  PcGeom gp = geo;
  gp.abl = abl;
  hipLaunchKernelGGL((pconv_kernel<BM, BN, NPB>), dim3((unsigned)tiles), dim3(PNT), 0, s, g, gp);
  spe_gemm_last_path = 3;
  return (int)hipGetLastError();
}

}  // namespace

// 1 = not a problem for this kernel (the caller takes gemm2 / gemm)
int spe_launch_pconv(const GemmArgs& g, hipStream_t s) {
  static const int en = [] { const char* e = getenv("SPE_PCONV"); return e ? atoi(e) : 1; }();
  static const int abl = [] { const char* e = getenv("SPE_PCONV_ABL"); return e ? atoi(e) : 0; }();
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
    return launch_pc<256, 64, 1>(g, c.geo, abl, s);
  }
  if (g.N % 256 == 0) {
    PcChoice c2{};
    const bool a = choose_block(g, 192, 256, cus, c), bq = choose_block(g, 256, 256, cus, c2);
    if (!a && !bq) return 1;
    // per-tile time ~ BM: compare rounds x BM
    if (bq && (!a || (long long)c2.rounds * 256 <= (long long)c.rounds * 192)) return launch_pc<256, 256, 2>(g, c2.geo, abl, s);
    return launch_pc<192, 256, 2>(g, c.geo, abl, s);
  }
  if (g.N % 128 == 0) {
    if (!choose_block(g, 256, 128, cus, c)) return 1;
    return launch_pc<256, 128, 2>(g, c.geo, abl, s);
  }
  return 1;
}
