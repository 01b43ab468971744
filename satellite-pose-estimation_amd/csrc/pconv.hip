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
// * One barrier per K-step, software-pipelined across it: a step's fragments are read from LDS
//   during the previous step's MFMAs, and the weight DMA of step s+2 is issued at step s's
//   barrier, so neither an LDS read nor a DMA is waited on right behind a barrier (the form with
//   the reads after the barrier and half a step of DMA lead ran the MFMA pipe ~35-40 % busy).
// * Fragment addresses: the A swizzle key does not depend on the fragment, so each (tap, kk)
//   costs one per-lane offset and one add per fragment.
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

// s_waitcnt through the builtin (not inline asm), so the compiler's own wait insertion sees it:
// a pending-unknown counter (e.g. a kernel-argument s_load it issued before an asm wait) makes
// it fall back to lgkmcnt(0) at the next LDS use.  gfx9 encoding: vmcnt [3:0] + [15:14],
// expcnt [6:4], lgkmcnt [11:8].
constexpr int waitcnt_enc(int vm, int lgkm) { return (vm & 15) | ((vm >> 4) << 14) | (7 << 4) | ((lgkm & 15) << 8); }
template <int N>
SPE_DEV void wait_vm() { __builtin_amdgcn_s_waitcnt(waitcnt_enc(N, 15)); }
SPE_DEV void wait_lgkm0() { __builtin_amdgcn_s_waitcnt(waitcnt_enc(63, 0)); }

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

  // ---- fragment read addresses.  A fragment i row fr = tile pixel m -> patch row of tap (0, 0),
  // as a byte offset.  The swizzle key of pixel m at tap (kh, kw) is (m + kh*TW + kw) & 7 and
  // m = wr*TMw + 16i + fr with TMw % 16 == 0, so the key is (fr + kh*TW + kw) & 7 for every
  // fragment of the lane: one per-lane offset per (tap, kk) serves all FM fragments.
  static_assert(TMw % 16 == 0, "key independent of the fragment");
  const int fg = lane >> 4, fr = lane & 15;
  int pb[FM];
#pragma unroll
  for (int i = 0; i < FM; ++i) {
    const int m = wr * TMw + 16 * i + fr;
    const int th = m / p.TW, tw = m - th * p.TW;
    pb[i] = th < p.TH ? (th * p.PW + tw) * 128 : 0;       // rows past the block read row 0 (discarded)
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

  // fragments of step (cb, tap), half kk: A from the patch of cb at the tap's row shift, B from
  // weight stage ws
  auto read_step = [&](u32x4* a, u32x4* bw, int cb, int tap, int ws, int kk) {
    const int kh = tap / 3, kw = tap - 3 * (tap / 3);
    const int sbase = (NPB == 2 ? (cb & 1) * PBYTES : 0) + (kh * p.PW + kw) * 128;
    const int t = (((fg ^ ((fr + kh * p.TW + kw) & 7)) << 4) + sbase) ^ (kk << 6);
    const char* wcur = wst + ws * WBYTES;
#pragma unroll
    for (int j = 0; j < FN; ++j) bw[j] = ld16(wcur + (brd[j] ^ (kk << 6)));
#pragma unroll
    for (int i = 0; i < FM; ++i) a[i] = ld16(smem + pb[i] + t);
  };
  auto mma = [&](const u32x4* af, const u32x4* bf) {
#pragma unroll
    for (int i = 0; i < FM; ++i)
#pragma unroll
      for (int j = 0; j < FN; ++j)
        acc[i][j] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(__builtin_bit_cast(bf16x8, bf[j]),
                                                            __builtin_bit_cast(bf16x8, af[i]), acc[i][j], 0, 0, 0);
  };
  auto sync = [&]() {
    wait_vm<0>();
    wait_lgkm0();
    __builtin_amdgcn_s_barrier();
  };

  // Pipeline.  Step s's fragments are read during iteration s-1, so no MFMA waits on an LDS
  // read issued behind a barrier; iteration s multiplies kk = 0 of step s, then at the barrier
  // (every wave's DMA of step s+1 landed, every wave done reading step s's weight stage) issues
  // step s+2's weights into that stage -- a whole iteration ahead of their use -- reads step
  // s+1's kk = 0 fragments into the registers the kk = 0 MFMAs just consumed, multiplies kk = 1,
  // and reads step s+1's kk = 1 fragments.  Two weight stages suffice.
  const int cbs = Cin >> 6, steps = 9 * cbs;
#pragma unroll
  for (int j = 0; j < PPW; ++j) issue_patch(0, 0, j);
  issue_w(0, 0);
  issue_w(1, 1);                                          // (steps >= 9)
  wait_vm<WPW>();                                         // patch 0 + step 0's weights
  wait_lgkm0();
  __builtin_amdgcn_s_barrier();
  u32x4 a0[FM], a1[FM], b0[FN], b1[FN];
  read_step(a0, b0, 0, 0, 0, 0);
  read_step(a1, b1, 0, 0, 0, 1);
  int cb = 0, tap = 0;
  // (the last step is peeled: every back edge then carries the same 10 pending fragment reads,
  // and the compiler's wait at the top counts only those of the next kk = 0 half)
  for (int s = 0; s + 1 < steps; ++s) {
    mma(a0, b0);
    __builtin_amdgcn_sched_barrier(0);
    int tapn = tap + 1, cbn = cb;
    if (tapn == 9) { tapn = 0; ++cbn; }
    sync();
    if (s + 2 < steps) issue_w(s + 2, s & 1);
    if constexpr (NPB == 2) {
      // the next channel block's whole patch at its first tap (compile-time piece indices: a
      // piece per tap, poff[tap], made the compiler version the loop on "this tap issues a
      // piece" with ~130 v_mov of the fragment registers on 5 of 9 taps -- 1.8 VALU per MFMA)
      if (tap == 0 && cb + 1 < cbs) {
#pragma unroll
        for (int j = 0; j < PPW; ++j) issue_patch(cb + 1, (cb + 1) & 1, j);
      }
    } else {
      if (cbn != cb) {                                    // one buffer: refill it once every wave is done
#pragma unroll
        for (int j = 0; j < PPW; ++j) issue_patch(cbn, 0, j);
        sync();
      }
    }
    read_step(a0, b0, cbn, tapn, (s + 1) & 1, 0);
    __builtin_amdgcn_sched_barrier(0);
    mma(a1, b1);
    __builtin_amdgcn_sched_barrier(0);
    read_step(a1, b1, cbn, tapn, (s + 1) & 1, 1);
    tap = tapn;
    cb = cbn;
  }
  mma(a0, b0);
  mma(a1, b1);

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
    PcChoice c2{}, c3{};
    const bool a = choose_block(g, 192, 256, cus, c), bq = choose_block(g, 256, 256, cus, c2),
               h = choose_block(g, 256, 128, cus, c3);
    if (!a && !bq && !h) return 1;
    // per-tile time ~ BM x BN: the fewest rounds x tile area.  (At 32 images the 26x26 layer-3
    // convs are 128 tiles of 192 x 256 -- one round on half the chip; 192 tiles of 256 x 128
    // take one round of two thirds of the work each.)
    const long long big = 1LL << 62;
    const long long ca = a ? c.rounds * 192LL * 256 : big, cb = bq ? c2.rounds * 256LL * 256 : big,
                    ch = h ? c3.rounds * 256LL * 128 : big;
    if (ch < ca && ch < cb) return launch_pc<256, 128, 2>(g, c3.geo, s);
    if (cb <= ca) return launch_pc<256, 256, 2>(g, c2.geo, s);
    return launch_pc<192, 256, 2>(g, c.geo, s);
  }
  if (g.N % 128 == 0) {
    if (!choose_block(g, 256, 128, cus, c)) return 1;
    return launch_pc<256, 128, 2>(g, c.geo, s);
  }
  return 1;
}
