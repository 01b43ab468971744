// ResNet stem + max-pool in one pass (bf16 models, pair-packed stem; REV/models/backbone.py:133
// -> torchvision ResNet conv1 7x7/s2/p3 + bn1 + relu + maxpool 3x3/s2/p1):
//
//     pool[ph][pw] = max over stem rows 2ph-1..2ph+1, cols 2pw-1..2pw+1 of relu(conv(x) + b)
//
// The stem output (B x 208 x 208 x 64 at 416^2, 354 MB) is the max-pool's only consumer; the two
// launches wrote it and read it back.  Here it never leaves registers: 88 MB of pooled output is
// all that is written.
//
// * Input: the zero-bordered 4-channel image (spe_launch_pack_input_pad4, border 3) and the
//   pair-packed stem weights (registry.cpp: k = (kh*8 + kw)*4 + ci, K = 224, each 16-byte chunk
//   = taps kw, kw+1 of one kernel row).
// * A workgroup owns a band of PR = 4 pool rows of one image and a range of at most 8 column
//   fragments, and stages the band's input rows into LDS once (buffer_load ... lds, lane-linear,
//   out-of-image pixels zero through the descriptor's range check); 72 KB of LDS, so two
//   workgroups share a CU and one's patch DMA runs under the other's MFMAs (16 waves per row band
//   in one workgroup: 0.141 vs 0.114 ms per step).
// * A wave owns one 16-pixel fragment of stem columns 14f-1 .. 14f+14 (seven pool columns 7f ..
//   7f+6: fragments overlap by two columns, so a wave needs no neighbour) and walks the band's
//   stem rows two at a time: per kernel row kh one 16-byte A read per stem row (the pixel's taps
//   kw = 2fg, 2fg+1) and four W fragments shared by both rows, MFMA(W, A) so a lane holds 4
//   channels of one pixel.  The 3x3 window is reduced in registers: the vertical max over stem
//   rows 2ph-1 (kept from the previous step), 2ph, 2ph+1, then two in-row shuffles.  Bias and ReLU
//   commute with the max (relu(max(x) + b) = max(relu(x + b))), so they are applied once per pooled
//   value; stem positions outside the image (row -1, columns -1 and >= So) enter as -inf, as the
//   max-pool's implicit padding does.
#include "spe_common.h"
#include "spe_kernels.h"

#include <algorithm>
#include <cstdlib>

namespace {

typedef __attribute__((address_space(3))) void* lds_ptr_t;
// PR pool rows per band, at most MAXW waves (fragments) per workgroup, OCC workgroups per CU
#ifndef SPE_SP_PR
#define SPE_SP_PR 4
#endif
#ifndef SPE_SP_MAXW
#define SPE_SP_MAXW 8
#endif
#ifndef SPE_SP_OCC
#define SPE_SP_OCC 2
#endif
constexpr int PR = SPE_SP_PR, MAXW = SPE_SP_MAXW, OCC = SPE_SP_OCC;
constexpr int PROWS = 4 * PR + 7;          // input rows a band reads
constexpr int WPITCH = 464;                // LDS W row: 448 B of K = 224 + 16 B (29 chunks, odd: conflict-free)
constexpr int KCH = 28;                    // 16-byte chunks of a W row
constexpr int LDS_PATCH = (PROWS * (28 * MAXW + 10) * 8 + 1023) / 1024 * 1024;   // patch capacity
static_assert(OCC * (LDS_PATCH + 64 * WPITCH) <= 160 * 1024, "LDS");
constexpr int PBAD = 0x7ffffff0;           // out-of-range buffer offset -> reads zeros

struct SpGeom {
  int S, SP;                               // input size and padded pitch S + 6
  int So, Po;                              // stem and pool output sizes
  int nfrag, fpg, groups, bands;           // fragments per row, per workgroup; workgroups per band; bands
  int pwid, pitch;                         // patch width (pixels) and row pitch (bytes)
};

__global__ __launch_bounds__(64 * MAXW, OCC) void stempool_kernel(const bf16* __restrict__ x, const bf16* __restrict__ w, int ldw,
                                                           const float* __restrict__ bias, bf16* __restrict__ out, int ldo,
                                                           SpGeom p) {
  __shared__ __attribute__((aligned(1024))) char lds[LDS_PATCH + 64 * WPITCH];
  char* const patch = lds;
  char* const wl = lds + LDS_PATCH;
  const int tid = threadIdx.x, lane = tid & 63;
  const int wid = __builtin_amdgcn_readfirstlane(tid >> 6);
  const int nw = blockDim.x >> 6;
  int t = blockIdx.x;
  const int grp = t % p.groups;
  t /= p.groups;
  const int band = t % p.bands, b = t / p.bands;
  const int p0 = band * PR, npr = min(PR, p.Po - p0);
  const int f0 = grp * p.fpg;
  const int row0 = 4 * p0 - 2, col0 = 28 * f0 - 2;  // first padded-input row / column of the patch

  // ---- patch: PROWS rows x pwid pixels (8 bytes each), lane-linear 1 KB pieces
  // one descriptor per image (64-bit base), so the 32-bit offsets never grow with the batch
  const __amdgpu_buffer_rsrc_t rx = __builtin_amdgcn_make_buffer_rsrc(
      (void*)((const char*)x + (size_t)b * p.SP * p.SP * 8), (short)0,
      (int)std::min<long long>((long long)p.SP * p.SP * 8, PBAD), 0x00020000);
  const int pieces = (PROWS * p.pitch + 1023) >> 10;
  for (int q = wid; q < pieces; q += nw) {
    const int o = q * 1024 + lane * 16;
    const int pr = o / p.pitch, pc = (o - pr * p.pitch) >> 3;
    const int ir = row0 + pr, ic = col0 + pc;
    const bool v = pr < PROWS && ir >= 0 && ir < p.SP && ic >= 0 && ic < p.SP;
    const int off = v ? ((ir * p.SP + ic) << 3) : PBAD;
    __builtin_amdgcn_raw_ptr_buffer_load_lds(rx, (lds_ptr_t)(patch + q * 1024), 16, off, 0, 0, 0);
  }
  // ---- weights: 64 rows x 28 chunks, padded pitch
  for (int i = tid; i < 64 * KCH; i += blockDim.x) {
    const int n = i / KCH, c = i - n * KCH;
    st16(wl + n * WPITCH + c * 16, ld16(w + (size_t)n * ldw + c * 8));
  }
  __builtin_amdgcn_s_waitcnt(0);            // (vmcnt, lgkmcnt, expcnt all zero)
  __syncthreads();

  const int f = f0 + wid;
  if (wid >= p.fpg || f >= p.nfrag) return;
  const int fg = lane >> 4, fr = lane & 15;
  const int c = 14 * f - 1 + fr;             // this lane's stem column
  const bool col_ok = c >= 0 && c < p.So;
  const int pcl = (28 * wid + 2 * fr + 2 * fg) * 8;   // the pixel's tap pair kw = 2fg, 2fg+1 (bytes)
  int woff[4];
#pragma unroll
  for (int nb = 0; nb < 4; ++nb) woff[nb] = (16 * nb + fr) * WPITCH + fg * 16;
  const float NEG = -__builtin_huge_valf();

  // stem rows r and r + 1 (rows past the image or before it come out as -inf)
  f32x4 ra[4], rb[4], prev[4];
  auto rows2 = [&](int r, bool two) {
#pragma unroll
    for (int nb = 0; nb < 4; ++nb) ra[nb] = rb[nb] = f32x4{0.f, 0.f, 0.f, 0.f};
    const char* pa = patch + (2 * r - row0) * p.pitch + pcl;
    // (compiler-only fence: the W fragments are loop-invariant LDS reads, and hoisting all 28 of
    // them out of the row loop would pin 112 registers)
    asm volatile("" ::: "memory");
#pragma unroll
    for (int kh = 0; kh < 7; ++kh) {
      u32x4 wv[4];
#pragma unroll
      for (int nb = 0; nb < 4; ++nb) wv[nb] = ld16(wl + woff[nb] + kh * 64);
      const bf16x8 a0 = __builtin_bit_cast(bf16x8, ld16(pa + kh * p.pitch));
#pragma unroll
      for (int nb = 0; nb < 4; ++nb)
        ra[nb] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(__builtin_bit_cast(bf16x8, wv[nb]), a0, ra[nb], 0, 0, 0);
      if (two) {
        const bf16x8 a1 = __builtin_bit_cast(bf16x8, ld16(pa + (kh + 2) * p.pitch));
#pragma unroll
        for (int nb = 0; nb < 4; ++nb)
          rb[nb] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(__builtin_bit_cast(bf16x8, wv[nb]), a1, rb[nb], 0, 0, 0);
      }
    }
    const bool oka = col_ok && r >= 0 && r < p.So, okb = col_ok && r + 1 >= 0 && r + 1 < p.So;
#pragma unroll
    for (int nb = 0; nb < 4; ++nb)
#pragma unroll
      for (int e = 0; e < 4; ++e) {
        if (!oka) ra[nb][e] = NEG;
        if (!okb) rb[nb][e] = NEG;
      }
  };

  // bias of the lane's channels 16 nb + 4 fg + e
  f32x4 bv[4];
#pragma unroll
  for (int nb = 0; nb < 4; ++nb) bv[nb] = *reinterpret_cast<const f32x4*>(bias + 16 * nb + 4 * fg);

  rows2(2 * p0 - 1, false);                  // the band's top row 2 p0 - 1
#pragma unroll
  for (int nb = 0; nb < 4; ++nb) prev[nb] = ra[nb];
  const int j = fr >> 1, pw = 7 * f + j;     // pool column of the even lanes fr = 2j (j < 7)
  const bool store = !(fr & 1) && j < 7 && pw < p.Po;
  for (int i = 0; i < npr; ++i) {
    const int ph = p0 + i;
    rows2(2 * ph, true);
    f32x4 v[4];
#pragma unroll
    for (int nb = 0; nb < 4; ++nb) {
#pragma unroll
      for (int e = 0; e < 4; ++e) {
        float m = __builtin_fmaxf(__builtin_fmaxf(prev[nb][e], ra[nb][e]), rb[nb][e]);
        const float m1 = __shfl_down(m, 1, 16), m2 = __shfl_down(m, 2, 16);
        v[nb][e] = __builtin_fmaxf(__builtin_fmaxf(m, m1), m2);
      }
      prev[nb] = rb[nb];
    }
    if (store) {
      bf16* op = out + ((size_t)(b * p.Po + ph) * p.Po + pw) * ldo + 4 * fg;
#pragma unroll
      for (int nb = 0; nb < 4; ++nb) {
        float o[4];
#pragma unroll
        for (int e = 0; e < 4; ++e) o[e] = __builtin_fmaxf(v[nb][e] + bv[nb][e], 0.f);
        st8(op + 16 * nb, u32x2{pack_bf16x2(o[0], o[1]), pack_bf16x2(o[2], o[3])});
      }
    }
  }
}

bool geom(int S, SpGeom& p) {
  p.S = S;
  p.SP = S + 6;
  p.So = (S + 6 - 7) / 2 + 1;               // 7x7 / stride 2 over the bordered input (= S / 2 for even S)
  p.Po = (p.So + 2 - 3) / 2 + 1;
  p.nfrag = (p.Po + 6) / 7;
  p.groups = (p.nfrag + MAXW - 1) / MAXW;
  p.fpg = (p.nfrag + p.groups - 1) / p.groups;
  p.bands = (p.Po + PR - 1) / PR;
  p.pwid = 28 * p.fpg + 10;
  p.pitch = p.pwid * 8;
  return PROWS * p.pitch <= LDS_PATCH;
}

}  // namespace

bool spe_stempool_enabled() {
  static const int on = [] { const char* e = getenv("SPE_STEMPOOL"); return e ? atoi(e) : 1; }();
  return on != 0;
}

bool spe_stempool_fits(int S) {
  SpGeom p;
  return S > 0 && geom(S, p);
}

int spe_launch_stempool(const void* x, const void* w, int ldw, const float* bias, void* out, int ldo, int B, int S,
                        hipStream_t s) {
  if (B <= 0) return 0;
  SpGeom p;
  if (!geom(S, p) || ldw < 224 || ldw % 8 || ldo < 64 || ldo % 4) return 1;
  hipLaunchKernelGGL(stempool_kernel, dim3(B * p.bands * p.groups), dim3(64 * p.fpg), 0, s, (const bf16*)x,
                     (const bf16*)w, ldw, bias, (bf16*)out, ldo, p);
  return (int)hipGetLastError();
}
