// Fused transformer FFN block for gfx950 (bf16 storage, fp32 accumulate):
//
//     y = LayerNorm( x + W2 . relu(W1 . x + b1) + b2 )          (post-norm, eps 1e-5)
//
// i.e. linear1 -> ReLU -> linear2 -> residual -> norm2 of TransformerEncoderLayer.forward_post
// (REV/models/transformer.py:164-167) and norm3 of the decoder layer (:235-238).  The
// [rows x 2048] hidden activation never leaves registers: per 192-row block each wave owns 48
// rows (32 in the split-F form) and keeps its x rows (as MFMA B fragments) and its 256 output columns (as transposed
// accumulators out^T[n][m]) in registers while the block streams W1/W2 in chunks of 32 hidden
// units through a three-slot LDS ring filled by global_load_lds (two chunks in flight):
//     H^T[j][m] = W1[j][:] . x[m][:]                 16x16x32 MFMAs, K = 256
//     out^T[n][m] += W2[n][j] . relu(H^T + b1)[j][m]   16x16x32 MFMAs, K = 32; the H^T accumulator
//                                                    is re-packed in registers as the B operand
//                                                    (k order permuted; W2 reads follow it)
// Each wave owns 16*MB rows (48 by default): every wave streams the whole chunk of weights
// from LDS, so more rows per wave means more MFMA work per LDS byte and per barrier.
// The epilogue adds b2 and the residual, does the row LayerNorm with two lane shuffles
// (each row's 256 columns live in 4 lanes) and stores bf16 in place over x.
// Versus two GEMM launches + a LayerNorm launch this removes the 2 x rows x 2048 x 2 B round
// trip of the hidden activation through HBM and two kernel boundaries per layer.
#include "spe_common.h"
#include "spe_kernels.h"

#include <cstdlib>
#include <type_traits>

namespace {

constexpr int NT = 256;
constexpr int BM = 128;                 // rows per block of the split-F (few-row) form: 32 per wave
constexpr int HC = 32;                  // hidden units per chunk
constexpr int D = 256;
constexpr int W1_BYTES = HC * D * 2;    // 16 KiB: W1[j][d], 32 rows of 512 B
constexpr int W2_BYTES = D * HC * 2;    // 16 KiB: W2[n][j], 256 rows of 64 B
constexpr int STAGE = W1_BYTES + W2_BYTES;
constexpr int FMAX = 4096;              // largest dim_feedforward (b1 staged in LDS)
constexpr int LOADS = (W1_BYTES + W2_BYTES) / 1024 / 4;   // DMA wave-instructions per wave per chunk

// Hidden-unit order inside a chunk.  Phase 1 computes H^T in two 16-row MFMA blocks; LDS row
// R of the W1 stage holds hidden unit P(R) = 8*((R&15)>>2) + 4*(R>>4) + (R&3), so lane group g
// ends up owning the 8 CONSECUTIVE hidden units 8g..8g+7 of the chunk: its B operand for phase
// 2 packs in order, its bias is one 32-byte read and its W2 A operand is one 16-byte read.
SPE_DEV int w1_src_row(int R) { return 8 * ((R & 15) >> 2) + 4 * (R >> 4) + (R & 3); }
// W1 stage: 16-byte chunk c of LDS row R at slot c ^ (R & 15) (conflict-free ds_read_b128)
SPE_DEV int w1_off(int R, int c) { return R * 512 + ((c ^ (R & 15)) << 4); }
// W2 stage: 16-byte chunk c (hidden 8c..8c+7) of row n at slot c ^ key(n), key = -(n>>2) & 3:
// each ds_read_b128 lane group's 16 reads hit 16 distinct 16-byte bank groups
SPE_DEV int w2_key(int n) { return (4 - ((n >> 2) & 3)) & 3; }
SPE_DEV int w2_off(int n, int c) { return n * 64 + ((c ^ w2_key(n)) << 4); }

typedef __attribute__((address_space(3))) void* lds_ptr_t;
template <int N>
SPE_DEV void wait_vmcnt() { asm volatile("s_waitcnt vmcnt(%0)" ::"n"(N) : "memory"); }

// One chunk's weights, global -> LDS directly (global_load_lds, 16 B per lane, linear LDS
// image per wave-instruction; the swizzles above are applied on the source side).
SPE_DEV void issue_chunk(const FfnArgs& a, int ch, char* st, int wid, int lane) {
#pragma unroll
  for (int i = 0; i < 4; ++i) {                 // W1: 16 instructions x 2 rows of 512 B
    const int ins = wid * 4 + i, R = 2 * ins + (lane >> 5), c = (lane & 31) ^ (R & 15);
    const char* src = (const char*)a.w1 + ((size_t)(ch * HC + w1_src_row(R)) * a.ld1 + c * 8) * 2;
    __builtin_amdgcn_global_load_lds((const void*)src, (lds_ptr_t)(st + ins * 1024), 16, 0, 0);
  }
#pragma unroll
  for (int i = 0; i < 4; ++i) {                 // W2: 16 instructions x 16 rows of 64 B
    const int ins = wid * 4 + i, n = 16 * ins + (lane >> 2), c = (lane & 3) ^ w2_key(n);
    const char* src = (const char*)a.w2 + (a.w2_chunked ? ((size_t)ch * D * HC + n * HC + c * 8) * 2
                                                        : ((size_t)n * a.ld2 + ch * HC + c * 8) * 2);
    __builtin_amdgcn_global_load_lds((const void*)src, (lds_ptr_t)(st + W1_BYTES + ins * 1024), 16, 0, 0);
  }
}

// The same chunk DMA through buffer_load ... lds: the per-lane part of each source address is
// a 32-bit voffset fixed for the kernel's life and the chunk's offset a scalar soffset, so a
// chunk costs 8 issue slots and no address VALU (global_load_lds needs a 64-bit per-lane address
// per instruction and chunk).  Out-of-range reads (num_records) return zero.
typedef short short2_t __attribute__((ext_vector_type(2)));
struct ChunkDma {
  __amdgpu_buffer_rsrc_t r1, r2;
  int vo1[4], vo2[4];
  SPE_DEV void init(const FfnArgs& a, int wid, int lane) {
    r1 = __builtin_amdgcn_make_buffer_rsrc((void*)a.w1, (short)0, a.F * a.ld1 * 2, 0x00020000);
    r2 = __builtin_amdgcn_make_buffer_rsrc((void*)a.w2, (short)0, D * (a.w2_chunked ? a.F : a.ld2) * 2, 0x00020000);
#pragma unroll
    for (int i = 0; i < 4; ++i) {
      const int ins = wid * 4 + i;
      const int R = 2 * ins + (lane >> 5), c = (lane & 31) ^ (R & 15);
      vo1[i] = (w1_src_row(R) * a.ld1 + c * 8) * 2;
      const int n = 16 * ins + (lane >> 2), c2 = (lane & 3) ^ w2_key(n);
      vo2[i] = ((a.w2_chunked ? n * HC : n * a.ld2) + c2 * 8) * 2;
    }
  }
  // piece i of 8 (0-3: W1, 4-7: W2), for spreading a chunk's DMA between MFMAs
  SPE_DEV void piece(const FfnArgs& a, int ch, char* st, int wid, int i) const {
    if (i < 4)
      __builtin_amdgcn_raw_ptr_buffer_load_lds(r1, (lds_ptr_t)(st + (wid * 4 + i) * 1024), 16, vo1[i], ch * HC * a.ld1 * 2, 0, 0);
    else
      __builtin_amdgcn_raw_ptr_buffer_load_lds(r2, (lds_ptr_t)(st + W1_BYTES + (wid * 4 + i - 4) * 1024), 16, vo2[i - 4],
                                               so2(a, ch), 0, 0);
  }
  SPE_DEV void issue(const FfnArgs& a, int ch, char* st, int wid) const {
    const int so1 = ch * HC * a.ld1 * 2, s2 = so2(a, ch);
#pragma unroll
    for (int i = 0; i < 4; ++i)
      __builtin_amdgcn_raw_ptr_buffer_load_lds(r1, (lds_ptr_t)(st + (wid * 4 + i) * 1024), 16, vo1[i], so1, 0, 0);
#pragma unroll
    for (int i = 0; i < 4; ++i)
      __builtin_amdgcn_raw_ptr_buffer_load_lds(r2, (lds_ptr_t)(st + W1_BYTES + (wid * 4 + i) * 1024), 16, vo2[i], s2, 0, 0);
  }
  // chunk ch's W2 columns: 64 bytes of every row at a 4 KB row stride, or (w2_chunked) one
  // contiguous 16 KB block -- the strided form's 256 lines per chunk fall into few L2 sets
  SPE_DEV static int so2(const FfnArgs& a, int ch) { return a.w2_chunked ? ch * D * HC * 2 : ch * HC * 2; }
};
// ReLU of two packed bf16: negative values (sign bit set) are negative as int16
SPE_DEV uint32_t relu_bf16x2(uint32_t v) {
  return __builtin_bit_cast(uint32_t, __builtin_elementwise_max(__builtin_bit_cast(short2_t, v), short2_t{0, 0}));
}

// epilogue shared by the FFN kernels: + b2 + residual, LayerNorm over n, bf16 store (and the
// optional y + pos second output)
template <int MB>
SPE_DEV void ffn_epilogue(const FfnArgs& a, f32x4 (&acc)[16][MB], int m0, int g, int c16) {
  // Lane holds, for each of its MB rows m = m0 + 16mb + c16, columns n = 16nb + 4g + r (r = 0..3, nb = 0..15).
#pragma unroll
  for (int mb = 0; mb < MB; ++mb) {
    const int m = m0 + 16 * mb + c16;
    const bool live = m < a.M;
    const bf16* xr = (const bf16*)a.x + (size_t)(live ? m : 0) * a.ldx;
    float s = 0.f;
#pragma unroll
    for (int nb = 0; nb < 16; ++nb) {
      const int n = 16 * nb + 4 * g;
      const f32x4 b2 = *reinterpret_cast<const f32x4*>(a.b2 + n);
      const u32x2 rv = live ? ld8(xr + n) : u32x2{0, 0};
      const float r0 = __uint_as_float(rv.x << 16), r1 = __uint_as_float(rv.x & 0xffff0000u);
      const float r2 = __uint_as_float(rv.y << 16), r3 = __uint_as_float(rv.y & 0xffff0000u);
      acc[nb][mb][0] += b2[0] + r0;
      acc[nb][mb][1] += b2[1] + r1;
      acc[nb][mb][2] += b2[2] + r2;
      acc[nb][mb][3] += b2[3] + r3;
      s += acc[nb][mb][0] + acc[nb][mb][1] + acc[nb][mb][2] + acc[nb][mb][3];
    }
    s += __shfl_xor(s, 16, 64);
    s += __shfl_xor(s, 32, 64);
    const float mean = s * (1.f / D);
    float q = 0.f;
#pragma unroll
    for (int nb = 0; nb < 16; ++nb)
#pragma unroll
      for (int r = 0; r < 4; ++r) {
        const float dv = acc[nb][mb][r] - mean;
        q += dv * dv;
      }
    q += __shfl_xor(q, 16, 64);
    q += __shfl_xor(q, 32, 64);
    const float rs = rsqrtf(q * (1.f / D) + 1e-5f);
    if (!live) continue;
    bf16* yr = (bf16*)a.y + (size_t)m * a.ldy;
    // optional second output y + pos (the encoder's last layer: the cross-attention K input)
    const bf16* pr = a.ypos ? (const bf16*)a.pos + (size_t)(m % a.pos_period) * D : nullptr;
    bf16* ypr = a.ypos ? (bf16*)a.ypos + (size_t)m * a.ldy : nullptr;
#pragma unroll
    for (int nb = 0; nb < 16; ++nb) {
      const int n = 16 * nb + 4 * g;
      const f32x4 ga = *reinterpret_cast<const f32x4*>(a.gamma + n);
      const f32x4 be = *reinterpret_cast<const f32x4*>(a.beta + n);
      float o[4];
#pragma unroll
      for (int r = 0; r < 4; ++r) o[r] = (acc[nb][mb][r] - mean) * rs * ga[r] + be[r];
      st8(yr + n, u32x2{pack_bf16x2(o[0], o[1]), pack_bf16x2(o[2], o[3])});
      if (ypr) {
        const u32x2 pv = ld8(pr + n);
        st8(ypr + n, u32x2{pack_bf16x2(o[0] + __uint_as_float(pv.x << 16), o[1] + __uint_as_float(pv.x & 0xffff0000u)),
                           pack_bf16x2(o[2] + __uint_as_float(pv.y << 16), o[3] + __uint_as_float(pv.y & 0xffff0000u))});
      }
    }
  }
}

// MB = 16-row MFMA blocks per wave (rows per wave = 16 MB, per block = 64 MB): more rows per
// wave = more MFMA work per byte of weights read from LDS (every wave reads the whole chunk).
template <int MB, int NSTAGE = 3>
__global__ __launch_bounds__(NT, 1) void ffn_ln_kernel(FfnArgs a) {
  constexpr int RB = 64 * MB;           // rows per block
  // one LDS array (a second __shared__ object beside in-flight global_load_lds can make the
  // compiler drain vmcnt before LDS reads): [NSTAGE weight stages][b1]
  __shared__ __attribute__((aligned(1024))) char lds[NSTAGE * STAGE + FMAX * 4];
  float* sb1 = reinterpret_cast<float*>(lds + NSTAGE * STAGE);
  const int tid = threadIdx.x, lane = tid & 63, wid = __builtin_amdgcn_readfirstlane(tid >> 6);
  const int g = lane >> 4, c16 = lane & 15;
  // split-F mode (few rows, e.g. the decoder's B*Q): block = (row tile, hidden-unit range);
  // the partial out^T of each range goes to a.partial and ffn_reduce_ln_kernel finishes
  const int S = a.partial ? a.splits : 1;
  const int split = blockIdx.x % S;
  const int m0 = (blockIdx.x / S) * RB + wid * 16 * MB;
  const int cps = a.F / HC / S;
  const int cbeg = split * cps, nchunks = cbeg + cps;   // chunk range [cbeg, nchunks)
  for (int i = tid; i < a.F; i += NT) sb1[i] = a.b1[i];

  // x rows of this wave as B fragments: xf[mb][ks] = x[m0 + 16mb + c16][32ks + 8g .. +7]
  bf16x8 xf[MB][8];
#pragma unroll
  for (int mb = 0; mb < MB; ++mb) {
    const int m = m0 + 16 * mb + c16;
    const bf16* xr = (const bf16*)a.x + (size_t)(m < a.M ? m : 0) * a.ldx;
#pragma unroll
    for (int ks = 0; ks < 8; ++ks)
      xf[mb][ks] = __builtin_bit_cast(bf16x8, m < a.M ? ld16(xr + 32 * ks + 8 * g) : u32x4{0, 0, 0, 0});
  }
  f32x4 acc[16][MB];
#pragma unroll
  for (int nb = 0; nb < 16; ++nb)
#pragma unroll
    for (int mb = 0; mb < MB; ++mb) acc[nb][mb] = f32x4{0, 0, 0, 0};
  // x (and b1) must have landed before the weight DMA starts: vmcnt is in-order, and with a load
  // of x still pending at the loop entry the compiler's merged wait state would drain every
  // in-flight chunk at the first MFMA of each step.  (An asm use of every x register makes the
  // compiler itself retire those loads here; an inline-asm s_waitcnt is invisible to it.)
#pragma unroll
  for (int mb = 0; mb < MB; ++mb)
#pragma unroll
    for (int ks = 0; ks < 8; ++ks) asm volatile("" ::"v"(xf[mb][ks]));
  wait_vmcnt<0>();
#pragma unroll
  for (int i = 0; i < NSTAGE - 1; ++i)
    if (cbeg + i < nchunks) issue_chunk(a, cbeg + i, lds + i * STAGE, wid, lane);

  int slot = 0;
  for (int ch = cbeg; ch < nchunks; ++ch) {
    // retire chunk ch (this wave's loads; chunks ch+1 .. ch+NSTAGE-2 may stay in flight), then
    // the barrier makes every wave's part visible and guarantees the slot of chunk
    // ch+NSTAGE-1 -- read in step ch-1 -- is free
    if (NSTAGE >= 4 && ch + 2 < nchunks) wait_vmcnt<2 * LOADS>();
    else if (ch + 1 < nchunks) wait_vmcnt<LOADS>();
    else wait_vmcnt<0>();
    // raw barrier: __syncthreads' fence would also drain the chunk still in flight
    asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
    __builtin_amdgcn_s_barrier();
    const int slot2 = slot == 0 ? NSTAGE - 1 : slot - 1;    // (ch + NSTAGE - 1) % NSTAGE
    const char* st = lds + slot * STAGE;
    slot = slot == NSTAGE - 1 ? 0 : slot + 1;
    // all of this chunk's fragment reads up front (one wave per SIMD: nothing else hides LDS
    // latency); the W2 reads land while the phase-1 MFMAs run
    u32x4 wa[8][2], wb[16];
#pragma unroll
    for (int ks = 0; ks < 8; ++ks)
#pragma unroll
      for (int jb = 0; jb < 2; ++jb) wa[ks][jb] = ld16(st + w1_off(16 * jb + c16, 4 * ks + g));
#pragma unroll
    for (int nb = 0; nb < 16; ++nb) wb[nb] = ld16(st + W1_BYTES + w2_off(16 * nb + c16, g));
    // chunk ch+2's loads go out after this chunk's LDS reads: issued before them, the compiler
    // (which cannot tell the DMA's slot from the read's) would drain them first
    if (ch + NSTAGE - 1 < nchunks) issue_chunk(a, ch + NSTAGE - 1, lds + slot2 * STAGE, wid, lane);
    __builtin_amdgcn_sched_barrier(0);
    // ---- H^T chunk: [32 j][32 m] = W1[j] . x[m]   (LDS row 16jb + 4g + r = hidden 8g + 4jb + r)
    f32x4 h[2][MB];
#pragma unroll
    for (int jb = 0; jb < 2; ++jb)
#pragma unroll
      for (int mb = 0; mb < MB; ++mb) h[jb][mb] = f32x4{0, 0, 0, 0};
#pragma unroll
    for (int ks = 0; ks < 8; ++ks) {
#pragma unroll
      for (int jb = 0; jb < 2; ++jb) {
        const bf16x8 w = __builtin_bit_cast(bf16x8, wa[ks][jb]);
#pragma unroll
        for (int mb = 0; mb < MB; ++mb)
          h[jb][mb] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(w, xf[mb][ks], h[jb][mb], 0, 0, 0);
      }
    }
    // ---- bias + ReLU, pack as the K=32 B operand: element e <-> hidden 8g + e of the chunk
    const f32x4 b1a = *reinterpret_cast<const f32x4*>(sb1 + ch * HC + 8 * g);
    const f32x4 b1b = *reinterpret_cast<const f32x4*>(sb1 + ch * HC + 8 * g + 4);
    bf16x8 hb[MB];
#pragma unroll
    for (int mb = 0; mb < MB; ++mb) {
      float v[8];
#pragma unroll
      for (int r = 0; r < 4; ++r) {
        v[r] = fmaxf(h[0][mb][r] + b1a[r], 0.f);
        v[4 + r] = fmaxf(h[1][mb][r] + b1b[r], 0.f);
      }
      hb[mb] = __builtin_bit_cast(bf16x8, pack16<bf16>(v));
    }
    // ---- out^T[n][m] += W2[n][chunk 8g..8g+7] . H^T[8g..8g+7][m]
#pragma unroll
    for (int nb = 0; nb < 16; ++nb) {
      const bf16x8 w = __builtin_bit_cast(bf16x8, wb[nb]);
#pragma unroll
      for (int mb = 0; mb < MB; ++mb)
        acc[nb][mb] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(w, hb[mb], acc[nb][mb], 0, 0, 0);
    }
  }

  if (a.partial) {                              // split-F: raw partial sums, finished elsewhere
#pragma unroll
    for (int mb = 0; mb < MB; ++mb) {
      const int m = m0 + 16 * mb + c16;
      if (m >= a.M) continue;
      float* pr = a.partial + ((size_t)split * a.M + m) * D;
#pragma unroll
      for (int nb = 0; nb < 16; ++nb) st16(pr + 16 * nb + 4 * g, __builtin_bit_cast(u32x4, acc[nb][mb]));
    }
    return;
  }

  ffn_epilogue<MB>(a, acc, m0, g, c16);
}

// Cross-chunk software pipeline (encoder FFN, many rows): step c multiplies phase 2 of chunk c
// (out^T += W2(c) . relu(H(c))) interleaved with phase 1 of chunk c+1 (H(c+1) = W1(c+1) . x), two
// independent MFMA streams, so no MFMA waits on the phase-1 -> bias/ReLU -> phase-2 dependency
// that stalls the one wave per SIMD in ffn_ln_kernel.  Four-slot ring: at step c chunk c+1 is
// retired (chunk c+2 stays in flight) and chunk c+3 is issued into the slot chunk c-1 left.
// SCHED: the step's 32 fragment reads are issued in consumption order a few MFMAs
// ahead of their use and its 8 DMA pieces spread between the MFMAs, with the instruction order
// pinned by sched_barrier: otherwise the compiler hoists every read to the top of the step and
// the one wave per SIMD waits for all 32 KiB of them before its MFMAs can run.
// PRE = reads issued ahead of the first MFMA (then one per MFMA triple).
template <int MB, bool SCHED = false, int PRE = 6>
__global__ __launch_bounds__(NT, 1) void ffn_pipe_kernel(FfnArgs a) {
  constexpr int NST = 4;
  __shared__ __attribute__((aligned(1024))) char lds[NST * STAGE + FMAX * 4];
  float* sb1 = reinterpret_cast<float*>(lds + NST * STAGE);
  // (wid wave-uniform in a scalar register: the DMA pieces' LDS addresses (m0) then need no
  // v_readfirstlane per piece)
  const int tid = threadIdx.x, lane = tid & 63, wid = __builtin_amdgcn_readfirstlane(tid >> 6);
  const int g = lane >> 4, c16 = lane & 15;
  const int m0 = a.row0 + blockIdx.x * 64 * MB + wid * 16 * MB;
  const int nch = a.F / HC;
  for (int i = tid; i < a.F; i += NT) sb1[i] = a.b1[i];
  bf16x8 xf[MB][8];
#pragma unroll
  for (int mb = 0; mb < MB; ++mb) {
    const int m = m0 + 16 * mb + c16;
    const bf16* xr = (const bf16*)a.x + (size_t)(m < a.M ? m : 0) * a.ldx;
#pragma unroll
    for (int ks = 0; ks < 8; ++ks)
      xf[mb][ks] = __builtin_bit_cast(bf16x8, m < a.M ? ld16(xr + 32 * ks + 8 * g) : u32x4{0, 0, 0, 0});
  }
  f32x4 acc[16][MB];
#pragma unroll
  for (int nb = 0; nb < 16; ++nb)
#pragma unroll
    for (int mb = 0; mb < MB; ++mb) acc[nb][mb] = f32x4{0, 0, 0, 0};
#pragma unroll
  for (int mb = 0; mb < MB; ++mb)
#pragma unroll
    for (int ks = 0; ks < 8; ++ks) asm volatile("" ::"v"(xf[mb][ks]));
  wait_vmcnt<0>();                               // (see ffn_ln_kernel: x retired before the DMA)
  ChunkDma dma;
  dma.init(a, wid, lane);
#pragma unroll
  for (int i = 0; i < NST - 1; ++i)
    if (i < nch) dma.issue(a, i, lds + i * STAGE, wid);

  u32x4 wa[8][2], wb[16];
  f32x4 h[2][MB];
  bf16x8 hb[MB];
  auto read_w1 = [&](const char* st) {
#pragma unroll
    for (int ks = 0; ks < 8; ++ks)
#pragma unroll
      for (int jb = 0; jb < 2; ++jb) wa[ks][jb] = ld16(st + w1_off(16 * jb + c16, 4 * ks + g));
  };
  auto read_w2 = [&](const char* st) {
#pragma unroll
    for (int nb = 0; nb < 16; ++nb) wb[nb] = ld16(st + W1_BYTES + w2_off(16 * nb + c16, g));
  };
  auto p1 = [&](int i) {                         // phase-1 MFMA i of 16 MB: (ks, jb, mb)
    const int ks = i / (2 * MB), jb = (i / MB) % 2, mb = i % MB;
    h[jb][mb] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(__builtin_bit_cast(bf16x8, wa[ks][jb]), xf[mb][ks],
                                                        h[jb][mb], 0, 0, 0);
  };
  auto p2 = [&](int i) {                         // phase-2 MFMA i of 16 MB: (nb, mb)
    const int nb = i / MB, mb = i % MB;
    acc[nb][mb] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(__builtin_bit_cast(bf16x8, wb[nb]), hb[mb],
                                                          acc[nb][mb], 0, 0, 0);
  };
  // H starts from b1 (the MFMAs accumulate onto the bias): h[jb][mb][r] <-> hidden 8g + 4jb + r
  auto init_h = [&](int ch) {
    const f32x4 b1a = *reinterpret_cast<const f32x4*>(sb1 + ch * HC + 8 * g);
    const f32x4 b1b = *reinterpret_cast<const f32x4*>(sb1 + ch * HC + 8 * g + 4);
#pragma unroll
    for (int mb = 0; mb < MB; ++mb) {
      h[0][mb] = b1a;
      h[1][mb] = b1b;
    }
  };
  // ReLU after the bf16 rounding (same result: rounding keeps the sign), on packed pairs
  auto pack_h = [&](bf16x8 (&out)[MB]) {
#pragma unroll
    for (int mb = 0; mb < MB; ++mb) {
      const uint32_t w0 = relu_bf16x2(pack_bf16x2(h[0][mb][0], h[0][mb][1]));
      const uint32_t w1 = relu_bf16x2(pack_bf16x2(h[0][mb][2], h[0][mb][3]));
      const uint32_t w2 = relu_bf16x2(pack_bf16x2(h[1][mb][0], h[1][mb][1]));
      const uint32_t w3 = relu_bf16x2(pack_bf16x2(h[1][mb][2], h[1][mb][3]));
      out[mb] = __builtin_bit_cast(bf16x8, u32x4{w0, w1, w2, w3});
    }
  };
  auto sync = [&]() {                            // raw barrier: keep the in-flight chunks
    asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
    __builtin_amdgcn_s_barrier();
  };

  // prologue: chunk 0 retired, its phase 1 alone
  if (nch > 2) wait_vmcnt<2 * LOADS>();
  else if (nch > 1) wait_vmcnt<LOADS>();
  else wait_vmcnt<0>();
  sync();
  read_w1(lds);
  init_h(0);
#pragma unroll
  for (int i = 0; i < 16 * MB; ++i) p1(i);
  pack_h(hb);

  // SCHED: the chunk loop unrolled by the ring's four slots (the slot a compile-time constant, so
  // every fragment read is a lane base + an immediate offset: no per-read address VALU)
  auto sched_step = [&](int c, auto SC) {
    constexpr int S = decltype(SC)::value;
    if (c + 2 < nch) wait_vmcnt<LOADS>();        // chunk c+1 landed, c+2 may stay in flight
    else wait_vmcnt<0>();
    sync();
    const char* st = lds + S * STAGE;
    const char* st1 = lds + ((S + 1) % NST) * STAGE;
    // read r in consumption order: r < 24 -> block k = r / 3: W1(c+1) ks = k jb 0, W2(c) nb = k,
    // W1(c+1) ks = k jb 1 (block k feeds interleaved steps MB*k .. MB*k + MB-1);
    // r >= 24 -> W2(c) nb = r - 16 (the tail)
    auto rd = [&](int r) {
      if (r < 24) {
        const int k = r / 3, q = r % 3;
        if (q == 1) wb[k] = ld16(st + W1_BYTES + w2_off(16 * k + c16, g));
        else wa[k][q >> 1] = ld16(st1 + w1_off(16 * (q >> 1) + c16, 4 * k + g));
      } else {
        wb[r - 16] = ld16(st + W1_BYTES + w2_off(16 * (r - 16) + c16, g));
      }
    };
    // chunk c+3's pieces are issued unconditionally (a branch would split the MFMA block and
    // the accumulators get copied across it): past the last chunk the buffer resource's range
    // check makes them zero-fill the free slot (c+3) % 4, which nothing reads any more
    char* dst = lds + ((S + 3) % NST) * STAGE;
    init_h(c + 1);
#pragma unroll
    for (int r = 0; r < PRE; ++r) rd(r);
    __builtin_amdgcn_sched_barrier(0);
    // interleaved steps t: p1(2t), p1(2t+1), p2(t); 3 reads per MB steps, one DMA piece per MB
    int issued = PRE;
#pragma unroll
    for (int t = 0; t < 8 * MB; ++t) {
      const int upto = PRE + (3 * (t + 1) + MB - 1) / MB < 32 ? PRE + (3 * (t + 1) + MB - 1) / MB : 32;
      for (; issued < upto; ++issued) rd(issued);
      if (t % MB == 1 % MB) dma.piece(a, c + 3, dst, wid, t / MB);
      p1(2 * t);
      p1(2 * t + 1);
      p2(t);
      __builtin_amdgcn_sched_barrier(0);
    }
    bf16x8 hb_next[MB];
    // tail: p2(8MB..16MB) in groups of MB (one W2 block each), the remaining reads and
    // H(c+1)'s pack between them
#pragma unroll
    for (int t = 8 * MB; t < 16 * MB; t += MB) {
      if (issued < 32) rd(issued++);
#pragma unroll
      for (int u = 0; u < MB; ++u) p2(t + u);
      if (t == 9 * MB) pack_h(hb_next);
      __builtin_amdgcn_sched_barrier(0);
    }
#pragma unroll
    for (int mb = 0; mb < MB; ++mb) hb[mb] = hb_next[mb];
  };
  if constexpr (SCHED) {
    static_assert(NST == 4, "unrolled by the ring's slots");
    for (int c = 0; c + 1 < nch; c += NST) {
      sched_step(c, std::integral_constant<int, 0>{});
      if (c + 2 < nch) sched_step(c + 1, std::integral_constant<int, 1>{});
      if (c + 3 < nch) sched_step(c + 2, std::integral_constant<int, 2>{});
      if (c + 4 < nch) sched_step(c + 3, std::integral_constant<int, 3>{});
    }
  } else
  for (int c = 0; c + 1 < nch; ++c) {
    if (c + 2 < nch) wait_vmcnt<LOADS>();        // chunk c+1 landed, c+2 may stay in flight
    else wait_vmcnt<0>();
    sync();
    const char* st = lds + (c % NST) * STAGE;
    const char* st1 = lds + ((c + 1) % NST) * STAGE;
    read_w2(st);
    read_w1(st1);
    if (c + 3 < nch) dma.issue(a, c + 3, lds + ((c + 3) % NST) * STAGE, wid);
    __builtin_amdgcn_sched_barrier(0);
    init_h(c + 1);
    // two phase-1 MFMAs per phase-2 MFMA until H(c+1) is complete, then the rest of phase 2
    // beside its bias / ReLU / pack
#pragma unroll
    for (int i = 0; i < 8 * MB; ++i) {
      p1(2 * i);
      p1(2 * i + 1);
      p2(i);
    }
    bf16x8 hb_next[MB];
    pack_h(hb_next);
#pragma unroll
    for (int i = 8 * MB; i < 16 * MB; ++i) p2(i);
#pragma unroll
    for (int mb = 0; mb < MB; ++mb) hb[mb] = hb_next[mb];
  }
  // last chunk: phase 2 alone
  if constexpr (SCHED) wait_vmcnt<0>();          // the zero-fill pieces past the end
  sync();
  read_w2(lds + ((nch - 1) % NST) * STAGE);
#pragma unroll
  for (int i = 0; i < 16 * MB; ++i) p2(i);

  ffn_epilogue<MB>(a, acc, m0, g, c16);
}

// split-F finish: y = LN(x + sum_s partial[s] + b2) (+ pos copy), one wave per row
__global__ __launch_bounds__(256) void ffn_reduce_ln_kernel(FfnArgs a) {
  const int lane = threadIdx.x & 63, m = blockIdx.x * 4 + (threadIdx.x >> 6);
  if (m >= a.M) return;
  const int n = 4 * lane;
  f32x4 v = *reinterpret_cast<const f32x4*>(a.b2 + n);
  for (int s = 0; s < a.splits; ++s) v += *reinterpret_cast<const f32x4*>(a.partial + ((size_t)s * a.M + m) * D + n);
  const u32x2 rv = ld8((const bf16*)a.x + (size_t)m * a.ldx + n);
  v[0] += __uint_as_float(rv.x << 16); v[1] += __uint_as_float(rv.x & 0xffff0000u);
  v[2] += __uint_as_float(rv.y << 16); v[3] += __uint_as_float(rv.y & 0xffff0000u);
  const float mean = wave_sum(v[0] + v[1] + v[2] + v[3]) * (1.f / D);
  float q = 0.f;
#pragma unroll
  for (int r = 0; r < 4; ++r) q += (v[r] - mean) * (v[r] - mean);
  const float rs = rsqrtf(wave_sum(q) * (1.f / D) + 1e-5f);
  const f32x4 ga = *reinterpret_cast<const f32x4*>(a.gamma + n), be = *reinterpret_cast<const f32x4*>(a.beta + n);
  float o[4];
#pragma unroll
  for (int r = 0; r < 4; ++r) o[r] = (v[r] - mean) * rs * ga[r] + be[r];
  st8((bf16*)a.y + (size_t)m * a.ldy + n, u32x2{pack_bf16x2(o[0], o[1]), pack_bf16x2(o[2], o[3])});
  if (a.ypos) {
    const u32x2 pv = ld8((const bf16*)a.pos + (size_t)(m % a.pos_period) * D + n);
    st8((bf16*)a.ypos + (size_t)m * a.ldy + n,
        u32x2{pack_bf16x2(o[0] + __uint_as_float(pv.x << 16), o[1] + __uint_as_float(pv.x & 0xffff0000u)),
              pack_bf16x2(o[2] + __uint_as_float(pv.y << 16), o[3] + __uint_as_float(pv.y & 0xffff0000u))});
  }
}

}  // namespace

// Rows below this many full row tiles per CU-wave run split-F (two launches, fp32 partials).
constexpr int SPLIT_ROWS = 128 * 64;

int spe_ffn_splits(int M, int F) {
  if (M >= SPLIT_ROWS) return 1;
  // up to ~64 workgroups: more splits spread the weights thinner but the fp32 partials the
  // reduce kernel reads grow with them (kbench ffndec, M = 704: 8 splits 23 us, 16: 25, 32: 34)
  int s = 1;
  while (s < 32 && (F / HC) % (2 * s) == 0 && ((M + BM - 1) / BM) * 2 * s <= 64) s *= 2;
  return s;
}

namespace {
__global__ __launch_bounds__(256) void ffn_w2_chunk_pack_kernel(const bf16* w, int ld, int F, bf16* dst) {
  const int i = blockIdx.x * 256 + threadIdx.x;   // one 16-byte piece: (chunk, row, 8 columns)
  if (i >= D * F / 8) return;
  const int q = i & 3, n = (i >> 2) & (D - 1), ch = i >> 10;
  st16(dst + (size_t)i * 8, ld16(w + (size_t)n * ld + ch * HC + 8 * q));
}
}  // namespace

int spe_launch_ffn_w2_chunk_pack(const void* w2, int ld2, int F, void* dst, hipStream_t s) {
  if (!w2 || !dst || F < HC || F % HC || ld2 < F || ld2 % 8) return -5;
  hipLaunchKernelGGL(ffn_w2_chunk_pack_kernel, dim3((D * F / 8 + 255) / 256), dim3(256), 0, s, (const bf16*)w2, ld2, F,
                     (bf16*)dst);
  return (int)hipGetLastError();
}

int spe_launch_ffn_reduce_ln(const FfnArgs& a, hipStream_t s) {
  if (a.M <= 0) return 0;
  if (a.D != D || !a.partial || a.splits < 1 || a.ldx % 8 || a.ldy % 8 || (a.ypos && (!a.pos || a.pos_period <= 0)))
    return -5;
  hipLaunchKernelGGL(ffn_reduce_ln_kernel, dim3((a.M + 3) / 4), dim3(256), 0, s, a);
  return (int)hipGetLastError();
}

int spe_launch_ffn_ln(const FfnArgs& a0, hipStream_t s) {
  FfnArgs a = a0;
  a.row0 = 0;
  if (a.M <= 0) return 0;
  if (a.ypos && (!a.pos || a.pos_period <= 0)) return -5;
  if (a.D != D || a.F % HC || a.F > FMAX || (a.ldx % 8) || (a.ldy % 8) || (a.ld1 % 8) || (a.ld2 % 8)) return -5;
  if (!a.partial) a.splits = 1;
  if (a.partial && (a.splits < 1 || (a.F / HC) % a.splits)) return -5;
  if (a.partial && a.splits > 1) {
    const int tiles = (a.M + BM - 1) / BM;
    hipLaunchKernelGGL(ffn_ln_kernel<2>, dim3(tiles * a.splits), dim3(NT), 0, s, a);
    hipLaunchKernelGGL(ffn_reduce_ln_kernel, dim3((a.M + 3) / 4), dim3(256), 0, s, a);
  } else {
    a.partial = nullptr;
    // 48 rows per wave (MB = 3, 493 VGPR+AGPR, no spills) measured 9 % faster than 32 (kbench,
    // B = 64 encoder FFN: 0.48 vs 0.53 ms); 64 rows spill.  SPE_FFN_MB overrides for A/B runs.
    static const int mb = [] { const char* e = getenv("SPE_FFN_MB"); return e ? atoi(e) : 3; }();
    static const int nst = [] { const char* e = getenv("SPE_FFN_NST"); return e ? atoi(e) : 4; }();
    static const int pipe = [] { const char* e = getenv("SPE_FFN_PIPE"); return e ? atoi(e) : 1; }();
    // SPE_FFN_SCHED: 0 = compiler-scheduled pipe loop, 3 / 6 / 9 = pinned schedule with that
    // many reads ahead (default 6)
    static const int sched = [] { const char* e = getenv("SPE_FFN_SCHED"); return e ? atoi(e) : 6; }();
    auto main_kernel = [&](int grid) {
      if (sched == 3) hipLaunchKernelGGL((ffn_pipe_kernel<3, true, 3>), dim3(grid), dim3(NT), 0, s, a);
      else if (sched == 9) hipLaunchKernelGGL((ffn_pipe_kernel<3, true, 9>), dim3(grid), dim3(NT), 0, s, a);
      else if (sched) hipLaunchKernelGGL((ffn_pipe_kernel<3, true, 6>), dim3(grid), dim3(NT), 0, s, a);
      else hipLaunchKernelGGL(ffn_pipe_kernel<3>, dim3(grid), dim3(NT), 0, s, a);
    };
    if (pipe && mb == 3 && a.F / HC >= 2) {
      // One workgroup per CU (144 KiB of LDS), so the grid runs in rounds of #CU tiles.  When the
      // last round would be partly idle and its rows fit one round of 128-row tiles, the whole
      // rounds take 192-row tiles and the rest goes to a second launch of 128-row tiles: the
      // last round then costs ~0.85 of a 192-row round (B = 64 encoder FFN: 0.445 -> 0.427 ms
      // unpinned).  SPE_FFN_TAIL=0 disables it for A/B runs.
      static const int tail = [] { const char* e = getenv("SPE_FFN_TAIL"); return e ? atoi(e) : 1; }();
      const int tiles = (a.M + 191) / 192, ncu = spe_cu_count();
      const int full = ncu > 0 ? tiles / ncu * ncu : 0, rest = a.M - full * 192;
      if (tail && full > 0 && rest > 0 && (rest + 127) / 128 <= ncu) {
        main_kernel(full);
        a.row0 = full * 192;
        if (sched) hipLaunchKernelGGL((ffn_pipe_kernel<2, true, 6>), dim3((rest + 127) / 128), dim3(NT), 0, s, a);
        else hipLaunchKernelGGL(ffn_pipe_kernel<2>, dim3((rest + 127) / 128), dim3(NT), 0, s, a);
      } else {
        main_kernel(tiles);
      }
    } else if (pipe && mb == 2 && a.F / HC >= 2) hipLaunchKernelGGL(ffn_pipe_kernel<2>, dim3((a.M + 127) / 128), dim3(NT), 0, s, a);
    else if (mb == 3 && nst == 4) hipLaunchKernelGGL((ffn_ln_kernel<3, 4>), dim3((a.M + 191) / 192), dim3(NT), 0, s, a);
    else if (mb == 3) hipLaunchKernelGGL(ffn_ln_kernel<3>, dim3((a.M + 191) / 192), dim3(NT), 0, s, a);
    else if (mb == 4) hipLaunchKernelGGL(ffn_ln_kernel<4>, dim3((a.M + 255) / 256), dim3(NT), 0, s, a);
    else hipLaunchKernelGGL(ffn_ln_kernel<2>, dim3((a.M + 127) / 128), dim3(NT), 0, s, a);
  }
  return (int)hipGetLastError();
}
