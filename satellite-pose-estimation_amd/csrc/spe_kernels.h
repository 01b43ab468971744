// Internal launcher interface between the C++ runtime (model.cpp, pnp host code) and the HIP
// kernels.  Not part of the public C ABI (include/spe.h).
#pragma once
#include <hip/hip_runtime.h>
#include <stdint.h>

enum { SPE_DTYPE_BF16 = 0, SPE_DTYPE_F32 = 1, SPE_DTYPE_F16 = 2,    // F16: attention operands only
       SPE_DTYPE_BF16_F16V = 3,     // attention only: bf16 q/k, fp16 V^T and P (bf16 models' encoder)
       SPE_DTYPE_F32X3 = 4,         // fp32 storage, split-bf16 (hi.hi + hi.lo + lo.hi) MFMA compute
       SPE_DTYPE_F32X6 = 5,         // fp32 storage, three-way split-bf16 (6 products, ~fp32) MFMA compute (GEMMs)
       SPE_DTYPE_F32H3 = 6 };       // fp32 storage, scaled two-way split-fp16 (3 products, ~fp32) MFMA compute (GEMMs)
enum { GEMM_LINEAR = 0, GEMM_LINEAR_ADD = 1, GEMM_CONV = 2 };
// GEMM epilogue activations: ReLU (ResNet, DETR FFN), SiLU (UNC hybrid encoder ConvNormLayer,
// hybrid_encoder.py:17-37), exact-erf GELU (UNC AIFI FFN, torch nn.GELU default)
enum { ACT_NONE = 0, ACT_RELU = 1, ACT_SILU = 2, ACT_GELU = 3 };

struct GemmArgs {
  const void* A; int lda;          // LINEAR*: A[m*lda + k]; CONV: NHWC input [B][H][W][Cin]
  const void* P; int ldp; int prow;// LINEAR_ADD: A += P[(m % prow)*ldp + k]
  int H, W, Cin, KH, KW, stride, pad, Ho, Wo;   // CONV geometry
  const void* B; int ldb;          // weights [N][ldb], ldb % 64 == 0
  int M, N, K;
  const float* bias;               // [N] or null
  const void* R; int ldr;          // residual [m*ldr + n] or null
  int act;                         // ACT_*: y = act(acc + bias + R), or act(acc + bias) + R
  int res_post;                    //   with res_post (CSPRepLayer's silu(rep(x1)) + x2)
  void* C; int ldc;                // output [m*ldc + n]
  int out_f32;                     // store fp32 instead of T
  int out_f16;                     // bf16 models: store fp16 instead of bf16 (fp16 attention operands)
  int vt_T, vt_B;                  // >0: head-transposed store (see gemm.hip)
  int vt_swz;                      // head-transposed 16-bit store with the attention's key order: within
                                   // each 16-token group the middle quads swap (vt_pos; vt_T % 16 == 0)
  int r_period;                    // >0: residual row = m % r_period (row-periodic add, e.g. pos . W^T)
  const float* ln_g; const float* ln_b;   // optional fused post-norm LayerNorm over N == 256 (bf16, large M)
  const void* B6; int b6_rows;     // fp32x6: the weights pre-split into bf16 planes [3][b6_rows][ldb] (h, m, l), or null
  void* S; int s_col0;             // fp32 models: columns n >= s_col0 stored instead as bf16 hi / lo planes for the
                                   // fp32x3 attention: rows -> hi [M][N - s_col0] then lo; head-transposed
                                   // (vt_T) -> hi in C's layout [vt_B][N][vt_T] then lo (s_col0 = 0)
  // fp32h3 (gemm.hip gemm_h3d): the weights as fp16 planes [2][h3_rows][ldb] (hi, lo of W[n] * 2^e_n)
  // with h3_sinv[n] = 2^-e_n; amax_a: device max |A| (the A operand's scale 2^13 / amax rounded to
  // a power of two; null = 1).  amax_c (fp32 GEMMs): max |stored output| * (amax_c_mul or 1) is
  // atomically maxed into *amax_c (float bits as uint, >= 0) -- the next GEMM's amax_a
  const void* H3; int h3_rows; const float* h3_sinv;
  const float* amax_a;
  float* amax_c; float amax_c_mul;
  // head-transposed S planes as fp16 instead of bf16 (the fp32h3 encoder attention's value operand):
  // hi / lo of x * vplane_scale(amax_a, s_l1, s_bmax), s_l1 = max_n sum_k |W[n][k]|, s_bmax = max |bias|
  int s_f16; float s_l1, s_bmax;
};
bool spe_gemm_ln_fusable(const GemmArgs& g);   // the large-tile kernel can fuse ln_g/ln_b for g
int spe_launch_gemm(const GemmArgs& g, int dtype, int mode, hipStream_t s);
// the fp32h3 kernels only: 1 (nothing launched) for a shape they do not serve, where spe_launch_gemm
// would fall through to the x6 path
int spe_launch_gemm_h3(const GemmArgs& g, int mode, hipStream_t s);

// Implicit-GEMM conv K order.  Multi-tap convs with Cin % 64 == 0 use channel-block-major order
// k = ((ci / 64) * KH*KW + tap) * 64 + ci % 64, so one 64-channel slice of the input window is
// reused by all taps in consecutive K-steps (L2-resident) instead of the whole Cin-deep window
// being streamed once per tap; other convs use k = tap * Cin + ci.  Weights are packed to match
// (registry.cpp make_conv).
__host__ __device__ inline bool conv_channel_blocked(int Cin, int taps) { return (Cin & 63) == 0 && taps > 1; }
__device__ __forceinline__ void conv_k_decode(int k, int Cin, int KW, int taps, int& kh, int& kw, int& ci) {
  int tap;
  if (conv_channel_blocked(Cin, taps)) {
    const int cb = k / (64 * taps), rem = k - cb * 64 * taps;
    tap = rem >> 6;
    ci = cb * 64 + (rem & 63);
  } else {
    tap = k / Cin;
    ci = k - tap * Cin;
  }
  kh = tap / KW;
  kw = tap - kh * KW;
}
// Bottleneck tail + next conv1 (btail.hip): y = relu(A . W3^T + b3 (+ R)), z = relu(y . W1p^T + b1)
// with W1p's columns in spe_btail_perm order.  bf16; N1 = n1 = 256 (layer 1), or the split-N
// form for 512 / 1024 (layers 2 / 3, residual row stride ldr = n1).
struct BtailArgs {
  const void* A; int lda; int k1;        // conv3 input [M][k1] (row stride lda)
  const void* R; int ldr;                // residual [M][n1] or null
  const void* w3; int ld3; const float* b3;   // [256][ld3]
  void* y; int ldy; int n1;              // block output [M][256]
  const void* w1; int ld1; const float* b1;   // next conv1, permuted columns [n2][ld1]
  void* z; int ldz; int n2;              // next conv1 output [M][n2]
  int M;
};
int spe_launch_btail(const BtailArgs& a, hipStream_t s);   // 1 = not applicable
int spe_btail_perm(int k);
bool spe_btail_enabled();
int spe_launch_gemm2(const GemmArgs& g, int mode, hipStream_t s);   // 1 = not applicable
int spe_launch_sgemm(const GemmArgs& g, int mode, hipStream_t s);   // 1 = not applicable
int spe_launch_lnproj(const GemmArgs& g, hipStream_t s);             // 1 = not applicable (lnproj.hip)
bool spe_lnproj_applies(const GemmArgs& g);
// bf16 GEMM + residual + LayerNorm in one launch: lnproj.hip at any row count, else the large-tile kernel
inline bool spe_ln_fusable(const GemmArgs& g) { return spe_lnproj_applies(g) || spe_gemm_ln_fusable(g); }
int spe_launch_pconv(const GemmArgs& g, hipStream_t s);             // 1 = not applicable (pconv.hip)
int spe_cu_count();               // CUs of the current device (cached; 256 on MI355X)
// kernel family of this thread's last spe_launch_gemm: 0 gemm.hip, 1 gemm2.hip, 2 gemm_stream.hip,
// 3 pconv.hip
extern thread_local int spe_gemm_last_path;

// Stored position of token t in a vt_swz V^T row: bits 2 and 3 swap (quads 0, 2, 1, 3 of every
// 16 tokens), the key order the attention's P^T operand has straight out of its S^T accumulator.
__host__ __device__ inline int vt_pos(int t) { return (t & ~12) | ((t & 4) << 1) | ((t & 8) >> 1); }

struct AttnArgs {
  const void* q; int ldq;          // query row b*Tq+i, head h at columns [h*32, h*32+32)
  const void* k; int ldk;          // key row b*Tk+j
  const void* vt;                  // V^T [B][H][32][Tk]
  int vt_swz;                      // V^T rows in vt_pos order (16-bit operands, Tk % 16 == 0): the
                                   // encoder kernel then stages K / V^T by LDS DMA
  void* o; int ldo;                // output row b*Tq+i
  int B, H, Tq, Tk;
  float scale;                     // softmax scale (1/sqrt(head_dim))
  int presplit;                    // fp32x3: k and vt are bf16 hi planes (k [B*Tk][ldk], vt [B][H][32][Tk]),
                                   // each followed by its lo plane (GemmArgs::S); Tk % 8 == 0.  With vt_swz
                                   // (V^T in vt_pos order, Tk % 16 == 0) the LDS-DMA split kernel (attn_split.hip)
  int v_f16;                       // presplit + vt_swz: the V^T planes are fp16 hi / lo of V * vplane_scale(
  const float* v_amax; float v_l1, v_bmax;   //   v_amax, v_l1, v_bmax) (GemmArgs::s_f16), P split to fp16
};
int spe_launch_attention_split(const AttnArgs& a, hipStream_t s);
int spe_launch_attention(const AttnArgs& a, int dtype, hipStream_t s);

// Decoder cross-attention against the encoder memory (bf16 path, xattn.hip): per image b and
// attention row r = q * 8 + h, u[b][q][h] = softmax(q'[b][q][h] . K^T) . V with K = memory +
// pos [T][256], V = memory [T][256], q' pre-scaled into the exp2 domain.
struct XattnArgs {
  const void* q; int ldq;          // q' rows b*Q + q, head h at columns [h*256, h*256 + 256)
  const void* k; int ldk;          // memory + pos, rows b*T + t
  const void* v; int ldv;          // memory, rows b*T + t
  void* u; int ldu;                // output rows b*Q + q, head h at columns [h*256, h*256 + 256)
  const void* wv; const float* bv; // optional: o_h = Wv_h u_h + bv_h written instead of u
  void* o; int ldo;                //   o rows b*Q + q, head h at columns [h*32, h*32 + 32)
  int B, Q, T, splits, tiles_per_split;
  float *pm, *pl, *pu;             // key-split partials [B][splits][8Q] (pu: x 256), required
  bool partials_only;              // stop at the partials (decproj's merge form consumes them)
  // fp32h3 (xattn_h3.hip): q' fp32; k / v the fp16 planes [B*T][512] (hi | lo) written by
  // spe_launch_xattn_h3_split from a memory bounded by *mem_amax; wv / bv / o fp32; max |o| raised into
  // *o_amax (the out-projection GEMM's scale input)
  const float* mem_amax; float* o_amax;
};
int spe_xattn_splits(int B, int Q, int T);
int spe_xattn_launch_splits(int T, int splits);   // the split count a launch with `splits` runs (partials' layout)
int spe_launch_xattn(const XattnArgs& a, hipStream_t s);
// fp32h3: kp = fp16 hi | lo of (mem + pos) * 2^sk, vp = of mem * 2^sv (powers of two from *mem_amax,
// vplane_scale), rows b*T + t of 512 halves; mem [B*T][256] fp32, pos [T][256] fp32
int spe_launch_xattn_h3_split(const float* mem, const float* pos, const float* mem_amax, void* kp, void* vp, int B,
                              int T, hipStream_t s);
int spe_launch_xattn_h3(const XattnArgs& a, hipStream_t s);

// Decoder self-attention block (bf16 only, decsa.hip), one workgroup per image, in place over tgt:
// tgt = LN(tgt + SelfAttn(q = k = tgt + qpos, v = tgt) . Wo^T + bo), 8 heads of 32, d = 256.
// The decoder kernels' weights are fragment-packed (spe_launch_wfrag_pack): [N/16][8][64][8] bf16,
// the 16-byte MFMA A fragment of lane l for column tile t and K-step ks at ((t*8 + ks)*64 + l)*8.
struct DecSaArgs {
  void* tgt; int ldt;              // [B*Q][ldt] bf16
  int B, Q;                        // Q <= 64
  const void* wqk; const float* bqk;   // in_proj rows 0..511 (packed), bias fp32
  const void* wv; const float* bv;     // in_proj rows 512..767 (packed)
  const void* qpos;                // [Q][512] bf16: query_pos . Wqk^T
  const void* wo; const float* bo;     // out_proj (packed)
  const float* g; const float* b;  // norm1
  float scale;                     // 1/sqrt(head_dim)
};
int spe_launch_decsa(const DecSaArgs& a, hipStream_t s);   // 1 = not applicable
// tgt = LN(tgt + x . Wo^T + bo), one workgroup per image (decsa.hip; bf16, d = 256, Q <= 64)
struct DecProjArgs {
  void* tgt; int ldt;              // [B*Q][ldt] bf16, in place
  const void* x; int ldx;          // [B*Q][ldx] bf16
  int B, Q;
  const void* wo; const float* bo; // out_proj (packed)
  const float* g; const float* b;
  // merge form (pm set, Q <= 48): x is the cross-attention's output computed here from xattn's
  // key-split partials (XattnArgs::partials_only) -- o_h = Wv_h u_h + bv_h, heads of 32
  const float *pm, *pl, *pu; int splits;
  const void* wv; const float* bv; // value rows of in_proj (packed)
};
// The decoder FFN's split-F product (decsa.hip, bf16, d = 256): partial [F/256][M][256] fp32 =
// relu(x . W1c^T + b1c) . W2c^T per 256-wide hidden chunk c; spe_launch_ffn_reduce_ln finishes.
// w1: W1 [F][256] fragment-packed; w2: chunk c's columns of W2 [256][F] packed at c * 256 * 256.
struct DecFfnArgs {
  const void* x; int ldx; int M, F;
  const void* w1; const float* b1; const void* w2;
  float* partial;
};
int spe_launch_decffn(const DecFfnArgs& a, hipStream_t s);
// y [M][ldy] = x . W^T (+ bias) + R[m % period] (decsa.hip; bf16, K = 256, N % 256 == 0; W packed)
struct DecQArgs {
  const void* x; int ldx; int M, N;
  const void* w; const float* bias;
  const void* R; int ldr; int period;   // optional row-periodic residual, bf16
  void* y; int ldy;
};
int spe_launch_decq(const DecQArgs& a, hipStream_t s);
// bf16 rows W [N][ld] (K = 256, N % 16 == 0) -> the fragment-packed layout above
int spe_launch_wfrag_pack(const void* w, int ld, int N, void* dst, hipStream_t s);
int spe_launch_decproj(const DecProjArgs& a, hipStream_t s);   // 1 = not applicable

// Fused FFN + residual + LayerNorm (bf16 only): y = LN(x + W2 relu(W1 x + b1) + b2).
// x / y may alias (each block reads and writes only its own rows).
struct FfnArgs {
  const void* x; int ldx;          // [M][256] bf16 (input and residual)
  const void* w1; int ld1;         // [F][ld1] bf16 (linear1.weight, K padded)
  const float* b1;                 // [F]
  const void* w2; int ld2;         // [256][ld2] bf16 (linear2.weight)
  const float* b2;                 // [256]
  const float* gamma; const float* beta;   // LayerNorm affine [256]
  void* y; int ldy;                // [M][256] bf16
  int M, D, F;
  const void* pos; void* ypos;     // optional: ypos = y + pos[m % pos_period] (bf16 [M][256])
  int pos_period;
  int splits; float* partial;      // optional split over F for few rows: fp32 [splits][M][256] workspace
  int row0;                        // first row of this launch's tiles (internal: the FFN tail launch)
  int w2_chunked;                  // w2 stored chunk-packed [F/32][256][32] (spe_launch_ffn_w2_chunk_pack); ld2 unused
};
// W2 [256][ld2] bf16 -> [F/32][256][32]: each 32-unit hidden chunk's columns as one contiguous block
int spe_launch_ffn_w2_chunk_pack(const void* w2, int ld2, int F, void* dst, hipStream_t s);
int spe_launch_ffn_ln(const FfnArgs& a, hipStream_t s);
// y = LN(x + sum_s partial[s] + b2) over a.splits fp32 partials [splits][M][256] (ffn.hip)
int spe_launch_ffn_reduce_ln(const FfnArgs& a, hipStream_t s);
// fp32h3 encoder FFN + residual + LayerNorm in one pass (ffn_h3.hip): fp32 x / y [M][256], W1 as its
// h3 finalize planes fp16 [2][F][ld1] (rows scaled by 2^e1), meta1 [F/32][64] = (2^-e1, b1) of each
// 32-unit hidden chunk, W2 as fp16 planes [2][256][ld2] (rows scaled by 2^e2) with the columns of
// every 32-wide chunk in spe_ffn_h3_perm order, sinv2 = 2^-e2; amax_x = the bound on |x| (the A
// scale), sh = the power-of-two scale of the hidden activation (from its static bound)
struct FfnH3Args {
  const float* x; int ldx;
  float* y; int ldy;
  int M, D, F;
  const void* w1; int ld1; const float* meta1;
  const void* w2; int ld2; const float* sinv2; const float* b2;
  const float* gamma; const float* beta;
  const float* amax_x; float sh;
};
int spe_launch_ffn_h3(const FfnH3Args& a, hipStream_t s);
int spe_ffn_h3_perm(int p);
int spe_ffn_splits(int M, int F);  // split count spe_launch_ffn_ln would use for M rows (1 = none)

int spe_launch_preprocess(const uint8_t* frames, int B, int H, int W, int C, const double* bbox, int S,
                          float* images, float* clip_bbox, int32_t* status, hipStream_t s);
// The model input: the ImageNet-normalised fp32 batch [B][3][S][S] (f32), or the 8-bit crops
// [B][S][S][ch] (u8, ch = 1 grayscale -- SPEED's frames, Image.convert('RGB') replicating them --
// or 3 RGB) that to_tensor + Normalize (REV/datasets/speed.py:25-41) turn into it: the pack kernels
// normalise u8 / 255, (x - mean) / std in fp32, the reference's operation order (bit-identical to
// the f32 input computed the same way)
struct ImageSrc {
  const float* f32; const uint8_t* u8; int ch;
};
// amax (fp32 output only, nullable): max |image| atomically maxed in (the stem GEMM's fp32h3 scale input)
// cpad: channels per packed pixel (8; fp32 models' DETR stem: 4, one 16-byte chunk)
int spe_launch_pack_input(const ImageSrc& img, void* out, int B, int S, int dtype, hipStream_t s, float* amax = nullptr,
                          int cpad = 8);
inline int spe_launch_pack_input(const float* img, void* out, int B, int S, int dtype, hipStream_t s,
                                 float* amax = nullptr, int cpad = 8) {
  return spe_launch_pack_input(ImageSrc{img, nullptr, 0}, out, B, S, dtype, s, amax, cpad);
}
// bf16 [B][S+6][S+6][4], zero border of 3 (the pair-packed stem's input, forward.cpp)
int spe_launch_pack_input_pad4(const ImageSrc& img, void* out, int B, int S, hipStream_t s);
// bf16 pair-packed stem (x: spe_launch_pack_input_pad4 layout, w: [64][ldw] k = (kh*8 + kw)*4 + ci)
// + bias + ReLU + 3x3/s2/p1 max-pool in one pass (stempool.hip); out [B][Po][Po] rows of stride
// ldo.  Returns 1 when the shape does not fit the kernel.
bool spe_stempool_enabled();
bool spe_stempool_fits(int S);
int spe_launch_stempool(const void* x, const void* w, int ldw, const float* bias, void* out, int ldo, int B, int S,
                        hipStream_t s);
int spe_launch_maxpool3s2(const void* in, void* out, int B, int H, int W, int C, int Ho, int Wo,
                          int dtype, hipStream_t s, int ldo = 0);   // ldo: output row stride (0 = C)
int spe_launch_upsample2x(const void* in, void* out, int B, int H, int W, int C, int dtype, hipStream_t s);
// conv3x3(pad 1)(upsample2x(x)) from the per-tap low-resolution products z [B*H*W][9*C]
// (elementwise.hip); out rows of stride ldo (a channel slice of a concat buffer)
int spe_launch_upconv_combine(const void* z, void* out, int ldo, int B, int H, int W, int C, int dtype, hipStream_t s);
int spe_launch_layernorm(const void* x, const float* gamma, const float* beta, void* out, float* out_f32,
                         int M, int D, int dtype, hipStream_t s);

struct HeadArgs {
  const float* hs;                 // [B*Q][256] fp32 (decoder_norm output of the last layer)
  int B, Q, D;
  const float* cls_wt; const float* cls_b;        // [D][12], [12]
  const float* pt_w0t; const float* pt_b0;        // [D][D]
  const float* pt_w1t; const float* pt_b1;
  const float* pt_w2t; const float* pt_b2;        // [D][2]
  const float* sg_w0t; const float* sg_b0;        // sigma head (nullable)
  const float* sg_w1t; const float* sg_b1;
  const float* sg_w2t; const float* sg_b2;        // [D][1]
  const float* clip_bbox;          // [B][4] (nullable -> no pixel rescale)
  float* logits;                   // [B][Q][12]
  float* points;                   // [B][Q][2] crop-normalised (sigmoid)
  float* probs;                    // [B][Q][12] softmax (nullable)
  float* points_px;                // [B][Q][2] image px (nullable)
  float* log_sigmas;               // [B][Q][2] (nullable)
  float* sigmas;                   // [B][Q][2] exp (nullable)
};
int spe_launch_heads(const HeadArgs& a, hipStream_t s);

// Set criterion (criterion.hip): Hungarian matching + losses for L layers of B images.
struct CritArgs {
  const float* logits;             // [L][B][Q][C]
  const float* points;             // [L][B][Q][2]
  const int32_t* tgt_labels;       // [B][T]
  const float* tgt_points;         // [B][T][2]
  int L, B, Q, C, T;
  float cost_class, cost_pts, eos_coef;
  double num_points;               // loss_points normaliser
  int32_t* match;                  // [L][B][T] matched query per target (out)
  double* partial;                 // [L][B][5] scratch
  double* losses;                  // [L][4] loss_ce, class_error, cardinality_error, loss_points (out)
};
int spe_launch_criterion(const CritArgs& a, hipStream_t s);

// Multi-model keypoint fusion (ensemble.hip): M models' PostProcess outputs -> one fused
// keypoint set per image in spe_pnp_batch's input layout.
struct EnsembleArgs {
  const float* points;             // [M][B][Q][2] image px
  const float* probs;              // [M][B][Q][C]
  int M, B, Q, C;
  float* fused_points;             // [B][C-1][2]
  float* fused_probs;              // [B][C-1][C] one-hot rows (background padding)
};
int spe_launch_ensemble_fuse(const EnsembleArgs& a, hipStream_t s);
int spe_launch_postprocess(const float* logits, const float* points, const float* clip_bbox, int B, int Q,
                           float* probs, float* points_px, hipStream_t s);

// ---- UNC RT-DETR (rtdetr.hip, rtdetr_model.cpp)
// nearest x2 (mode 0) / bicubic x0.5 (mode 1) resample of NHWC [B][H][W][C] (row stride ldi)
// into [B][Ho][Wo] rows of stride ldo (a channel slice of a concat buffer)
int spe_launch_resample2x(const void* in, int ldi, void* out, int ldo, int B, int H, int W, int C, int mode, int dtype,
                          hipStream_t s);
struct RtSelectArgs {
  const float* logits; int C;      // enc_score_head [level-major rows][C] fp32
  const void* memory; int ldm;     // output_memory (enc_output), level-major rows, T
  const float* anchors;            // [L][2] per-image token anchors (logit domain)
  int B, Q, D, levels;
  int lvl_start[5];                // token offsets of the levels within an image, [levels] = L
  int* topk;                       // [B][Q] selected token indices, descending score
  void* target; int ldt;           // [B*Q][D] T gathered output_memory rows
  float* sel_logits;               // [B*Q][C]
  float* sel_anchors;              // [B*Q][2]
};
int spe_launch_query_select(const RtSelectArgs& a, int dtype, hipStream_t s);
int spe_launch_qpos_hidden(const float* ref, const float* w0, const float* b0, void* out, int rows, int H, int dtype,
                           hipStream_t s);
struct RtDeformArgs {
  const void* value; int ldv;      // level-major rows [lvl_rows0[l] + b*H_l*W_l + y*W_l + x], T, heads h*32+c
  const float* so_aw; int ld_so;   // [rows][2*H*NL*NP offsets | H*NL*NP attention logits] fp32
  const float* ref;                // [rows][2] reference points (sigmoid domain)
  void* out; int ldo;              // [rows][256] T
  int rows, Q, heads, levels, points;
  int lvl_h[4], lvl_w[4], lvl_rows0[4];
};
int spe_launch_msdeform(const RtDeformArgs& a, int dtype, hipStream_t s);
struct RtHeadArgs {
  int rows, Q, C;
  const float* hs;                 // [rows][256] fp32 layer output (score head input; null: no score head)
  const float* cls_w; const float* cls_b;   // [C][256], [C]
  const void* h2; int ld_h2;       // T: box hidden (cols 0..255), sigma hidden (cols 256..511)
  const float* box_w2; const float* box_b2; // [2][256], [2]
  const float* sig_w2; const float* sig_b2; // [1][256], [1] (null: no sigma head)
  const float* pt_add; int pt_add_invsig;   // [rows][2]: anchors, or reference points (inverse_sigmoid)
  float* logits; float* probs;     // [rows][C]
  float* points;                   // [rows][2] sigmoid
  const float* clip_bbox; float* points_px;
  float* log_sigmas; float* sigmas;         // [rows][2]
};
int spe_launch_head_finish(const RtHeadArgs& a, int dtype, hipStream_t s);
