// Internal state of a spe_model (shared by registry.cpp and forward.cpp).
#pragma once
#include <hip/hip_runtime.h>

#include <cstdint>
#include <map>
#include <string>
#include <vector>

#include "../../include/spe.h"
#include "spe_kernels.h"

struct Conv {              // conv / linear packed as [N][Kpad] in T, bias fp32
  void* w = nullptr;
  float* bias = nullptr;
  int N = 0, K = 0, Kpad = 0, Cin = 0, KH = 1, KW = 1, stride = 1, pad = 0;
  float l1max = 0.f, bmax = 0.f;   // linears: max_n sum_k |W[n][k]| and max |bias| (|y| <= max |x| l1max + bmax)
};

struct Block {
  Conv c1, c2, c3, ds;
  Conv c3ds;               // bf16, stride-1 first block: [W3 | Wds] over [t2 | x] (K = w + cin), or empty
  Conv c1p;                // bf16, input = a layer-1 block output: conv1 with K columns in spe_btail_perm
                           // order, fused into the previous block's tail (btail.hip), or empty
  bool has_ds = false;
  int stride = 1;
};

struct Enc {
  Conv qk, v, o, l1, l2;
  float *n1g, *n1b, *n2g, *n2b;
  // fp32h3: device bounds on |norm1 / norm2 output| (max|gamma| sqrt(D - 1) + max|beta|: |x - mean|
  // / std <= sqrt(D - 1)), the scale input of the GEMMs that read them
  float *n1_bound = nullptr, *n2_bound = nullptr;
  void* pos_qk = nullptr;   // bf16 / fp32x6 models: pos . W_qk^T [tokens][512] (row-periodic residual)
  // fp32h3, the one-pass FFN (ffn_h3.hip): (2^-e1, b1) per 32-unit chunk, W2's planes with the columns
  // in spe_ffn_h3_perm order, and the hidden activation's power-of-two scale from its static bound
  float* ffn_meta1 = nullptr;
  void* ffn_w2p = nullptr;
  float ffn_sh = 0.f;
  void* ffn_w2c = nullptr;  // bf16: linear2's weight chunk-packed for the fused FFN (spe_launch_ffn_w2_chunk_pack)
};

struct Dec {
  Conv sqk, sv, so, cq, co, l1, l2;
  float *n1g, *n1b, *n2g, *n2b, *n3g, *n3b;
  float *n1_bound = nullptr, *n2_bound = nullptr, *n3_bound = nullptr;   // fp32h3 (see Enc)
  void* qpos_sqk = nullptr; // bf16 / fp32x6 models: query_pos . W_sqk^T [Q][512]
  void* qpos_cq = nullptr;  // bf16 models: query_pos . W_cq^T [Q][256]
  // cross-attention against the memory (spe_use_xattn, xattn.hip): q' = tgt . Wqk^T + xq_r
  // with Wq/Wk folded per head at finalize; xv = the value projection rows of in_proj
  Conv xq, xv;
  void* xq_r = nullptr;     // [Q][8*256] bf16: query_pos . Wqk^T + bqk (scaled)
  // bf16, d = 256: sqk / sv / so / co / xv fragment-packed for the decoder kernels (decsa.hip)
  void *fsqk = nullptr, *fsv = nullptr, *fso = nullptr, *fco = nullptr, *fxv = nullptr;
  void *fxq = nullptr;                   // xq packed (the folded cross-attention query projection)
  void *fl1 = nullptr, *fl2 = nullptr;   // linear1 / linear2 packed (fl2 per 256-wide hidden chunk; F % 256 == 0)
};

// fp32h3 activation-scale slots in the workspace: [0, SPE_AMAX_BB) written by the backbone stage,
// [SPE_AMAX_BB, SPE_AMAX_SLOTS) by the transformer stage (each stage zeroes its own range first)
// (the transformer stage's range is [SPE_AMAX_BB, SPE_AMAX_DEC), the decoder stage's [SPE_AMAX_DEC, SPE_AMAX_SLOTS))
constexpr int SPE_AMAX_BB = 96, SPE_AMAX_DEC = 112, SPE_AMAX_SLOTS = 136;   // decoder: 3 slots a layer

struct Ws {                // workspace layout (byte offsets)
  size_t x0, stem, pool, bufA, bufB, t1, t2, ds, xs8, up, cat, neck;
  size_t src, srcpos, qkv, vt, ao, tmp, ffn, ck, cvt;
  size_t kpl;                // fp32x3 / fp32x6: the encoder K as bf16 hi / lo planes (0 = none)
  size_t tgt, dtmp, dqkv, dvt, dao, dqc, dffn, dffnpart, hs;
  size_t xq, xu, xpm, xpl, xpu;           // cross-attention against the memory (xattn.hip)
  size_t xvp;                // fp32h3: the memory's fp16 value planes (xattn_h3.hip; the key planes go to srcpos)
  size_t amax;               // fp32h3: max |activation| slots (SPE_AMAX_SLOTS floats; backbone, then transformer)
  size_t total;
};

// Per-launch HIP-event profiler (spe_model_profile_*): brackets every launch whose kind
// starts with `filter` with events on the launch stream and accumulates algorithmic work.
struct ProfRecord {
  std::string kind, name;
  double flops, bytes;
  hipEvent_t beg, end;
};
struct Profiler {
  bool on = false;
  std::string filter;
  std::vector<ProfRecord> recs;
  std::vector<hipEvent_t> pool;
  size_t next_event = 0;
};

// ---- UNC RT-DETR (rtdetr_model.cpp)
struct RtBlock {             // PResNet BasicBlock / BottleNeck; shortcut conv (first block of a stage)
  Conv a, b, c, sc;          // variant d stride-2 shortcut: AvgPool2d(2, 2) + 1x1 folded into a 2x2/2 conv
  bool has_sc = false, bottleneck = false;
  int stride = 1, cin = 0, cout = 0;
};
struct RtCsp {               // CSPRepLayer, one RepVggBlock folded into one 3x3 conv (convert_to_deploy)
  Conv c1, c2, rep, c3;
  bool has_c3 = false;
};
struct RtHead {              // score / box MLP / sigma MLP heads of one layer (rtdetr_decoder.py:298-372)
  Conv h1, box1, sig1;       // h1: box.layers.0 | sigma.layers.0 stacked (N = 512, or 256 without sigma)
  float *cls_w = nullptr, *cls_b = nullptr, *box_w2 = nullptr, *box_b2 = nullptr;
  float *sig_w2 = nullptr, *sig_b2 = nullptr;   // last layers, fp32 [out][256]
};
struct RtDec {               // decoder layer + its heads
  Conv sqk, sv, so, soaw, oproj, l1, l2;   // soaw: sampling_offsets | attention_weights (N = 288)
  float *n1g, *n1b, *n2g, *n2b, *n3g, *n3b;
  RtHead head;
};
struct RtModel {
  spe_rtdetr_config cfg{};
  int L = 0, lvl_s[3] = {0, 0, 0}, lvl_start[4] = {0, 0, 0, 0};
  Conv stem[3];
  std::vector<RtBlock> blocks;
  int stage_first[4] = {0, 0, 0, 0}, stage_n[4] = {0, 0, 0, 0};
  Conv in_proj[3];
  Conv aqk, av, ao, al1, al2;          // AIFI encoder layer
  float *an1g, *an1b, *an2g, *an2b;
  void* aifi_pos = nullptr;             // [s2*s2][256] T, 2D sin-cos table
  Conv lateral[2];
  RtCsp fpn[2], pan[2];
  Conv dec_in[3], enc_out, enc_score, vproj;   // vproj: every layer's value_proj, N = 256 * dec_layers
  float *eo_g, *eo_b;
  float* anchors = nullptr;             // [L][2] fp32, logit domain
  RtHead enc_head;                      // enc_bbox_head (+ anchors, sigmoid): the initial reference points
  float *qp_w0 = nullptr, *qp_b0 = nullptr;   // query_pos_head layer 0 [512][2], [512]
  Conv qp_l1;
  std::vector<RtDec> dec;
};

struct spe_model {
  int family = 0;            // 0: DETR (REV), 1: RT-DETR (UNC)
  int x3 = 0;                // fp32 model computed with split-bf16 MFMA (SPE_DTYPE_F32X3_, _F32X6_)
  int x6 = 0;                // ... with the GEMMs / convs on the three-way split path (SPE_DTYPE_F32X6_)
  int h3 = 0;                // ... and the backbone / encoder GEMMs on the scaled fp16 split path (SPE_DTYPE_F32H3_)
  // fp32x6 models: fp32 weight block -> (its bf16 planes [3][rows][Kpad] h, m, l, rows), written
  // at finalize next to each packed weight (upload_rows) so the x6 GEMM never splits weights
  std::map<const void*, std::pair<const void*, int>> w6;
  // fp32h3 models: fp32 weight block -> its fp16 planes [2][rows][Kpad] (hi, lo of the row scaled by
  // 2^e_r) and the per-row 2^-e_r (upload_rows)
  struct H3W { const void* planes; int rows; const float* sinv; };
  std::map<const void*, H3W> wh3;
  RtModel* rt = nullptr;
  spe_model_config cfg{};
  int esz = 2;
  std::vector<std::pair<std::string, std::vector<int64_t>>> spec;
  std::map<std::string, std::vector<float>> host;
  bool finalized = false;
  char* dmem = nullptr;
  size_t dbytes = 0, dused = 0;
  int upload_err = 0;
  Conv stem, s8, s16, outc, inproj, crossK, crossV;
  Conv s16taps;            // bf16 models: s16_latern as 9 per-tap [256][1024] blocks (spe_use_upconv)
  Conv neckip;             // input_proj . output_conv as one 3x3 conv 512 -> hidden (spe_use_neckfold)
  std::vector<Block> blocks;
  std::vector<Enc> enc;
  std::vector<Dec> dec;
  void* pos = nullptr;     // [tokens][256] T
  void* qpos = nullptr;    // [Q][256] T
  void* pos_crossK = nullptr;  // bf16 / fp32x6 models: pos . W_crossK^T [tokens][L*256]
  float *dng = nullptr, *dnb = nullptr;
  HeadArgs head{};
  Profiler prof;
};

int spe_fail(int code, const std::string& msg);
// RT-DETR runtime hooks (rtdetr_model.cpp)
int spe_rtdetr_build_device(spe_model* m);
int64_t spe_rtdetr_workspace(const spe_model* m, int B);

// bf16 models take the decoder cross-attention against the memory itself (xattn.hip) when the
// last encoder layer can emit memory + pos (fused FFN); fp32h3 models too, on the memory's fp16
// planes (xattn_h3.hip), when the 8 * Q attention rows fit one 96-row work-group group (Q <= 12:
// BASELINE configs 2-4 and the north star).  At config 5 (Q = 40: four groups, each re-reading the
// memory) the fold measured no gain (48.75 vs 48.96 ms a step) and moved one of the precision study's
// 32 images to a RANSAC outcome none of three fp32 implementations reach, so
// Q > 12 keeps the projected K / V^T and the exact-f32 attention.  SPE_XATTN_H3=0: that path for
// every Q (A/B runs).
inline bool spe_use_xattn(const spe_model* m) {
  static const bool h3 = [] { const char* e = getenv("SPE_XATTN_H3"); return e ? atoi(e) != 0 : true; }();
  const auto& c = m->cfg;
  return (c.dtype == SPE_DTYPE_BF16_ || (h3 && m->h3 && 8 * c.num_queries <= 96)) && c.hidden_dim == 256 &&
         c.nheads == 8 && c.dim_feedforward % 32 == 0 && c.enc_layers > 0;
}
// bf16 and fp32x3 models evaluate s16_latern(up16sto8s(xs16)) at the low resolution (one
// per-tap GEMM + upconv_combine: exact by linearity, a different rounding order); the exact-f32
// parity mode keeps the reference's upsample-then-conv order
inline bool spe_use_upconv(const spe_model* m) {
  return (m->cfg.dtype == SPE_DTYPE_BF16_ || m->x3) && m->cfg.input_size % 16 == 0;
}
// bf16 and fp32x3 models fold input_proj (1x1 + bias) into output_conv (3x3 + bias): nothing
// nonlinear sits between them (REV/models/backbone.py:141, detr_speed.py:81), so
// input_proj(output_conv(x)) is one 3x3 conv 512 -> hidden_dim with per-tap weights
// W_ip . W_oc[:, :, kh, kw] and bias W_ip . b_oc + b_ip (folded in double at finalize): half the
// output_conv multiply-adds, no 512-channel neck output round trip, no input_proj launch.  The
// exact-f32 parity mode keeps the reference's two convolutions.  SPE_NECK_FOLD=0 disables it.
bool spe_use_neckfold(const spe_model* m);
Ws spe_plan(const spe_model* m, int B);
