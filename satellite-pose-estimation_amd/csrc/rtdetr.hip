// Kernels of the UNC RT-DETR keypoint model that have no counterpart in the DETR path
// (SURVEY §8f.4); everything else (convs, linears, attention, LayerNorm, heads) reuses the
// GEMM / attention / elementwise / heads kernels.
//
//   resample2x     HybridEncoder FPN nearest x2 upsample and PAN bicubic x0.5 downsample
//                  (UNC/src/zoo/rtdetr/hybrid_encoder.py:371-397: F.interpolate nearest /
//                  bicubic, align_corners=False, a = -0.75, clamped taps), NHWC, writing a
//                  channel slice of the concat buffer the CSPRepLayer reads
//   query_select   RTDETRTransformer._get_decoder_input (rtdetr_decoder.py:613-667): per image,
//                  torch.topk(max over classes of enc_score_head, num_queries) (descending),
//                  gather of output_memory rows (decoder target), encoder class logits and
//                  anchors; one workgroup per image
//   qpos_hidden    query_pos_head layer 0 (MLP(2, 512, 256), rtdetr_decoder.py:459,298-300):
//                  relu(W0 . ref + b0) with K = 2, written as the A operand of layer 1's GEMM
//   head_finish    the last layers of the score / box / sigma heads (rtdetr_decoder.py:335-372):
//                  logits = hs W_c^T + b_c, box = sigmoid(h2_box W_2^T + b_2 + inverse_sigmoid(ref))
//                  (or + anchors for the encoder selection, :638), log-sigma = h2_sig w^T + b
//                  repeated to 2, and the fused RTDETRPostProcessor; the heads' 256-wide hidden
//                  layers run as GEMMs before it.  One wave per query row.
//   msdeform       MSDeformableAttention core (rtdetr_decoder.py:105-196 + utils.py:15-64):
//                  per (query, head) softmax over levels x points of the attention logits,
//                  sampling location = ref + offset / (W_l, H_l), bilinear grid_sample
//                  (align_corners=False, zero padding) of the level's value map, weighted sum
//
// Memory (the decoder's value input) is level-major: rows [level][image][y * W_l + x].
#include "spe_common.h"
#include "spe_kernels.h"

#include <algorithm>

namespace {

// ---------------------------------------------------------------- resample2x
// MODE 0: nearest x2 (out (y, x) <- in (y/2, x/2)); MODE 1: bicubic x0.5 (out (y, x) <- 4x4
// taps around in (2y + 0.5, 2x + 0.5), weights -3/32, 19/32, 19/32, -3/32, indices clamped),
// rows first then columns like ATen's separable cpu_upsample_generic.
template <typename T, int MODE>
__global__ void resample2x_kernel(const T* __restrict__ in, int ldi, T* __restrict__ out, int ldo, int B, int H, int W,
                                  int C) {
  constexpr int CE = Chunk<T>::CE;
  const int Ho = MODE == 0 ? 2 * H : H / 2, Wo = MODE == 0 ? 2 * W : W / 2;
  const int cch = C / CE;
  const size_t n = (size_t)B * Ho * Wo * cch;
  for (size_t i = blockIdx.x * (size_t)blockDim.x + threadIdx.x; i < n; i += (size_t)gridDim.x * blockDim.x) {
    const int c = (int)(i % cch);
    size_t r = i / cch;
    const int ox = (int)(r % Wo);
    r /= Wo;
    const int oy = (int)(r % Ho);
    const int b = (int)(r / Ho);
    T* dst = out + (((size_t)b * Ho + oy) * Wo + ox) * ldo + c * CE;
    if constexpr (MODE == 0) {
      st16(dst, ld16(in + (((size_t)b * H + (oy >> 1)) * W + (ox >> 1)) * ldi + c * CE));
    } else {
      const float wt[4] = {-0.09375f, 0.59375f, 0.59375f, -0.09375f};
      float acc[CE];
#pragma unroll
      for (int e = 0; e < CE; ++e) acc[e] = 0.f;
#pragma unroll
      for (int j = 0; j < 4; ++j) {
        const int y = min(max(2 * oy - 1 + j, 0), H - 1);
        float row[CE];
#pragma unroll
        for (int e = 0; e < CE; ++e) row[e] = 0.f;
#pragma unroll
        for (int k = 0; k < 4; ++k) {
          const int x = min(max(2 * ox - 1 + k, 0), W - 1);
          float f[CE];
          unpack16<T>(ld16(in + (((size_t)b * H + y) * W + x) * ldi + c * CE), f);
#pragma unroll
          for (int e = 0; e < CE; ++e) row[e] = k == 0 ? f[e] * wt[0] : row[e] + f[e] * wt[k];
        }
#pragma unroll
        for (int e = 0; e < CE; ++e) acc[e] = j == 0 ? row[e] * wt[0] : acc[e] + row[e] * wt[j];
      }
      st16(dst, pack16<T>(acc));
    }
  }
}

// ---------------------------------------------------------------- query_select
constexpr int SEL_NT = 256;
constexpr int SEL_MAXL = 12288;       // tokens per image (640 input: 6400 + 1600 + 400)

template <typename T>
__global__ __launch_bounds__(SEL_NT) void query_select_kernel(RtSelectArgs a) {
  __shared__ float sc[SEL_MAXL];
  __shared__ float rv[SEL_NT / 64];
  __shared__ int ri[SEL_NT / 64];
  __shared__ int sel[64];
  const int b = blockIdx.x, tid = threadIdx.x, lane = tid & 63, wid = tid >> 6;
  const int L = a.lvl_start[a.levels];
  // token t of image b lives at level-major row  lvl_rows0[l] + b * hw_l + (t - lvl_start[l])
  auto row_of = [&](int t) {
    int l = 0;
    while (l + 1 < a.levels && t >= a.lvl_start[l + 1]) ++l;
    const int hw = a.lvl_start[l + 1] - a.lvl_start[l];
    return (size_t)a.B * a.lvl_start[l] + (size_t)b * hw + (t - a.lvl_start[l]);
  };
  for (int t = tid; t < L; t += SEL_NT) {
    const float* lg = a.logits + row_of(t) * a.C;
    float mx = lg[0];
    bool nan = mx != mx;
    for (int c = 1; c < a.C; ++c) { mx = fmaxf(mx, lg[c]); nan |= lg[c] != lg[c]; }
    // torch: max(-1) propagates NaN and topk ranks NaN above every number; NaN is kept
    // out of sc (it marks taken tokens below), so a NaN score ranks as +inf
    sc[t] = nan ? INFINITY : mx;
  }
  __syncthreads();
  // Q rounds of block argmax: descending values, lower token index first among equal values;
  // taken tokens hold NaN, which fails every comparison
  for (int k = 0; k < a.Q; ++k) {
    float bv = -INFINITY;
    int bi = 0x7fffffff;
    for (int t = tid; t < L; t += SEL_NT) {
      const float v = sc[t];
      if (v > bv || (v == bv && t < bi)) { bv = v; bi = t; }
    }
#pragma unroll
    for (int o = 32; o > 0; o >>= 1) {
      const float ov = __shfl_xor(bv, o, 64);
      const int oi = __shfl_xor(bi, o, 64);
      if (ov > bv || (ov == bv && oi < bi)) { bv = ov; bi = oi; }
    }
    if (lane == 0) { rv[wid] = bv; ri[wid] = bi; }
    __syncthreads();
    if (tid == 0) {
      float v = rv[0];
      int idx = ri[0];
      for (int w = 1; w < SEL_NT / 64; ++w)
        if (rv[w] > v || (rv[w] == v && ri[w] < idx)) { v = rv[w]; idx = ri[w]; }
      if (idx < 0 || idx >= L) idx = 0;         // unreachable while L >= Q (host-checked)
      sel[k] = idx;
      sc[idx] = __builtin_nanf("");
      a.topk[(size_t)b * a.Q + k] = idx;
    }
    __syncthreads();
  }
  // gathers: decoder target rows, encoder logits of the selected queries, anchors
  const int D = a.D;
  for (int k = 0; k < a.Q; ++k) {
    const size_t src = row_of(sel[k]), dst = (size_t)b * a.Q + k;
    const T* mr = (const T*)a.memory + src * a.ldm;
    T* tr = (T*)a.target + dst * a.ldt;
    for (int c = tid; c < D; c += SEL_NT) tr[c] = mr[c];
    if (tid < a.C) a.sel_logits[dst * a.C + tid] = a.logits[src * a.C + tid];
    if (tid < 2) a.sel_anchors[dst * 2 + tid] = a.anchors[(size_t)sel[k] * 2 + tid];
  }
}

// ---------------------------------------------------------------- qpos_hidden
template <typename T>
__global__ void qpos_hidden_kernel(const float* __restrict__ ref, const float* __restrict__ w0, const float* __restrict__ b0,
                                   T* __restrict__ out, int rows, int H) {
  const size_t n = (size_t)rows * H;
  for (size_t i = blockIdx.x * (size_t)blockDim.x + threadIdx.x; i < n; i += (size_t)gridDim.x * blockDim.x) {
    const int j = (int)(i % H);
    const size_t r = i / H;
    const float v = ref[2 * r] * w0[2 * j] + ref[2 * r + 1] * w0[2 * j + 1] + b0[j];
    out[i] = from_f32<T>(fmaxf(v, 0.f));
  }
}


// ---------------------------------------------------------------- head_finish
template <typename T>
__global__ __launch_bounds__(256) void head_finish_kernel(RtHeadArgs a) {
  const int lane = threadIdx.x & 63, row = blockIdx.x * 4 + (threadIdx.x >> 6);
  if (row >= a.rows) return;
  const int C = a.C;
  auto dot = [&](const float* x, const float* w) {       // 256-long, 4 per lane, wave reduction
    const float4 xv = *reinterpret_cast<const float4*>(x + 4 * lane);
    const float4 wv = *reinterpret_cast<const float4*>(w + 4 * lane);
    return wave_sum(xv.x * wv.x + xv.y * wv.y + xv.z * wv.z + xv.w * wv.w);
  };
  auto dotT = [&](const T* x, const float* w) {
    float f[4];
#pragma unroll
    for (int e = 0; e < 4; ++e) f[e] = to_f32(x[4 * lane + e]);
    const float4 wv = *reinterpret_cast<const float4*>(w + 4 * lane);
    return wave_sum(f[0] * wv.x + f[1] * wv.y + f[2] * wv.z + f[3] * wv.w);
  };
  if (a.cls_w) {
    float lg[16];
    const float* hs = a.hs + (size_t)row * 256;
    for (int c = 0; c < C; ++c) lg[c] = dot(hs, a.cls_w + (size_t)c * 256) + a.cls_b[c];
    if (lane == 0) {
      float mx = -INFINITY, e[16], sum = 0.f;
      for (int c = 0; c < C; ++c) { a.logits[(size_t)row * C + c] = lg[c]; mx = fmaxf(mx, lg[c]); }
      for (int c = 0; c < C; ++c) { e[c] = expf(lg[c] - mx); sum += e[c]; }
      if (a.probs)
        for (int c = 0; c < C; ++c) a.probs[(size_t)row * C + c] = e[c] / sum;
    }
  }
  const T* h2 = (const T*)a.h2 + (size_t)row * a.ld_h2;
  float dx = dotT(h2, a.box_w2) + a.box_b2[0];
  float dy = dotT(h2, a.box_w2 + 256) + a.box_b2[1];
  float sg = a.sig_w2 ? dotT(h2 + 256, a.sig_w2) + a.sig_b2[0] : 0.f;
  if (lane != 0) return;
  float ax = a.pt_add[(size_t)row * 2], ay = a.pt_add[(size_t)row * 2 + 1];
  if (a.pt_add_invsig) {            // inverse_sigmoid (UNC/src/zoo/rtdetr/utils.py:10-12)
    auto invsig = [](float v) {
      v = fminf(fmaxf(v, 0.f), 1.f);
      return logf(fmaxf(v, 1e-5f) / fmaxf(1.f - v, 1e-5f));
    };
    ax = invsig(ax);
    ay = invsig(ay);
  }
  dx = dx + ax;
  dy = dy + ay;
  const float px = 1.f / (1.f + expf(-dx)), py = 1.f / (1.f + expf(-dy));
  a.points[(size_t)row * 2] = px;
  a.points[(size_t)row * 2 + 1] = py;
  if (a.points_px && a.clip_bbox) {
    const float* bb = a.clip_bbox + (size_t)(row / a.Q) * 4;
    a.points_px[(size_t)row * 2] = px * (bb[2] - bb[0]) + bb[0];
    a.points_px[(size_t)row * 2 + 1] = py * (bb[3] - bb[1]) + bb[1];
  }
  if (a.sig_w2) {
    if (a.log_sigmas) { a.log_sigmas[(size_t)row * 2] = sg; a.log_sigmas[(size_t)row * 2 + 1] = sg; }
    if (a.sigmas) { const float e = expf(sg); a.sigmas[(size_t)row * 2] = e; a.sigmas[(size_t)row * 2 + 1] = e; }
  }
}

// ---------------------------------------------------------------- msdeform
// One workgroup of 256 threads per query row; thread = output channel h*32 + c.  The 8 heads'
// softmax over levels x points (<= 32 logits each) is computed by the first lanes into LDS.
template <typename T>
__global__ __launch_bounds__(256) void msdeform_kernel(RtDeformArgs a) {
  constexpr int MAXP = 8 * 4 * 4;      // heads x levels x points
  __shared__ float w[MAXP], lx[MAXP], ly[MAXP];
  const int row = blockIdx.x, tid = threadIdx.x;
  const int b = row / a.Q;
  const int H = a.heads, NL = a.levels, NP = a.points, LP = NL * NP;
  const float* so = a.so_aw + (size_t)row * a.ld_so;        // [H][NL][NP][2] offsets, then [H][NL*NP] logits
  const float rx = a.ref[2 * row], ry = a.ref[2 * row + 1];
  if (tid < H) {
    const float* lg = so + 2 * H * LP + tid * LP;
    float mx = lg[0];
    for (int i = 1; i < LP; ++i) mx = fmaxf(mx, lg[i]);
    float s = 0.f;
    for (int i = 0; i < LP; ++i) { const float e = expf(lg[i] - mx); w[tid * LP + i] = e; s += e; }
    for (int i = 0; i < LP; ++i) w[tid * LP + i] = w[tid * LP + i] / s;
  }
  if (tid < H * LP) {
    const int l = (tid % LP) / NP;
    const float Wl = (float)a.lvl_w[l], Hl = (float)a.lvl_h[l];
    // sampling_locations = ref + offset / (W_l, H_l); grid = 2 loc - 1; grid_sample unnormalises
    // ((grid + 1) * size - 1) / 2 (align_corners=False)
    const float locx = rx + so[2 * tid] / Wl, locy = ry + so[2 * tid + 1] / Hl;
    const float gx = 2.f * locx - 1.f, gy = 2.f * locy - 1.f;
    lx[tid] = ((gx + 1.f) * Wl - 1.f) / 2.f;
    ly[tid] = ((gy + 1.f) * Hl - 1.f) / 2.f;
  }
  __syncthreads();
  const int h = tid >> 5, c = tid & 31;
  if (h >= H) return;
  float acc = 0.f;
  for (int l = 0; l < NL; ++l) {
    const int Wl = a.lvl_w[l], Hl = a.lvl_h[l];
    const T* vbase = (const T*)a.value + ((size_t)a.lvl_rows0[l] + (size_t)b * Wl * Hl) * a.ldv + h * 32 + c;
    for (int p = 0; p < NP; ++p) {
      const int s = h * LP + l * NP + p;
      const float ix = lx[s], iy = ly[s];
      const float fx = floorf(ix), fy = floorf(iy);
      const int x0 = (int)fx, y0 = (int)fy;
      const float tx = ix - fx, ty = iy - fy;
      // ATen grid_sampler_2d bilinear: nw/ne/sw/se weights, out-of-range corners read as zero
      const float nw = (1.f - tx) * (1.f - ty), ne = tx * (1.f - ty), sw = (1.f - tx) * ty, se = tx * ty;
      auto at = [&](int y, int x) {
        return (x >= 0 && x < Wl && y >= 0 && y < Hl) ? to_f32(vbase[((size_t)y * Wl + x) * a.ldv]) : 0.f;
      };
      const float v = at(y0, x0) * nw + at(y0, x0 + 1) * ne + at(y0 + 1, x0) * sw + at(y0 + 1, x0 + 1) * se;
      acc += v * w[s];
    }
  }
  ((T*)a.out)[(size_t)row * a.ldo + tid] = from_f32<T>(acc);
}

}  // namespace

int spe_launch_resample2x(const void* in, int ldi, void* out, int ldo, int B, int H, int W, int C, int mode, int dtype,
                          hipStream_t s) {
  const int ce = dtype == SPE_DTYPE_BF16 ? 8 : 4;
  if (B <= 0) return 0;
  if (C % ce || ldi % ce || ldo % ce || (mode == 1 && (H % 2 || W % 2))) return -5;
  const size_t px = (size_t)B * H * W * (mode == 0 ? 4 : 1) / (mode == 0 ? 1 : 4);
  const size_t n = px * (C / ce);
  const int blocks = (int)std::min<size_t>((n + 255) / 256, 65535);
  if (dtype == SPE_DTYPE_BF16) {
    if (mode == 0) hipLaunchKernelGGL((resample2x_kernel<bf16, 0>), dim3(blocks), dim3(256), 0, s, (const bf16*)in, ldi, (bf16*)out, ldo, B, H, W, C);
    else hipLaunchKernelGGL((resample2x_kernel<bf16, 1>), dim3(blocks), dim3(256), 0, s, (const bf16*)in, ldi, (bf16*)out, ldo, B, H, W, C);
  } else {
    if (mode == 0) hipLaunchKernelGGL((resample2x_kernel<float, 0>), dim3(blocks), dim3(256), 0, s, (const float*)in, ldi, (float*)out, ldo, B, H, W, C);
    else hipLaunchKernelGGL((resample2x_kernel<float, 1>), dim3(blocks), dim3(256), 0, s, (const float*)in, ldi, (float*)out, ldo, B, H, W, C);
  }
  return (int)hipGetLastError();
}

int spe_launch_query_select(const RtSelectArgs& a, int dtype, hipStream_t s) {
  if (a.B <= 0) return 0;
  if (a.levels < 1 || a.levels > 4 || a.lvl_start[a.levels] > SEL_MAXL || a.Q < 1 || a.Q > 64 ||
      a.Q > a.lvl_start[a.levels] || a.C < 1 || a.C > 256)
    return -5;
  if (dtype == SPE_DTYPE_BF16) hipLaunchKernelGGL(query_select_kernel<bf16>, dim3(a.B), dim3(SEL_NT), 0, s, a);
  else hipLaunchKernelGGL(query_select_kernel<float>, dim3(a.B), dim3(SEL_NT), 0, s, a);
  return (int)hipGetLastError();
}

int spe_launch_qpos_hidden(const float* ref, const float* w0, const float* b0, void* out, int rows, int H, int dtype,
                           hipStream_t s) {
  if (rows <= 0) return 0;
  const size_t n = (size_t)rows * H;
  const int blocks = (int)std::min<size_t>((n + 255) / 256, 65535);
  if (dtype == SPE_DTYPE_BF16) hipLaunchKernelGGL(qpos_hidden_kernel<bf16>, dim3(blocks), dim3(256), 0, s, ref, w0, b0, (bf16*)out, rows, H);
  else hipLaunchKernelGGL(qpos_hidden_kernel<float>, dim3(blocks), dim3(256), 0, s, ref, w0, b0, (float*)out, rows, H);
  return (int)hipGetLastError();
}

int spe_launch_msdeform(const RtDeformArgs& a, int dtype, hipStream_t s) {
  if (a.rows <= 0) return 0;
  if (a.heads * 32 != 256 || a.heads * a.levels * a.points > 128 || a.levels > 4 || a.points > 4) return -5;
  if (dtype == SPE_DTYPE_BF16) hipLaunchKernelGGL(msdeform_kernel<bf16>, dim3(a.rows), dim3(256), 0, s, a);
  else hipLaunchKernelGGL(msdeform_kernel<float>, dim3(a.rows), dim3(256), 0, s, a);
  return (int)hipGetLastError();
}

int spe_launch_head_finish(const RtHeadArgs& a, int dtype, hipStream_t s) {
  if (a.rows <= 0) return 0;
  if (a.C > 16 || !a.points || !a.pt_add || !a.h2 || (a.cls_w && (!a.hs || !a.logits))) return -5;
  const int blocks = (a.rows + 3) / 4;
  if (dtype == SPE_DTYPE_BF16) hipLaunchKernelGGL(head_finish_kernel<bf16>, dim3(blocks), dim3(256), 0, s, a);
  else hipLaunchKernelGGL(head_finish_kernel<float>, dim3(blocks), dim3(256), 0, s, a);
  return (int)hipGetLastError();
}
