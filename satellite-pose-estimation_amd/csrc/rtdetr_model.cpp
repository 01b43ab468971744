// Native runtime of the UNC RT-DETR keypoint model: parameter space in the
// reference's state_dict order (spe/rtdetr_spec.py mirrors it and tests pin it to the reference
// model's own keys), BatchNorm folding and the inference-time reparameterisations the reference
// itself defines, workspace plan and the launch sequence of RTDETR.forward in eval
// (UNC/src/zoo/rtdetr/rtdetr.py:36-53):
//
//   PResNet-vd (UNC/nn/backbone/presnet.py:156-265) -> HybridEncoder (hybrid_encoder.py:332-401)
//   -> RTDETRTransformer (rtdetr_decoder.py:505-710) -> RTDETRPostProcessor
//      (rtdetr_postprocessor.py:44-76)
//
// Folds: every ConvNormLayer's eval BatchNorm into its conv; RepVggBlock's 3x3 + 1x1 branches
// into one 3x3 conv (RepVggBlock.convert_to_deploy, hybrid_encoder.py:55-95); the variant-d
// shortcut AvgPool2d(2, 2, ceil_mode) + 1x1 conv into one 2x2 stride-2 conv with w/4 per tap
// (exact for the even feature sizes of inputs that are multiples of 32).
#include <hip/hip_runtime.h>

#include <cmath>
#include <cstdio>
#include <cstring>

#include "launch.h"
#include "model_state.h"
#include "registry.h"

#define fail spe_fail

namespace {

const int RESNET_CFG18[4] = {2, 2, 2, 2}, RESNET_CFG50[4] = {3, 4, 6, 3};

std::vector<std::pair<std::string, std::vector<int64_t>>> rt_spec(const spe_rtdetr_config& c) {
  std::vector<std::pair<std::string, std::vector<int64_t>>> s;
  const int64_t d = 256, C = c.num_classes + 1;
  auto add = [&](const std::string& k, std::vector<int64_t> sh) { s.emplace_back(k, std::move(sh)); };
  auto bn = [&](const std::string& p, int64_t ch) {
    for (const char* n : {"weight", "bias", "running_mean", "running_var"}) add(p + "." + n, {ch});
  };
  auto cnl = [&](const std::string& p, int64_t cin, int64_t cout, int64_t k) {
    add(p + ".conv.weight", {cout, cin, k, k});
    bn(p + ".norm", cout);
  };
  auto lin = [&](const std::string& p, int64_t o, int64_t i) { add(p + ".weight", {o, i}); add(p + ".bias", {o}); };
  auto mlp = [&](const std::string& p, std::vector<int64_t> dims) {
    for (size_t j = 0; j + 1 < dims.size(); ++j) lin(p + ".layers." + std::to_string(j), dims[j + 1], dims[j]);
  };
  auto mha = [&](const std::string& p) {
    add(p + ".in_proj_weight", {3 * d, d});
    add(p + ".in_proj_bias", {3 * d});
    lin(p + ".out_proj", d, d);
  };
  add("temper_param", {1});
  cnl("backbone.conv1.conv1_1", 3, 32, 3);
  cnl("backbone.conv1.conv1_2", 32, 32, 3);
  cnl("backbone.conv1.conv1_3", 32, 64, 3);
  const bool bott = c.depth >= 50;
  const int64_t exp = bott ? 4 : 1;
  const int* nb = bott ? RESNET_CFG50 : RESNET_CFG18;
  const int64_t widths[4] = {64, 128, 256, 512};
  int64_t cin = 64;
  for (int i = 0; i < 4; ++i)
    for (int j = 0; j < nb[i]; ++j) {
      const std::string p = "backbone.res_layers." + std::to_string(i) + ".blocks." + std::to_string(j);
      const int64_t co = widths[i];
      const bool s2 = j == 0 && i > 0;
      auto shortcut = [&] { if (j == 0) cnl(s2 ? p + ".short.conv" : p + ".short", cin, co * exp, 1); };
      if (bott) {
        cnl(p + ".branch2a", cin, co, 1);
        cnl(p + ".branch2b", co, co, 3);
        cnl(p + ".branch2c", co, co * exp, 1);
        shortcut();
      } else {                       // BasicBlock registers `short` before its branches
        shortcut();
        cnl(p + ".branch2a", cin, co, 3);
        cnl(p + ".branch2b", co, co, 3);
      }
      cin = co * exp;
    }
  const int NL = 3, NP = 4, H = 8, P = H * NL * NP;
  for (int l = 0; l < NL; ++l) cnl("decoder.input_proj." + std::to_string(l), d, d, 1);
  for (int i = 0; i < c.dec_layers; ++i) {
    const std::string p = "decoder.decoder.layers." + std::to_string(i);
    mha(p + ".self_attn");
    add(p + ".norm1.weight", {d}); add(p + ".norm1.bias", {d});
    lin(p + ".cross_attn.sampling_offsets", 2 * P, d);
    lin(p + ".cross_attn.attention_weights", P, d);
    lin(p + ".cross_attn.value_proj", d, d);
    lin(p + ".cross_attn.output_proj", d, d);
    add(p + ".norm2.weight", {d}); add(p + ".norm2.bias", {d});
    lin(p + ".linear1", c.dec_ff, d);
    lin(p + ".linear2", d, c.dec_ff);
    add(p + ".norm3.weight", {d}); add(p + ".norm3.bias", {d});
  }
  for (int i = 0; i < c.dec_layers; ++i) mlp("decoder.decoder.sigma_embed." + std::to_string(i), {d, d, d, 1});
  mlp("decoder.query_pos_head", {2, 2 * d, d});
  lin("decoder.enc_output.0", d, d);
  add("decoder.enc_output.1.weight", {d}); add("decoder.enc_output.1.bias", {d});
  lin("decoder.enc_score_head", C, d);
  mlp("decoder.enc_bbox_head", {d, d, d, 2});
  for (int i = 0; i < c.dec_layers; ++i) lin("decoder.dec_score_head." + std::to_string(i), C, d);
  for (int i = 0; i < c.dec_layers; ++i) mlp("decoder.dec_bbox_head." + std::to_string(i), {d, d, d, 2});
  const int64_t bc[3] = {128 * exp, 256 * exp, 512 * exp};
  for (int l = 0; l < 3; ++l) {
    add("encoder.input_proj." + std::to_string(l) + ".0.weight", {d, bc[l], 1, 1});
    bn("encoder.input_proj." + std::to_string(l) + ".1", d);
  }
  add("encoder.encoder_fusion_input.weight", {d, 3 * d, 1, 1});
  const std::string a = "encoder.encoder.0.layers.0";
  mha(a + ".self_attn");
  lin(a + ".linear1", c.enc_ff, d);
  lin(a + ".linear2", d, c.enc_ff);
  for (const char* n : {"norm1", "norm2"}) { add(a + "." + n + ".weight", {d}); add(a + "." + n + ".bias", {d}); }
  for (int i = 0; i < 2; ++i) cnl("encoder.lateral_convs." + std::to_string(i), d, d, 1);
  const int64_t h = c.csp_hidden;
  for (const char* blocks : {"fpn_blocks", "pan_blocks"})
    for (int i = 0; i < 2; ++i) {
      const std::string p = std::string("encoder.") + blocks + "." + std::to_string(i);
      cnl(p + ".conv1", 2 * d, h, 1);
      cnl(p + ".conv2", 2 * d, h, 1);
      cnl(p + ".bottlenecks.0.conv1", h, h, 3);
      cnl(p + ".bottlenecks.0.conv2", h, h, 1);
      if (h != d) cnl(p + ".conv3", h, d, 1);
    }
  return s;
}

// rows [r0, r0+n) of several [*, K] weights stacked into one linear (one GEMM for several heads)
Conv stack_linears(spe_model* m, const std::vector<std::pair<std::string, std::string>>& parts, int K) {
  std::vector<float> rows, bias;
  int N = 0;
  for (auto& pr : parts) {
    const auto& w = m->host[pr.first];
    const auto& b = m->host[pr.second];
    rows.insert(rows.end(), w.begin(), w.end());
    bias.insert(bias.end(), b.begin(), b.end());
    N += (int)b.size();
  }
  Conv c;
  c.N = N; c.K = K; c.Kpad = pad64(K); c.Cin = K;
  c.w = upload_rows(m, rows, N, K, c.Kpad);
  c.bias = upload_f32(m, bias.data(), bias.size());
  return c;
}

RtHead make_head(spe_model* m, const std::string& cls, const std::string& box, const std::string& sigma) {
  RtHead h;
  std::vector<std::pair<std::string, std::string>> first{{box + ".layers.0.weight", box + ".layers.0.bias"}};
  if (!sigma.empty()) first.emplace_back(sigma + ".layers.0.weight", sigma + ".layers.0.bias");
  h.h1 = stack_linears(m, first, 256);
  h.box1 = make_linear(m, box + ".layers.1.weight", box + ".layers.1.bias", 0, 256, 256);
  h.box_w2 = upload_key(m, box + ".layers.2.weight");
  h.box_b2 = upload_key(m, box + ".layers.2.bias");
  if (!sigma.empty()) {
    h.sig1 = make_linear(m, sigma + ".layers.1.weight", sigma + ".layers.1.bias", 0, 256, 256);
    h.sig_w2 = upload_key(m, sigma + ".layers.2.weight");
    h.sig_b2 = upload_key(m, sigma + ".layers.2.bias");
  }
  if (!cls.empty()) {
    h.cls_w = upload_key(m, cls + ".weight");
    h.cls_b = upload_key(m, cls + ".bias");
  }
  return h;
}

// HybridEncoder.build_2d_sincos_position_embedding (hybrid_encoder.py:306-330) for a w x h grid,
// [w*h][256] in the reference's flatten order (meshgrid(w, h, 'ij'): token t <-> (t / h, t % h))
std::vector<float> sincos_2d(int w, int h, int d) {
  const int pd = d / 4;
  std::vector<float> omega(pd), out((size_t)w * h * d);
  for (int i = 0; i < pd; ++i) omega[i] = 1.0f / std::pow(10000.0f, (float)i / (float)pd);
  for (int t = 0; t < w * h; ++t) {
    const float gw = (float)(t / h), gh = (float)(t % h);
    float* o = &out[(size_t)t * d];
    for (int i = 0; i < pd; ++i) {
      const float ow = gw * omega[i], oh = gh * omega[i];
      o[i] = std::sin(ow);
      o[pd + i] = std::cos(ow);
      o[2 * pd + i] = std::sin(oh);
      o[3 * pd + i] = std::cos(oh);
    }
  }
  return out;
}

// RTDETRTransformer._generate_anchors (rtdetr_decoder.py:577-611): per token (x+0.5)/W,
// (y+0.5)/H, logit, +inf outside (eps, 1 - eps)
std::vector<float> make_anchors(const RtModel& r) {
  std::vector<float> a;
  const float eps = 1e-2f;
  for (int l = 0; l < 3; ++l) {
    const int s = r.lvl_s[l];
    for (int y = 0; y < s; ++y)
      for (int x = 0; x < s; ++x) {
        const float ax = ((float)x + 0.5f) / (float)s, ay = ((float)y + 0.5f) / (float)s;
        const bool valid = ax > eps && ax < 1 - eps && ay > eps && ay < 1 - eps;
        a.push_back(valid ? std::log(ax / (1 - ax)) : INFINITY);
        a.push_back(valid ? std::log(ay / (1 - ay)) : INFINITY);
      }
  }
  return a;
}

RtCsp make_csp(spe_model* m, const std::string& p, int h) {
  RtCsp c;
  c.c1 = make_conv(m, p + ".conv1.conv.weight", p + ".conv1.norm", "", 0, 1, 0);
  c.c2 = make_conv(m, p + ".conv2.conv.weight", p + ".conv2.norm", "", 0, 1, 0);
  std::vector<float> w3, b3, w1, b1;
  fold_conv(m, p + ".bottlenecks.0.conv1.conv.weight", p + ".bottlenecks.0.conv1.norm", "", w3, b3);
  fold_conv(m, p + ".bottlenecks.0.conv2.conv.weight", p + ".bottlenecks.0.conv2.norm", "", w1, b1);
  for (int co = 0; co < h; ++co) {                    // pad the 1x1 branch into the 3x3 centre tap
    for (int ci = 0; ci < h; ++ci) w3[((size_t)co * h + ci) * 9 + 4] += w1[(size_t)co * h + ci];
    b3[co] += b1[co];
  }
  c.rep = pack_conv(m, w3, b3, h, h, 3, 3, 0, 1, 1);
  c.has_c3 = h != 256;
  if (c.has_c3) c.c3 = make_conv(m, p + ".conv3.conv.weight", p + ".conv3.norm", "", 0, 1, 0);
  return c;
}

// ---- workspace plan
struct RtWs {
  size_t x0, bufA, bufB, t1, t2, sc, f0, f1, f2;
  size_t cat0, cat1, catp0, catp1, aqk, avt, aao, atmp, affn, aout;
  size_t x1, x2, y, inner1, p3, n4, n5;
  size_t mem, omem, elog, value;
  size_t topk, tgt, slog, sanc, refs, qh, qpos, hh1, hh2, dqk, dvt, dao, dtmp, t1d, t2d, soaw, dcr, dffn, hs, lgt;
  size_t total;
};

RtWs rt_plan(const spe_model* m, int B) {
  const RtModel& r = *m->rt;
  const auto& c = r.cfg;
  const size_t E = m->esz, S = c.input_size, Q = c.num_queries, L = r.L, BQ = (size_t)B * Q;
  const size_t s0 = r.lvl_s[0], s1 = r.lvl_s[1], s2 = r.lvl_s[2];
  const size_t exp = c.depth >= 50 ? 4 : 1;
  RtWs w{};
  size_t off = 0;
  auto take = [&](size_t bytes) { size_t o = off; off += (bytes + 255) & ~size_t(255); return o; };
  const size_t big = (size_t)B * S * S * 16 * E;     // stride 2 x 64 ch == stride 4 x 256 ch
  w.x0 = take((size_t)B * S * S * 8 * E);
  w.bufA = take(big); w.bufB = take(big); w.t1 = take(big); w.t2 = take(big); w.sc = take(big);
  w.f0 = take((size_t)B * s0 * s0 * 128 * exp * E);
  w.f1 = take((size_t)B * s1 * s1 * 256 * exp * E);
  w.f2 = take((size_t)B * s2 * s2 * 512 * exp * E);
  w.cat0 = take((size_t)B * s0 * s0 * 512 * E);
  w.cat1 = take((size_t)B * s1 * s1 * 512 * E);
  w.catp0 = take((size_t)B * s1 * s1 * 512 * E);
  w.catp1 = take((size_t)B * s2 * s2 * 512 * E);
  const size_t T2 = (size_t)B * s2 * s2;
  w.aqk = take(T2 * 512 * E); w.avt = take(T2 * 256 * E); w.aao = take(T2 * 256 * E); w.atmp = take(T2 * 256 * E);
  w.affn = take(T2 * c.enc_ff * E); w.aout = take(T2 * 256 * E);
  const size_t hmax = (size_t)B * s0 * s0 * c.csp_hidden * E;
  w.x1 = take(hmax); w.x2 = take(hmax); w.y = take(hmax);
  w.inner1 = take((size_t)B * s1 * s1 * 256 * E);
  w.p3 = take((size_t)B * s0 * s0 * 256 * E);
  w.n4 = take((size_t)B * s1 * s1 * 256 * E);
  w.n5 = take((size_t)B * s2 * s2 * 256 * E);
  w.mem = take((size_t)B * L * 256 * E);
  w.omem = take((size_t)B * L * 256 * E);
  w.elog = take((size_t)B * L * (c.num_classes + 1) * 4);
  w.value = take((size_t)B * L * 256 * c.dec_layers * E);
  w.topk = take(BQ * 4);
  w.tgt = take(BQ * 256 * E);
  w.hh1 = take(BQ * 512 * E); w.hh2 = take(BQ * 512 * E);
  w.slog = take(BQ * (c.num_classes + 1) * 4); w.sanc = take(BQ * 2 * 4);
  w.refs = take((size_t)(c.dec_layers + 1) * BQ * 2 * 4);
  w.qh = take(BQ * 512 * E); w.qpos = take(BQ * 256 * E);
  w.dqk = take(BQ * 512 * E); w.dvt = take(BQ * 256 * E); w.dao = take(BQ * 256 * E); w.dtmp = take(BQ * 256 * E);
  w.t1d = take(BQ * 256 * E); w.t2d = take(BQ * 256 * E);
  w.soaw = take(BQ * 288 * 4); w.dcr = take(BQ * 256 * E); w.dffn = take(BQ * c.dec_ff * E);
  w.hs = take(BQ * 256 * 4);
  w.lgt = take(BQ * (c.num_classes + 1) * 4);
  w.total = off;
  return w;
}

#define CK(x)                                                                         \
  do {                                                                                \
    int _r = (x);                                                                     \
    if (_r != 0) {                                                                    \
      char _b[256];                                                                   \
      snprintf(_b, sizeof _b, "%s failed (%d) at %s:%d", #x, _r, __FILE__, __LINE__);  \
      return fail(_r < 0 ? SPE_E_LAUNCH : _r, _b);                                    \
    }                                                                                 \
  } while (0)

}  // namespace

int spe_rtdetr_build_device(spe_model* m) {
  RtModel& r = *m->rt;
  const auto& c = r.cfg;
  const int d = 256;
  const std::string bb = "backbone.conv1.conv1_";
  r.stem[0] = make_conv(m, bb + "1.conv.weight", bb + "1.norm", "", 8, 2, 1);
  r.stem[1] = make_conv(m, bb + "2.conv.weight", bb + "2.norm", "", 0, 1, 1);
  r.stem[2] = make_conv(m, bb + "3.conv.weight", bb + "3.norm", "", 0, 1, 1);
  r.blocks.clear();
  const bool bott = c.depth >= 50;
  const int* nb = bott ? RESNET_CFG50 : RESNET_CFG18;
  const int widths[4] = {64, 128, 256, 512}, exp = bott ? 4 : 1;
  int cin = 64;
  for (int i = 0; i < 4; ++i) {
    r.stage_first[i] = (int)r.blocks.size();
    r.stage_n[i] = nb[i];
    for (int j = 0; j < nb[i]; ++j) {
      const std::string p = "backbone.res_layers." + std::to_string(i) + ".blocks." + std::to_string(j);
      RtBlock b;
      b.bottleneck = bott;
      b.stride = (j == 0 && i > 0) ? 2 : 1;
      b.cin = cin;
      b.cout = widths[i] * exp;
      if (bott) {
        b.a = make_conv(m, p + ".branch2a.conv.weight", p + ".branch2a.norm", "", 0, 1, 0);
        b.b = make_conv(m, p + ".branch2b.conv.weight", p + ".branch2b.norm", "", 0, b.stride, 1);
        b.c = make_conv(m, p + ".branch2c.conv.weight", p + ".branch2c.norm", "", 0, 1, 0);
      } else {
        b.a = make_conv(m, p + ".branch2a.conv.weight", p + ".branch2a.norm", "", 0, b.stride, 1);
        b.b = make_conv(m, p + ".branch2b.conv.weight", p + ".branch2b.norm", "", 0, 1, 1);
      }
      if (j == 0) {
        b.has_sc = true;
        if (b.stride == 2) {     // AvgPool2d(2, 2, ceil_mode) + ConvNormLayer(1x1) == 2x2/2 conv, w/4 per tap
          std::vector<float> w1, bias;
          fold_conv(m, p + ".short.conv.conv.weight", p + ".short.conv.norm", "", w1, bias);
          std::vector<float> w4((size_t)b.cout * cin * 4);
          for (size_t k = 0; k < (size_t)b.cout * cin; ++k)
            for (int t = 0; t < 4; ++t) w4[k * 4 + t] = w1[k] * 0.25f;
          b.sc = pack_conv(m, w4, bias, b.cout, cin, 2, 2, 0, 2, 0);
        } else {
          b.sc = make_conv(m, p + ".short.conv.weight", p + ".short.norm", "", 0, 1, 0);
        }
      }
      r.blocks.push_back(b);
      cin = b.cout;
    }
  }
  for (int l = 0; l < 3; ++l) {
    const std::string p = "encoder.input_proj." + std::to_string(l);
    r.in_proj[l] = make_conv(m, p + ".0.weight", p + ".1", "", 0, 1, 0);
  }
  const std::string a = "encoder.encoder.0.layers.0";
  r.aqk = make_linear(m, a + ".self_attn.in_proj_weight", a + ".self_attn.in_proj_bias", 0, 2 * d, d);
  r.av = make_linear(m, a + ".self_attn.in_proj_weight", a + ".self_attn.in_proj_bias", 2 * d, d, d);
  r.ao = make_linear(m, a + ".self_attn.out_proj.weight", a + ".self_attn.out_proj.bias", 0, d, d);
  r.al1 = make_linear(m, a + ".linear1.weight", a + ".linear1.bias", 0, c.enc_ff, d);
  r.al2 = make_linear(m, a + ".linear2.weight", a + ".linear2.bias", 0, d, c.enc_ff);
  r.an1g = upload_key(m, a + ".norm1.weight"); r.an1b = upload_key(m, a + ".norm1.bias");
  r.an2g = upload_key(m, a + ".norm2.weight"); r.an2b = upload_key(m, a + ".norm2.bias");
  r.aifi_pos = upload_T(m, sincos_2d(r.lvl_s[2], r.lvl_s[2], d));
  for (int i = 0; i < 2; ++i) {
    const std::string p = "encoder.lateral_convs." + std::to_string(i);
    r.lateral[i] = make_conv(m, p + ".conv.weight", p + ".norm", "", 0, 1, 0);
  }
  for (int i = 0; i < 2; ++i) {
    r.fpn[i] = make_csp(m, "encoder.fpn_blocks." + std::to_string(i), c.csp_hidden);
    r.pan[i] = make_csp(m, "encoder.pan_blocks." + std::to_string(i), c.csp_hidden);
  }
  for (int l = 0; l < 3; ++l) {
    const std::string p = "decoder.input_proj." + std::to_string(l);
    r.dec_in[l] = make_conv(m, p + ".conv.weight", p + ".norm", "", 0, 1, 0);
  }
  r.enc_out = make_linear(m, "decoder.enc_output.0.weight", "decoder.enc_output.0.bias", 0, d, d);
  r.eo_g = upload_key(m, "decoder.enc_output.1.weight");
  r.eo_b = upload_key(m, "decoder.enc_output.1.bias");
  r.enc_score = make_linear(m, "decoder.enc_score_head.weight", "decoder.enc_score_head.bias", 0, c.num_classes + 1, d);
  std::vector<std::pair<std::string, std::string>> vp;
  for (int i = 0; i < c.dec_layers; ++i) {
    const std::string p = "decoder.decoder.layers." + std::to_string(i) + ".cross_attn.value_proj";
    vp.emplace_back(p + ".weight", p + ".bias");
  }
  r.vproj = stack_linears(m, vp, d);
  const auto anc = make_anchors(r);
  r.anchors = upload_f32(m, anc.data(), anc.size());
  r.enc_head = make_head(m, "", "decoder.enc_bbox_head", "");
  r.qp_w0 = upload_key(m, "decoder.query_pos_head.layers.0.weight");
  r.qp_b0 = upload_key(m, "decoder.query_pos_head.layers.0.bias");
  r.qp_l1 = make_linear(m, "decoder.query_pos_head.layers.1.weight", "decoder.query_pos_head.layers.1.bias", 0, d, 2 * d);
  r.dec.clear();
  for (int i = 0; i < c.dec_layers; ++i) {
    const std::string p = "decoder.decoder.layers." + std::to_string(i), is = std::to_string(i);
    RtDec e;
    e.sqk = make_linear(m, p + ".self_attn.in_proj_weight", p + ".self_attn.in_proj_bias", 0, 2 * d, d);
    e.sv = make_linear(m, p + ".self_attn.in_proj_weight", p + ".self_attn.in_proj_bias", 2 * d, d, d);
    e.so = make_linear(m, p + ".self_attn.out_proj.weight", p + ".self_attn.out_proj.bias", 0, d, d);
    e.soaw = stack_linears(m, {{p + ".cross_attn.sampling_offsets.weight", p + ".cross_attn.sampling_offsets.bias"},
                               {p + ".cross_attn.attention_weights.weight", p + ".cross_attn.attention_weights.bias"}}, d);
    e.oproj = make_linear(m, p + ".cross_attn.output_proj.weight", p + ".cross_attn.output_proj.bias", 0, d, d);
    e.l1 = make_linear(m, p + ".linear1.weight", p + ".linear1.bias", 0, c.dec_ff, d);
    e.l2 = make_linear(m, p + ".linear2.weight", p + ".linear2.bias", 0, d, c.dec_ff);
    e.n1g = upload_key(m, p + ".norm1.weight"); e.n1b = upload_key(m, p + ".norm1.bias");
    e.n2g = upload_key(m, p + ".norm2.weight"); e.n2b = upload_key(m, p + ".norm2.bias");
    e.n3g = upload_key(m, p + ".norm3.weight"); e.n3b = upload_key(m, p + ".norm3.bias");
    e.head = make_head(m, "decoder.dec_score_head." + is, "decoder.dec_bbox_head." + is, "decoder.decoder.sigma_embed." + is);
    r.dec.push_back(e);
  }
  return 0;
}

int64_t spe_rtdetr_workspace(const spe_model* m, int B) { return (int64_t)rt_plan(m, B).total; }

extern "C" {

int spe_rtdetr_create(const spe_rtdetr_config* cfg, spe_model** out) {
  if (!cfg || !out) return fail(SPE_E_ARG, "null argument");
  if (cfg->depth != 18 && cfg->depth != 50) return fail(SPE_E_ARG, "PResNet depth must be 18 or 50");
  if (cfg->input_size % 32 || cfg->input_size < 64) return fail(SPE_E_ARG, "input_size must be a multiple of 32, >= 64");
  if (cfg->num_queries < 1 || cfg->num_queries > 64) return fail(SPE_E_ARG, "num_queries must be in [1, 64]");
  if (cfg->dec_layers < 1 || cfg->enc_ff % 64 || cfg->dec_ff % 64 || cfg->csp_hidden % 64 || cfg->csp_hidden < 64 ||
      cfg->csp_hidden > 256 || cfg->num_classes < 1 || cfg->num_classes > 15)
    return fail(SPE_E_ARG, "bad RT-DETR configuration");
  if (cfg->dtype != SPE_DTYPE_BF16_ && cfg->dtype != SPE_DTYPE_F32_) return fail(SPE_E_ARG, "bad dtype");
  spe_model* m = new spe_model();
  m->family = 1;
  m->rt = new RtModel();
  m->rt->cfg = *cfg;
  m->esz = cfg->dtype == SPE_DTYPE_BF16_ ? 2 : 4;
  m->cfg.dtype = cfg->dtype;
  m->cfg.input_size = cfg->input_size;
  m->cfg.num_queries = cfg->num_queries;
  m->spec = rt_spec(*cfg);
  RtModel& r = *m->rt;
  r.L = 0;
  for (int l = 0; l < 3; ++l) {
    r.lvl_s[l] = cfg->input_size >> (3 + l);
    r.lvl_start[l] = r.L;
    r.L += r.lvl_s[l] * r.lvl_s[l];
  }
  r.lvl_start[3] = r.L;
  if (cfg->num_queries > r.L) return (delete m->rt, delete m, fail(SPE_E_ARG, "num_queries exceeds the encoder tokens"));
  *out = m;
  return 0;
}

int spe_rtdetr_forward(spe_model* m, void* stream, const float* images, int B, void* workspace, int64_t ws_bytes,
                       const spe_rtdetr_outputs* out) {
  if (!m || !workspace || !images || B <= 0 || !out || !out->logits || !out->points) return fail(SPE_E_ARG, "bad argument");
  if (m->family != 1) return fail(SPE_E_ARG, "not an RT-DETR model");
  if (!m->finalized) return fail(SPE_E_STATE, "model not finalized");
  const RtWs w = rt_plan(m, B);
  if ((int64_t)w.total > ws_bytes) return fail(SPE_E_WORKSPACE, "workspace too small");
  hipStream_t s = (hipStream_t)stream;
  const RtModel& r = *m->rt;
  const auto& c = r.cfg;
  const int dt = c.dtype, S = c.input_size, d = 256, Q = c.num_queries, C = c.num_classes + 1, E = m->esz;
  const int BQ = B * Q, h = c.csp_hidden;
  char* ws = (char*)workspace;
  auto P = [&](size_t o) { return (void*)(ws + o); };
  auto ln = [&](const char* kind, const void* x, const float* g, const float* b, void* y, float* y32, int M) {
    return run_other(m, kind, 0.0, (double)M * d * 2 * E, s,
                     [&] { return spe_launch_layernorm(x, g, b, y, y32, M, d, dt, s); });
  };

  // conv as an implicit GEMM, or a plain GEMM over NHWC rows when it is 1x1 / stride 1; the
  // residual R (same row layout as the output) is added before the activation
  auto cgemm = [&](const char* kind, const Conv& cv, const void* in, int Hin, void* outp, int ldc, int act,
                   const void* R) {
    GemmArgs g;
    int mode = GEMM_CONV;
    if (cv.KH == 1 && cv.KW == 1 && cv.stride == 1 && cv.pad == 0) {
      g = linear_args(cv, in, cv.Cin, B * Hin * Hin, outp, ldc);
      mode = GEMM_LINEAR;
    } else {
      g = conv_args(cv, in, B, Hin, Hin, outp, ldc);
    }
    g.act = act;
    g.R = R; g.ldr = ldc;
    return run_gemm(m, kind, g, mode, s);
  };

  // ---------------- PResNet-vd (presnet.py:248-265)
  CK(run_other(m, "eltwise.pack", 0.0, (double)B * S * S * (12 + 8 * E), s,
               [&] { return spe_launch_pack_input(images, P(w.x0), B, S, dt, s); }));
  int H = S;
  size_t cur = w.x0;
  const size_t stem_out[3] = {w.bufA, w.bufB, w.bufA};
  for (int i = 0; i < 3; ++i) {
    GemmArgs g = conv_args(r.stem[i], P(cur), B, H, H, P(stem_out[i]), r.stem[i].N);
    g.act = ACT_RELU;
    CK(run_gemm(m, "rt.conv.stem", g, GEMM_CONV, s));
    H = g.Ho;
    cur = stem_out[i];
  }
  const int Hp = (H + 2 - 3) / 2 + 1;
  CK(run_other(m, "eltwise.maxpool", 0.0, (double)B * 64 * (H * H + Hp * Hp) * E, s,
               [&] { return spe_launch_maxpool3s2(P(cur), P(w.bufB), B, H, H, 64, Hp, Hp, dt, s); }));
  H = Hp;
  cur = w.bufB;
  const size_t feat[3] = {w.f0, w.f1, w.f2};
  for (int st = 0; st < 4; ++st)
    for (int j = 0; j < r.stage_n[st]; ++j) {
      const RtBlock& b = r.blocks[r.stage_first[st] + j];
      const int Ho = H / b.stride;
      const bool last = j == r.stage_n[st] - 1;
      const size_t outbuf = (last && st > 0) ? feat[st - 1] : (cur == w.bufA ? w.bufB : w.bufA);
      size_t res = cur;
      if (b.has_sc) {
        CK(cgemm(b.stride == 2 ? "rt.conv.short" : "rt.conv.1x1", b.sc, P(cur), H, P(w.sc), b.cout, ACT_NONE, nullptr));
        res = w.sc;
      }
      CK(cgemm(b.bottleneck ? "rt.conv.1x1" : "rt.conv.3x3", b.a, P(cur), H, P(w.t1), b.a.N, ACT_RELU, nullptr));
      const int Ha = (H + 2 * b.a.pad - b.a.KH) / b.a.stride + 1;
      if (b.bottleneck) {
        CK(cgemm("rt.conv.3x3", b.b, P(w.t1), Ha, P(w.t2), b.b.N, ACT_RELU, nullptr));
        CK(cgemm("rt.conv.1x1", b.c, P(w.t2), Ho, P(outbuf), b.cout, ACT_RELU, P(res)));
      } else {
        CK(cgemm("rt.conv.3x3", b.b, P(w.t1), Ha, P(outbuf), b.cout, ACT_RELU, P(res)));
      }
      H = Ho;
      cur = outbuf;
    }

  // ---------------- HybridEncoder (hybrid_encoder.py:332-401)
  const int s0 = r.lvl_s[0], s1 = r.lvl_s[1], s2 = r.lvl_s[2];
  const int fch[3] = {r.blocks[r.stage_first[1]].cout, r.blocks[r.stage_first[2]].cout, r.blocks[r.stage_first[3]].cout};
  {  // input_proj (1x1 + BN): levels 0 / 1 straight into the second half of their FPN concat
    GemmArgs g0 = linear_args(r.in_proj[0], P(w.f0), fch[0], B * s0 * s0, (char*)P(w.cat0) + d * E, 2 * d);
    CK(run_gemm(m, "rt.enc.proj", g0, GEMM_LINEAR, s));
    GemmArgs g1 = linear_args(r.in_proj[1], P(w.f1), fch[1], B * s1 * s1, (char*)P(w.cat1) + d * E, 2 * d);
    CK(run_gemm(m, "rt.enc.proj", g1, GEMM_LINEAR, s));
    GemmArgs g2 = linear_args(r.in_proj[2], P(w.f2), fch[2], B * s2 * s2, P(w.aout), d);
    CK(run_gemm(m, "rt.enc.proj", g2, GEMM_LINEAR, s));
  }
  {  // AIFI: one post-norm transformer encoder layer on the stride-32 level (GELU FFN)
    const int T = s2 * s2, M = B * T;
    GemmArgs gq = linear_args(r.aqk, P(w.aout), d, M, P(w.aqk), 2 * d);
    gq.P = r.aifi_pos; gq.ldp = d; gq.prow = T;
    CK(run_gemm(m, "rt.aifi.qk", gq, GEMM_LINEAR_ADD, s));
    GemmArgs gv = linear_args(r.av, P(w.aout), d, M, P(w.avt), 8);
    gv.vt_T = T; gv.vt_B = B;
    CK(run_gemm(m, "rt.aifi.v", gv, GEMM_LINEAR, s));
    AttnArgs at{};
    at.q = P(w.aqk); at.ldq = 2 * d;
    at.k = (char*)P(w.aqk) + d * E; at.ldk = 2 * d;
    at.vt = P(w.avt);
    at.o = P(w.aao); at.ldo = d;
    at.B = B; at.H = 8; at.Tq = T; at.Tk = T; at.scale = 1.0f / std::sqrt(32.0f);
    CK(run_attn(m, "rt.attn.aifi", at, dt, s));
    GemmArgs go = linear_args(r.ao, P(w.aao), d, M, P(w.atmp), d);
    go.R = P(w.aout); go.ldr = d;
    CK(run_gemm(m, "rt.aifi.o", go, GEMM_LINEAR, s));
    CK(ln("rt.ln", P(w.atmp), r.an1g, r.an1b, P(w.aout), nullptr, M));
    GemmArgs g1 = linear_args(r.al1, P(w.aout), d, M, P(w.affn), c.enc_ff);
    g1.act = ACT_GELU;
    CK(run_gemm(m, "rt.aifi.ffn", g1, GEMM_LINEAR, s));
    GemmArgs g2 = linear_args(r.al2, P(w.affn), c.enc_ff, M, P(w.atmp), d);
    g2.R = P(w.aout); g2.ldr = d;
    CK(run_gemm(m, "rt.aifi.ffn", g2, GEMM_LINEAR, s));
    CK(ln("rt.ln", P(w.atmp), r.an2g, r.an2b, P(w.aout), nullptr, M));
  }
  // CSPRepLayer over a [rows][512] concat: conv1 / conv2 (1x1 + BN + SiLU), RepVGG 3x3 + SiLU + x2,
  // conv3 (1x1 + BN + SiLU) when hidden != 256
  auto csp = [&](const RtCsp& k, size_t in, int hw, size_t outb) -> int {
    const int M = B * hw * hw;
    GemmArgs g1 = linear_args(k.c1, P(in), 2 * d, M, P(w.x1), h);
    g1.act = ACT_SILU;
    int rc = run_gemm(m, "rt.csp.1x1", g1, GEMM_LINEAR, s);
    if (rc) return rc;
    GemmArgs g2 = linear_args(k.c2, P(in), 2 * d, M, P(w.x2), h);
    g2.act = ACT_SILU;
    if ((rc = run_gemm(m, "rt.csp.1x1", g2, GEMM_LINEAR, s))) return rc;
    GemmArgs g3 = conv_args(k.rep, P(w.x1), B, hw, hw, k.has_c3 ? P(w.y) : P(outb), h);
    g3.act = ACT_SILU; g3.R = P(w.x2); g3.ldr = h; g3.res_post = 1;
    if ((rc = run_gemm(m, "rt.csp.rep", g3, GEMM_CONV, s))) return rc;
    if (k.has_c3) {
      GemmArgs g4 = linear_args(k.c3, P(w.y), h, M, P(outb), d);
      g4.act = ACT_SILU;
      rc = run_gemm(m, "rt.csp.1x1", g4, GEMM_LINEAR, s);
    }
    return rc;
  };
  auto resample = [&](size_t in, int ldi, size_t outp, int hw, int mode) {
    return run_other(m, "rt.resample", 0.0, (double)B * hw * hw * d * E * (mode == 0 ? 5 : 1.25), s,
                     [&] { return spe_launch_resample2x(P(in), ldi, P(outp), 2 * d, B, hw, hw, d, mode, dt, s); });
  };
  {  // top-down FPN; each lateral output also lands in the second half of its PAN concat
    GemmArgs l0 = linear_args(r.lateral[0], P(w.aout), d, B * s2 * s2, (char*)P(w.catp1) + d * E, 2 * d);
    l0.act = ACT_SILU;
    CK(run_gemm(m, "rt.enc.lateral", l0, GEMM_LINEAR, s));
    CK(resample(w.catp1 + d * E, 2 * d, w.cat1, s2, 0));
    CK(csp(r.fpn[0], w.cat1, s1, w.inner1));
    GemmArgs l1 = linear_args(r.lateral[1], P(w.inner1), d, B * s1 * s1, (char*)P(w.catp0) + d * E, 2 * d);
    l1.act = ACT_SILU;
    CK(run_gemm(m, "rt.enc.lateral", l1, GEMM_LINEAR, s));
    CK(resample(w.catp0 + d * E, 2 * d, w.cat0, s1, 0));
    CK(csp(r.fpn[1], w.cat0, s0, w.p3));
  }
  {  // bottom-up PAN (bicubic x0.5)
    CK(run_other(m, "rt.resample", 0.0, (double)B * s0 * s0 * d * E * 1.25, s,
                 [&] { return spe_launch_resample2x(P(w.p3), d, P(w.catp0), 2 * d, B, s0, s0, d, 1, dt, s); }));
    CK(csp(r.pan[0], w.catp0, s1, w.n4));
    CK(run_other(m, "rt.resample", 0.0, (double)B * s1 * s1 * d * E * 1.25, s,
                 [&] { return spe_launch_resample2x(P(w.n4), d, P(w.catp1), 2 * d, B, s1, s1, d, 1, dt, s); }));
    CK(csp(r.pan[1], w.catp1, s2, w.n5));
  }

  // ---------------- RTDETRTransformer (rtdetr_decoder.py:505-710)
  const size_t lvl_out[3] = {w.p3, w.n4, w.n5};
  for (int l = 0; l < 3; ++l) {   // level-major memory: rows [B * lvl_start[l] + b * hw_l + t]
    GemmArgs g = linear_args(r.dec_in[l], P(lvl_out[l]), d, B * r.lvl_s[l] * r.lvl_s[l],
                             (char*)P(w.mem) + (size_t)B * r.lvl_start[l] * d * E, d);
    CK(run_gemm(m, "rt.dec.proj", g, GEMM_LINEAR, s));
  }
  const int ML = B * r.L;
  {  // enc_output: Linear + LayerNorm
    GemmArgs g = linear_args(r.enc_out, P(w.mem), d, ML, P(w.omem), d);
    GemmArgs gf = g;
    gf.ln_g = r.eo_g; gf.ln_b = r.eo_b;
    if (E == 2 && spe_ln_fusable(gf)) {
      CK(run_gemm(m, "rt.dec.enc_out", gf, GEMM_LINEAR, s));
    } else {
      CK(run_gemm(m, "rt.dec.enc_out", g, GEMM_LINEAR, s));
      CK(ln("rt.ln", P(w.omem), r.eo_g, r.eo_b, P(w.omem), nullptr, ML));
    }
  }
  {
    GemmArgs g = linear_args(r.enc_score, P(w.omem), d, ML, P(w.elog), C);
    g.out_f32 = 1;
    CK(run_gemm(m, "rt.dec.enc_score", g, GEMM_LINEAR, s));
  }
  {  // every layer's value projection of the memory in one GEMM
    GemmArgs g = linear_args(r.vproj, P(w.mem), d, ML, P(w.value), r.vproj.N);
    CK(run_gemm(m, "rt.dec.value", g, GEMM_LINEAR, s));
  }
  RtSelectArgs sa{};
  sa.logits = (const float*)P(w.elog); sa.C = C;
  sa.memory = P(w.omem); sa.ldm = d;
  sa.anchors = r.anchors;
  sa.B = B; sa.Q = Q; sa.D = d; sa.levels = 3;
  for (int l = 0; l < 4; ++l) sa.lvl_start[l] = r.lvl_start[l];
  sa.topk = out->topk ? out->topk : (int*)P(w.topk);
  sa.target = P(w.tgt); sa.ldt = d;
  sa.sel_logits = out->enc_logits ? out->enc_logits : (float*)P(w.slog);
  sa.sel_anchors = (float*)P(w.sanc);
  CK(run_other(m, "rt.select", 0.0, (double)ML * C * 4, s, [&] { return spe_launch_query_select(sa, dt, s); }));
  // heads: the 256-wide hidden layers as GEMMs (box | sigma side by side), then head_finish
  auto heads = [&](const RtHead& k, const void* x, const float* hs32, RtHeadArgs ha) -> int {
    GemmArgs g1 = linear_args(k.h1, x, d, BQ, P(w.hh1), 2 * d);
    g1.act = ACT_RELU;
    int rc = run_gemm(m, "rt.heads", g1, GEMM_LINEAR, s);
    if (rc) return rc;
    GemmArgs g2 = linear_args(k.box1, P(w.hh1), 2 * d, BQ, P(w.hh2), 2 * d);
    g2.act = ACT_RELU;
    if ((rc = run_gemm(m, "rt.heads", g2, GEMM_LINEAR, s))) return rc;
    if (k.sig_w2) {
      GemmArgs g3 = linear_args(k.sig1, (char*)P(w.hh1) + d * E, 2 * d, BQ, (char*)P(w.hh2) + d * E, 2 * d);
      g3.act = ACT_RELU;
      if ((rc = run_gemm(m, "rt.heads", g3, GEMM_LINEAR, s))) return rc;
    }
    ha.rows = BQ; ha.Q = Q; ha.C = C;
    ha.hs = hs32; ha.cls_w = k.cls_w; ha.cls_b = k.cls_b;
    ha.h2 = P(w.hh2); ha.ld_h2 = 2 * d;
    ha.box_w2 = k.box_w2; ha.box_b2 = k.box_b2; ha.sig_w2 = k.sig_w2; ha.sig_b2 = k.sig_b2;
    return run_other(m, "rt.heads", 0.0, (double)BQ * d * 4, s, [&] { return spe_launch_head_finish(ha, dt, s); });
  };
  float* refs = (float*)P(w.refs);
  auto ref_buf = [&](int i) { return refs + (size_t)i * BQ * 2; };
  {  // initial reference points: sigmoid(enc_bbox_head(target) + anchors) (= enc_topk_bboxes)
    RtHeadArgs ha{};
    ha.pt_add = sa.sel_anchors; ha.pt_add_invsig = 0;
    ha.points = out->enc_points ? out->enc_points : ref_buf(0);
    CK(heads(r.enc_head, P(w.tgt), nullptr, ha));
    if (out->enc_points)
      CK((int)hipMemcpyAsync(ref_buf(0), out->enc_points, (size_t)BQ * 2 * 4, hipMemcpyDeviceToDevice, s));
  }
  size_t tgt = w.tgt;
  for (int i = 0; i < c.dec_layers; ++i) {
    const RtDec& e = r.dec[i];
    const bool last = i == c.dec_layers - 1;
    const float* ref = ref_buf(i);
    // query_pos_head(ref): relu(W0 ref + b0) (K = 2) -> Linear(512 -> 256)
    CK(run_other(m, "rt.qpos", 0.0, (double)BQ * 512 * E, s,
                 [&] { return spe_launch_qpos_hidden(ref, r.qp_w0, r.qp_b0, P(w.qh), BQ, 2 * d, dt, s); }));
    GemmArgs gp = linear_args(r.qp_l1, P(w.qh), 2 * d, BQ, P(w.qpos), d);
    CK(run_gemm(m, "rt.gemm.dec", gp, GEMM_LINEAR, s));
    // self-attention: q = k = tgt + qpos, v = tgt
    GemmArgs gq = linear_args(e.sqk, P(tgt), d, BQ, P(w.dqk), 2 * d);
    gq.P = P(w.qpos); gq.ldp = d; gq.prow = BQ;
    CK(run_gemm(m, "rt.gemm.dec", gq, GEMM_LINEAR_ADD, s));
    GemmArgs gv = linear_args(e.sv, P(tgt), d, BQ, P(w.dvt), 8);
    gv.vt_T = Q; gv.vt_B = B;
    CK(run_gemm(m, "rt.gemm.dec", gv, GEMM_LINEAR, s));
    AttnArgs at{};
    at.q = P(w.dqk); at.ldq = 2 * d;
    at.k = (char*)P(w.dqk) + d * E; at.ldk = 2 * d;
    at.vt = P(w.dvt);
    at.o = P(w.dao); at.ldo = d;
    at.B = B; at.H = 8; at.Tq = Q; at.Tk = Q; at.scale = 1.0f / std::sqrt(32.0f);
    CK(run_attn(m, "rt.attn.dec_self", at, dt, s));
    GemmArgs go = linear_args(e.so, P(w.dao), d, BQ, P(w.dtmp), d);
    go.R = P(tgt); go.ldr = d;
    CK(run_gemm(m, "rt.gemm.dec", go, GEMM_LINEAR, s));
    CK(ln("rt.ln", P(w.dtmp), e.n1g, e.n1b, P(w.t1d), nullptr, BQ));
    // multi-scale deformable cross-attention, query = tgt + qpos
    GemmArgs gs = linear_args(e.soaw, P(w.t1d), d, BQ, P(w.soaw), e.soaw.N);
    gs.P = P(w.qpos); gs.ldp = d; gs.prow = BQ; gs.out_f32 = 1;
    CK(run_gemm(m, "rt.gemm.dec", gs, GEMM_LINEAR_ADD, s));
    RtDeformArgs da{};
    da.value = (const char*)P(w.value) + (size_t)i * d * E; da.ldv = r.vproj.N;
    da.so_aw = (const float*)P(w.soaw); da.ld_so = e.soaw.N;
    da.ref = ref;
    da.out = P(w.dcr); da.ldo = d;
    da.rows = BQ; da.Q = Q; da.heads = 8; da.levels = 3; da.points = 4;
    for (int l = 0; l < 3; ++l) {
      da.lvl_h[l] = da.lvl_w[l] = r.lvl_s[l];
      da.lvl_rows0[l] = B * r.lvl_start[l];
    }
    CK(run_other(m, "rt.msdeform", 0.0, (double)BQ * 96 * 4 * 32 * E, s, [&] { return spe_launch_msdeform(da, dt, s); }));
    GemmArgs gc = linear_args(e.oproj, P(w.dcr), d, BQ, P(w.dtmp), d);
    gc.R = P(w.t1d); gc.ldr = d;
    CK(run_gemm(m, "rt.gemm.dec", gc, GEMM_LINEAR, s));
    CK(ln("rt.ln", P(w.dtmp), e.n2g, e.n2b, P(w.t2d), nullptr, BQ));
    // FFN (ReLU) + norm3
    GemmArgs g1 = linear_args(e.l1, P(w.t2d), d, BQ, P(w.dffn), c.dec_ff);
    g1.act = ACT_RELU;
    CK(run_gemm(m, "rt.gemm.dec", g1, GEMM_LINEAR, s));
    GemmArgs g2 = linear_args(e.l2, P(w.dffn), c.dec_ff, BQ, P(w.dtmp), d);
    g2.R = P(w.t2d); g2.ldr = d;
    CK(run_gemm(m, "rt.gemm.dec", g2, GEMM_LINEAR, s));
    tgt = (tgt == w.tgt) ? w.t1d : w.tgt;          // t1d is free again once the FFN residual is read
    CK(ln("rt.ln", P(w.dtmp), e.n3g, e.n3b, P(tgt), (float*)P(w.hs), BQ));
    // heads: score, refined points sigmoid(box MLP + inverse_sigmoid(ref)), sigma (+ PostProcess)
    RtHeadArgs ha{};
    ha.pt_add = ref; ha.pt_add_invsig = 1;
    const size_t aoff = (size_t)i * BQ;
    if (last) {
      ha.logits = out->logits; ha.points = out->points;
      ha.log_sigmas = out->log_sigmas;
      ha.clip_bbox = out->clip_bbox;
      ha.probs = out->clip_bbox ? out->probs : nullptr;
      ha.points_px = out->clip_bbox ? out->points_px : nullptr;
      ha.sigmas = out->clip_bbox ? out->sigmas : nullptr;
    } else {
      ha.logits = out->aux_logits ? out->aux_logits + aoff * C : (float*)P(w.lgt);
      ha.points = ref_buf(i + 1);
      ha.log_sigmas = out->aux_log_sigmas ? out->aux_log_sigmas + aoff * 2 : nullptr;
    }
    CK(heads(e.head, P(tgt), (const float*)P(w.hs), ha));
    if (last && out->hs)
      CK((int)hipMemcpyAsync(out->hs, P(w.hs), (size_t)BQ * 256 * 4, hipMemcpyDeviceToDevice, s));
    if (!last && out->aux_points)
      CK((int)hipMemcpyAsync(out->aux_points + aoff * 2, ref_buf(i + 1), (size_t)BQ * 2 * 4, hipMemcpyDeviceToDevice, s));
  }
  return 0;
}

}  // extern "C"
