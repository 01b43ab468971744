// Batched pose solver + SPEED score on gfx950: one 64-lane wave per image.
//
// Replaces the per-image host loop SpeedEval.update -> SimplePoseSolver.__call__
// (REV/datasets/speed.py:351-363, REV/utils/speed_eval.py:164-242) and its sigma variant
// (UNC/utils/speed_eval.py:332-420):
//   selection      lane-parallel argmax over the 12 class probabilities, then first-seen label
//                  order / best score per label (REV/utils/speed_eval.py:184-206)
//   RANSAC         OpenCV 4.4 RANSACPointSetRegistrator semantics made parallel without changing
//                  results: the cv::RNG(-1) subset stream is drawn serially (lane 0) for the
//                  maximum iteration budget, every hypothesis (P3P on 4 / EPnP on 5 points) and
//                  its float32 inlier count is evaluated lane-parallel, then the adaptive
//                  iteration count / best-model update is replayed in order — identical to the
//                  serial loop because a hypothesis never depends on earlier ones.
//   refit + refine EPnP on the consensus set (12x12 MtM eigen-decomposition, Gauss-Newton
//                  betas), then CvLevMarq (<= 20 iters) for the REV path or the sigma-weighted
//                  Huber LM for the UNC path; Rodrigues; Blender mat3_to_quat (float32).
// Status codes follow the reference's exception mapping (REV/datasets/speed.py:355-363).
#include "spe_common.h"
#include "pnp_math.h"
#include "spe_pnp.h"

namespace {

constexpr int WAVE = 64;
constexpr int MAXIT = 256;

__global__ __launch_bounds__(WAVE) void pnp_kernel(PnpArgs a) {
  const int b = blockIdx.x;
  const int lane = threadIdx.x;
  __shared__ int s_lab[WAVE];
  __shared__ float s_score[WAVE];
  __shared__ int s_nl, s_order[MAXN], s_bestq[MAXN];
  __shared__ float s_img[2 * MAXN], s_wld[3 * MAXN], s_sig[2 * MAXN];
  __shared__ unsigned char s_idx[MAXIT][5];
  __shared__ int s_ok[MAXIT], s_good[MAXIT];
  __shared__ uint32_t s_mask[MAXIT];
  __shared__ double s_rt[MAXIT][6];

  const cam_t k = {a.K[0], a.K[4], a.K[2], a.K[5]};
  const int Q = a.Q, C = a.C;

  // ---- correspondence selection
  for (int q = lane; q < Q; q += WAVE) {
    const float* p = a.probs + ((size_t)b * Q + q) * C;
    int lab = 0;
    float sc = p[0];
    for (int c = 1; c < C; ++c)
      if (p[c] > sc) { sc = p[c]; lab = c; }
    if (q < WAVE) { s_lab[q] = lab; s_score[q] = sc; }
  }
  __syncthreads();
  if (lane == 0) {
    int nl = 0;
    float best_s[MAXN];
    for (int q = 0; q < Q && q < WAVE; ++q) {
      const int lab = s_lab[q];
      if (lab == C - 1) continue;
      int j;
      for (j = 0; j < nl; ++j) if (s_order[j] == lab) break;
      if (j == nl) { if (nl < MAXN) { s_order[nl] = lab; s_bestq[nl] = q; best_s[nl] = s_score[q]; nl++; } }
      else if (s_score[q] > best_s[j]) { s_bestq[j] = q; best_s[j] = s_score[q]; }
    }
    s_nl = nl;
    for (int j = 0; j < nl; ++j) {
      const int q = s_bestq[j];
      s_img[2 * j] = a.points[((size_t)b * Q + q) * 2];
      s_img[2 * j + 1] = a.points[((size_t)b * Q + q) * 2 + 1];
      for (int c = 0; c < 3; ++c) s_wld[3 * j + c] = (float)a.world[3 * s_order[j] + c];
      s_sig[2 * j] = a.sigmas ? a.sigmas[((size_t)b * Q + q) * 2] : 1.f;
      s_sig[2 * j + 1] = a.sigmas ? a.sigmas[((size_t)b * Q + q) * 2 + 1] : 1.f;
    }
  }
  __syncthreads();
  const int nl = s_nl;

  double rvec[3] = {0, 0, 0}, t[3] = {0, 0, 0};
  int status = SPE_PNP_OK;
  uint32_t inl = 0;
  bool have_pose = false;

  if (nl == 0) {
    status = SPE_PNP_NO_FG;
  } else if (nl < 4) {
    status = SPE_PNP_CV_ERROR;
  } else if (a.mode == SPE_PNP_EPNP || a.mode == SPE_PNP_EPNP_LM) {
    if (lane == 0) {
      double wd[3 * MAXN], id[2 * MAXN];
      for (int i = 0; i < 3 * nl; ++i) wd[i] = s_wld[i];
      for (int i = 0; i < 2 * nl; ++i) id[i] = s_img[i];
      epnp_solve(&k, nl, wd, id, 1, rvec, t);
      if (a.mode == SPE_PNP_EPNP_LM) lm_refine(&k, nl, wd, id, rvec, t);
      inl = (nl >= 32) ? 0xffffffffu : ((1u << nl) - 1);
      have_pose = true;
    }
  } else {
    const int kernel = (a.mode == SPE_PNP_RANSAC_P3P_LM || nl == 4) ? 0 : 1;
    const int mp = kernel == 0 ? 4 : 5;
    bool ok = false;
    if (nl == mp) {
      // model_points == npoints: direct solve on all points (solvepnp.cpp)
      if (lane == 0) {
        if (kernel == 0) {
          ok = p3p_solve4(&k, s_img, s_wld, rvec, t) != 0;
        } else {
          double wd[15], id[10];
          for (int i = 0; i < 15; ++i) wd[i] = s_wld[i];
          for (int i = 0; i < 10; ++i) id[i] = s_img[i];
          epnp_solve(&k, 5, wd, id, 1, rvec, t);
          ok = true;
        }
        s_ok[0] = ok;
        s_mask[0] = (1u << nl) - 1;
      }
      __syncthreads();
      ok = s_ok[0];
      if (!ok) status = SPE_PNP_UNPINNED;
      inl = s_mask[0];
    } else {
      const int iters = a.ransac_iters < MAXIT ? a.ransac_iters : MAXIT;
      // 1. subset stream of cv::RNG((uint64)-1), drawn in order
      if (lane == 0) {
        rng_t rng = {(uint64_t)-1};
        for (int it = 0; it < iters; ++it) {
          int idx[5];
          for (int i = 0; i < mp; ++i) {
            for (;;) {
              int v = rng_uniform(&rng, 0, nl), j;
              idx[i] = v;
              for (j = 0; j < i; ++j) if (v == idx[j]) break;
              if (j == i) break;
            }
            s_idx[it][i] = (unsigned char)idx[i];
          }
        }
      }
      __syncthreads();
      // 2. hypotheses + float32 inlier sets, lane-parallel
      const float thr2 = (float)((double)a.repro * (double)a.repro);
      for (int it = lane; it < iters; it += WAVE) {
        float si[10], sw[15];
        for (int i = 0; i < mp; ++i) {
          const int j = s_idx[it][i];
          si[2 * i] = s_img[2 * j]; si[2 * i + 1] = s_img[2 * j + 1];
          for (int c = 0; c < 3; ++c) sw[3 * i + c] = s_wld[3 * j + c];
        }
        double r[3], tt[3];
        int okh;
        if (kernel == 0) {
          okh = p3p_solve4(&k, si, sw, r, tt);
        } else {
          double wd[15], id[10];
          for (int i = 0; i < 15; ++i) wd[i] = sw[i];
          for (int i = 0; i < 10; ++i) id[i] = si[i];
          epnp_solve(&k, 5, wd, id, 1, r, tt);
          okh = 1;
        }
        int good = 0;
        uint32_t m = 0;
        if (okh) {
          double R[9];
          rodrigues_r2R(r, R);
          for (int i = 0; i < nl; ++i) {
            float uv[2];
            project_f(&k, R, tt, s_wld + 3 * i, uv);
            if (sq_err_f(s_img + 2 * i, uv) <= thr2) { m |= 1u << i; good++; }
          }
        }
        s_ok[it] = okh;
        s_good[it] = good;
        s_mask[it] = m;
        for (int c = 0; c < 3; ++c) { s_rt[it][c] = r[c]; s_rt[it][3 + c] = tt[c]; }
      }
      __syncthreads();
      // 3. serial replay of the adaptive loop; refit + refine on lane 0
      if (lane == 0) {
        int niters = iters > 1 ? iters : 1, maxGood = 0, best = -1, last = -1;
        for (int it = 0; it < niters; ++it) {
          if (!s_ok[it]) continue;
          last = it;
          if (s_good[it] > (maxGood > mp - 1 ? maxGood : mp - 1)) {
            best = it;
            maxGood = s_good[it];
            niters = (int)ransac_update(a.confidence, (double)(nl - maxGood) / nl, mp, niters);
          }
        }
        if (maxGood > 0) {
          inl = s_mask[best];
          double wd[3 * MAXN], id[2 * MAXN];
          int m = 0;
          for (int i = 0; i < nl; ++i)
            if (inl & (1u << i)) {
              for (int c = 0; c < 3; ++c) wd[3 * m + c] = s_wld[3 * i + c];
              id[2 * m] = s_img[2 * i]; id[2 * m + 1] = s_img[2 * i + 1];
              m++;
            }
          epnp_solve(&k, m, wd, id, 0, rvec, t);
          s_ok[0] = 1;
        } else if (last >= 0) {
          for (int c = 0; c < 3; ++c) { rvec[c] = s_rt[last][c]; t[c] = s_rt[last][3 + c]; }
          s_ok[0] = 2;
        } else {
          s_ok[0] = 0;
        }
        s_mask[0] = inl;
      }
      __syncthreads();
      ok = s_ok[0] == 1;
      if (s_ok[0] == 2) status = SPE_PNP_RANSAC_FALLBACK;
      if (s_ok[0] == 0) status = SPE_PNP_UNPINNED;
      inl = s_mask[0];
    }
    if (ok && lane == 0) {
      double wi[3 * MAXN], ii[2 * MAXN], sg[2 * MAXN];
      int m = 0;
      for (int i = 0; i < nl; ++i)
        if (inl & (1u << i)) {
          for (int c = 0; c < 3; ++c) wi[3 * m + c] = s_wld[3 * i + c];
          for (int c = 0; c < 2; ++c) { ii[2 * m + c] = s_img[2 * i + c]; sg[2 * m + c] = s_sig[2 * i + c]; }
          m++;
        }
      if (a.mode == SPE_PNP_RANSAC_P3P_LM) lm_refine(&k, m, wi, ii, rvec, t);
      else sigma_lm(&k, m, wi, ii, sg, 0.005, rvec, t);
    }
    have_pose = status == SPE_PNP_OK || status == SPE_PNP_RANSAC_FALLBACK;
  }

  if (lane != 0) return;
  float qf[4] = {0.f, 0.f, 0.f, 0.f};
  if (have_pose) {
    double R[9];
    rodrigues_r2R(rvec, R);
    blender_quat(R, qf);
  } else {
    t[0] = t[1] = t[2] = 0;
  }
  for (int i = 0; i < 4; ++i) a.quat[4 * b + i] = qf[i];
  for (int i = 0; i < 3; ++i) a.tvec[3 * b + i] = t[i];
  if (a.rvec) for (int i = 0; i < 3; ++i) a.rvec[3 * b + i] = have_pose ? rvec[i] : 0.0;
  if (a.status) a.status[b] = status;
  if (a.n_corr) a.n_corr[b] = nl;
  if (a.inlier_mask) a.inlier_mask[b] = inl;
  if (a.corr_label) for (int j = 0; j < MAXN; ++j) a.corr_label[MAXN * b + j] = j < nl ? s_order[j] : -1;
}

// SPEED score (REV/utils/speed_eval.py:245-262): q sign-normalised, s_t = |dt|/|t_gt|,
// s_q = 2 acos(min(|q.q_gt|, 1)); failures arrive as zero poses (REV/datasets/speed.py:355-363).
__global__ void score_kernel(const float* __restrict__ quat, const double* __restrict__ tvec,
                             const double* __restrict__ q_gt, const double* __restrict__ t_gt, int B,
                             double* __restrict__ s_t, double* __restrict__ s_q) {
  const int b = blockIdx.x * blockDim.x + threadIdx.x;
  if (b >= B) return;
  double qp[4], qg[4];
  const double sp = quat[4 * b] < 0 ? -1 : 1, sg = q_gt[4 * b] < 0 ? -1 : 1;
  for (int i = 0; i < 4; ++i) { qp[i] = (double)quat[4 * b + i] * sp; qg[i] = q_gt[4 * b + i] * sg; }
  double dn = 0, gn = 0;
  for (int i = 0; i < 3; ++i) {
    const double d = tvec[3 * b + i] - t_gt[3 * b + i];
    dn += d * d;
    gn += t_gt[3 * b + i] * t_gt[3 * b + i];
  }
  s_t[b] = sqrt(dn) / sqrt(gn);
  const double d = fabs(qp[0] * qg[0] + qp[1] * qg[1] + qp[2] * qg[2] + qp[3] * qg[3]);
  s_q[b] = 2 * acos(d < 1 ? d : 1);
}

}  // namespace

int spe_launch_pnp(const PnpArgs& a, hipStream_t s) {
  if (a.B <= 0) return 0;
  if (a.Q > WAVE || a.C < 2 || a.C - 1 > MAXN) return -7;
  hipLaunchKernelGGL(pnp_kernel, dim3(a.B), dim3(WAVE), 0, s, a);
  return (int)hipGetLastError();
}

int spe_launch_score(const float* quat, const double* tvec, const double* q_gt, const double* t_gt, int B, double* s_t,
                     double* s_q, hipStream_t s) {
  if (B <= 0) return 0;
  hipLaunchKernelGGL(score_kernel, dim3((B + 127) / 128), dim3(128), 0, s, quat, tvec, q_gt, t_gt, B, s_t, s_q);
  return (int)hipGetLastError();
}
