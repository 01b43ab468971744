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
//   EPnP           wave-cooperative: M^T M entries across lanes, the 12x12 eigen-decomposition
//                  as a round-parallel Jacobi (6 disjoint rotations per round, column pass then
//                  row pass through LDS), betas / Gauss-Newton / pose on lane 0
//   refine         CvLevMarq (<= 20 iters) for the REV path or the sigma-weighted Huber LM for
//                  the UNC path; Rodrigues; Blender mat3_to_quat (float32).
// Status codes follow the reference's exception mapping (REV/datasets/speed.py:355-363).
// Compiled with -ffp-contract=off: together with pnp_math.h's deterministic transcendentals the
// index outputs (correspondences, inlier sets) match oracle/pnp_ref.c bit for bit.
#include "spe_common.h"
#include "pnp_math.h"
#include "spe_pnp.h"

namespace {

constexpr int WAVE = 64;
constexpr int MAXIT = 256;

struct EpnpShared {
  epnp_t e;
  double a[144], v[144], tmp[144], ut[144];
  double L[60], rho[6], err[4], Rs[4][9], ts[4][3];
  double c[6], s[6];
  int P[6], Q[6], pair_of[12], is_p[12];
  int stop;
};

// Round-parallel Jacobi on sh.a (12x12, LDS) with eigenvectors in sh.v: the same IEEE operation
// sequence as jacobi12_rr() (pnp_math.h / oracle), with the 144 element updates spread over lanes.
__device__ void jacobi12_rr_wave(EpnpShared& sh, int lane) {
  for (int e = lane; e < 144; e += WAVE) sh.v[e] = (e / 12 == e % 12) ? 1.0 : 0.0;
  __syncthreads();
  for (int sweep = 0; sweep < 60; ++sweep) {
    if (lane == 0) {
      double off = 0, diag = 0;
      for (int i = 0; i < 12; ++i) {
        diag += sh.a[i * 12 + i] * sh.a[i * 12 + i];
        for (int j = i + 1; j < 12; ++j) off += sh.a[i * 12 + j] * sh.a[i * 12 + j];
      }
      sh.stop = (off <= 1e-30 * diag || off == 0);
    }
    __syncthreads();
    if (sh.stop) break;
    for (int r = 0; r < 11; ++r) {
      if (lane < 6) {
        int P[6], Q[6];
        rr_pairs(r, P, Q);
        const int p = P[lane], q = Q[lane];
        double c, s;
        jacobi_cs(sh.a[p * 12 + p], sh.a[q * 12 + q], sh.a[p * 12 + q], &c, &s);
        sh.c[lane] = c; sh.s[lane] = s; sh.P[lane] = p; sh.Q[lane] = q;
        sh.pair_of[p] = lane; sh.pair_of[q] = lane;
        sh.is_p[p] = 1; sh.is_p[q] = 0;
      }
      __syncthreads();
      double vnew[3];
#pragma unroll
      for (int t = 0; t < 3; ++t) {
        const int e = lane + WAVE * t;
        if (e < 144) {
          const int i = e / 12, j = e % 12, kk = sh.pair_of[j];
          const double c = sh.c[kk], s = sh.s[kk];
          const double x = sh.a[i * 12 + sh.P[kk]], y = sh.a[i * 12 + sh.Q[kk]];
          sh.tmp[e] = sh.is_p[j] ? c * x - s * y : s * x + c * y;
          const double vx = sh.v[i * 12 + sh.P[kk]], vy = sh.v[i * 12 + sh.Q[kk]];
          vnew[t] = sh.is_p[j] ? c * vx - s * vy : s * vx + c * vy;
        }
      }
      __syncthreads();
#pragma unroll
      for (int t = 0; t < 3; ++t) {
        const int e = lane + WAVE * t;
        if (e < 144) {
          const int i = e / 12, j = e % 12, kk = sh.pair_of[i];
          const double c = sh.c[kk], s = sh.s[kk];
          const double x = sh.tmp[sh.P[kk] * 12 + j], y = sh.tmp[sh.Q[kk] * 12 + j];
          sh.a[e] = sh.is_p[i] ? c * x - s * y : s * x + c * y;
          sh.v[e] = vnew[t];
        }
      }
      __syncthreads();
    }
  }
}

// solvePnPGeneric(EPNP) on the correspondences selected by `mask` (all lanes call; the pose is
// valid on lane 0).  img_is_float: round the undistorted coordinates to float32 (OpenCV keeps
// the input depth: float inputs on the direct path, double on the RANSAC refit).
__device__ void epnp_solve_wave(EpnpShared& sh, const cam_t* k, const float* img_f, const float* wld_f, int nl,
                                uint32_t mask, int img_is_float, double* rvec, double* tvec, int lane) {
  if (lane == 0) {
    double wd[3 * MAXN], nrm[2 * MAXN];
    int m = 0;
    for (int i = 0; i < nl; ++i)
      if (mask & (1u << i)) {
        for (int c = 0; c < 3; ++c) wd[3 * m + c] = wld_f[3 * i + c];
        double un = ((double)img_f[2 * i] - k->cx) * (1. / k->fx);
        double vn = ((double)img_f[2 * i + 1] - k->cy) * (1. / k->fy);
        if (img_is_float) { un = (float)un; vn = (float)vn; }
        nrm[2 * m] = un; nrm[2 * m + 1] = vn;
        m++;
      }
    epnp_setup(&sh.e, k, m, wd, nrm);
  }
  __syncthreads();
  for (int e = lane; e < 144; e += WAVE) sh.a[e] = epnp_mtm_entry(&sh.e, e / 12, e % 12);
  __syncthreads();
  jacobi12_rr_wave(sh, lane);
  if (lane == 0) {
    double ev[12], w[12];
    for (int i = 0; i < 12; ++i) ev[i] = sh.a[i * 12 + i];
    eig_sort_desc(12, ev, sh.v, w, sh.ut);
    epnp_L_rho(&sh.e, sh.ut, sh.L, sh.rho);
  }
  __syncthreads();
  if (lane >= 1 && lane <= 3)   // the three beta approximations (epnp_finish) on three lanes
    sh.err[lane] = epnp_approx(&sh.e, sh.ut, sh.L, sh.rho, lane, sh.Rs[lane], sh.ts[lane]);
  __syncthreads();
  if (lane == 0) {
    const int N = epnp_pick(sh.err);
    for (int i = 0; i < 3; ++i) tvec[i] = sh.ts[N][i];
    rodrigues_R2r(sh.Rs[N], rvec);
  }
  __syncthreads();
}

// Correspondence selection (REV/utils/speed_eval.py:152-206): lane-parallel argmax over the C
// class probabilities, then (lane 0) first-seen label order with the best-score query per label.
struct SelShared {
  int lab[WAVE];
  float score[WAVE];
  int nl, order[MAXN], bestq[MAXN];
  float img[2 * MAXN], wld[3 * MAXN], sig[2 * MAXN];
};

__device__ void select_correspondences(const PnpArgs& a, int b, int lane, SelShared& sh) {
  const int Q = a.Q, C = a.C;
  for (int q = lane; q < Q; q += WAVE) {
    const float* p = a.probs + ((size_t)b * Q + q) * C;
    int lab = 0;
    float sc = p[0];
    for (int c = 1; c < C; ++c)
      if (p[c] > sc) { sc = p[c]; lab = c; }
    if (q < WAVE) { sh.lab[q] = lab; sh.score[q] = sc; }
  }
  __syncthreads();
  if (lane == 0) {
    int nl = 0;
    float best_s[MAXN];
    for (int q = 0; q < Q && q < WAVE; ++q) {
      const int lab = sh.lab[q];
      if (lab == C - 1) continue;
      int j;
      for (j = 0; j < nl; ++j) if (sh.order[j] == lab) break;
      if (j == nl) { if (nl < MAXN) { sh.order[nl] = lab; sh.bestq[nl] = q; best_s[nl] = sh.score[q]; nl++; } }
      else if (sh.score[q] > best_s[j]) { sh.bestq[j] = q; best_s[j] = sh.score[q]; }
    }
    sh.nl = nl;
    for (int j = 0; j < nl; ++j) {
      const int q = sh.bestq[j];
      sh.img[2 * j] = a.points[((size_t)b * Q + q) * 2];
      sh.img[2 * j + 1] = a.points[((size_t)b * Q + q) * 2 + 1];
      for (int c = 0; c < 3; ++c) sh.wld[3 * j + c] = (float)a.world[3 * sh.order[j] + c];
      sh.sig[2 * j] = a.sigmas ? a.sigmas[((size_t)b * Q + q) * 2] : 1.f;
      sh.sig[2 * j + 1] = a.sigmas ? a.sigmas[((size_t)b * Q + q) * 2 + 1] : 1.f;
    }
  }
  __syncthreads();
}

// ---------------------------------------------------------------- wave-parallel refinement
// CvLevMarq (lm_refine) and the sigma-weighted Huber LM (sigma_lm) of pnp_math.h with the
// per-point work spread over lanes.  Every lane holds the (uniform) 6-vector state; lane j
// projects correspondence j and writes its two residual / Jacobian rows to LDS at its rank
// among the selected points; lane e then forms normal-equation entry e by the serial loop over
// rows, in the serial code's row order and association, so g / H / the cost are the serial
// code's values bit for bit.  The 6x6 step is a register Cholesky on every lane (the serial code
// solves with a Jacobi pseudo-inverse in scratch memory, which dominated the solver's time);
// when a pivot falls below 1e-10 of the largest diagonal the wave takes the serial
// pseudo-inverse (lane 0) instead, so rank-deficient steps keep cv::solve(DECOMP_SVD) semantics.
struct LmShared {
  double J[2 * MAXN][6];
  double r[2 * MAXN];        // residual rows (lm: proj - img; sigma: w * (proj - xn))
  double w[2 * MAXN];        // sigma: per-row weight
  double red[48];            // reduced normal equations: H[36], g[6], cost
  double x[6];               // fallback step
};

// S x = b for symmetric S (lower triangle read); false when S is not safely positive definite
__device__ __forceinline__ bool chol6_solve(const double* S, const double* b, double* x) {
  double L[6][6], y[6];
  double maxd = 0;
#pragma unroll
  for (int i = 0; i < 6; ++i) maxd = fmax(maxd, fabs(S[i * 7]));
  const double thr = maxd * 1e-10;
#pragma unroll
  for (int j = 0; j < 6; ++j) {
    double s = S[j * 6 + j];
#pragma unroll
    for (int p = 0; p < j; ++p) s -= L[j][p] * L[j][p];
    if (!(s > thr)) return false;
    L[j][j] = sqrt(s);
    const double inv = 1.0 / L[j][j];
#pragma unroll
    for (int i = j + 1; i < 6; ++i) {
      double t = S[i * 6 + j];
#pragma unroll
      for (int p = 0; p < j; ++p) t -= L[i][p] * L[j][p];
      L[i][j] = t * inv;
    }
  }
#pragma unroll
  for (int i = 0; i < 6; ++i) {
    double t = b[i];
#pragma unroll
    for (int p = 0; p < i; ++p) t -= L[i][p] * y[p];
    y[i] = t / L[i][i];
  }
#pragma unroll
  for (int i = 5; i >= 0; --i) {
    double t = y[i];
#pragma unroll
    for (int p = i + 1; p < 6; ++p) t -= L[p][i] * x[p];
    x[i] = t / L[i][i];
  }
  return true;
}

__device__ void solve6_wave(LmShared& sh, const double* S, const double* b, double* x, int lane) {
  if (chol6_solve(S, b, x)) return;        // uniform: every lane holds the same S, b
  if (lane == 0) sym_solve(6, S, b, sh.x);
  __syncthreads();
#pragma unroll
  for (int i = 0; i < 6; ++i) x[i] = sh.x[i];
  __syncthreads();
}

// One correspondence per lane: its world point, pixel observation and row rank (-1 = unused).
struct LmPoint {
  double M[3], obs[2], sig[2];
  int row;
};

__device__ LmPoint lm_point(const float* img_f, const float* wld_f, const float* sig_f, int nl, uint32_t mask,
                            int lane) {
  LmPoint p{};
  p.row = -1;
  if (lane < nl && (mask >> lane) & 1u) {
    p.row = __popc(mask & ((1u << lane) - 1u));
    for (int c = 0; c < 3; ++c) p.M[c] = wld_f[3 * lane + c];
    for (int c = 0; c < 2; ++c) { p.obs[c] = img_f[2 * lane + c]; p.sig[c] = sig_f ? sig_f[2 * lane + c] : 1.0; }
  }
  return p;
}

// project_jac for this lane's point (k: camera; unit camera for normalised coordinates)
__device__ __forceinline__ void lm_project(const cam_t* k, const double* R, const double* dRdr, const double* t,
                                           const LmPoint& pt, double* proj, double (*J)[6]) {
  const double* M = pt.M;
  double X = R[0] * M[0] + R[1] * M[1] + R[2] * M[2] + t[0];
  double Y = R[3] * M[0] + R[4] * M[1] + R[5] * M[2] + t[1];
  double Z = R[6] * M[0] + R[7] * M[1] + R[8] * M[2] + t[2];
  double z = Z ? 1. / Z : 1;
  double x = X * z, y = Y * z;
  proj[0] = x * k->fx + k->cx;
  proj[1] = y * k->fy + k->cy;
  if (!J) return;
#pragma unroll
  for (int j = 0; j < 3; ++j) {
    const double* d = dRdr + 9 * j;
    double dX = d[0] * M[0] + d[1] * M[1] + d[2] * M[2];
    double dY = d[3] * M[0] + d[4] * M[1] + d[5] * M[2];
    double dZ = d[6] * M[0] + d[7] * M[1] + d[8] * M[2];
    J[0][j] = k->fx * (z * dX - x * z * dZ);
    J[1][j] = k->fy * (z * dY - y * z * dZ);
  }
  J[0][3] = k->fx * z; J[0][4] = 0; J[0][5] = -k->fx * x * z;
  J[1][3] = 0; J[1][4] = k->fy * z; J[1][5] = -k->fy * y * z;
}

// lm_refine (pnp_math.h) over the selected correspondences, all lanes; result uniform
__device__ void lm_refine_wave(LmShared& sh, const cam_t* k, const LmPoint& pt, int n, double* rvec, double* tvec,
                               int lane) {
  double param[6] = {rvec[0], rvec[1], rvec[2], tvec[0], tvec[1], tvec[2]}, prev[6];
  double JtJ[36], JtErr[6];
  int lambdaLg10 = -3, iters = 0;
  double prevErrNorm = DBL_MAX;
  const int m = 2 * n;
  // rows of the current param: residual (+ Jacobian) of this lane's point
  auto rows = [&](const double* p, bool jac) {
    double R[9], dRdr[27], proj[2], J[2][6];
    rodrigues_r2R(p, R);
    if (jac) rodrigues_jac(p, dRdr);
    if (pt.row >= 0) {
      lm_project(k, R, dRdr, p + 3, pt, proj, jac ? J : nullptr);
      for (int a = 0; a < 2; ++a) {
        sh.r[2 * pt.row + a] = proj[a] - pt.obs[a];
        if (jac)
          for (int c = 0; c < 6; ++c) sh.J[2 * pt.row + a][c] = J[a][c];
      }
    }
    __syncthreads();
  };
  auto err_norm = [&]() {     // serial sum of squares, every lane (LDS broadcast reads)
    double s = 0;
    for (int i = 0; i < m; ++i) { double r = sh.r[i]; s += r * r; }
    return sqrt(s);
  };
  rows(param, true);
  for (;;) {
    if (lane < 42) {          // normal-equation entry per lane, serial row order
      double s = 0;
      if (lane < 36) {
        const int a = lane / 6, b = lane % 6;
        for (int i = 0; i < m; ++i) s += sh.J[i][a] * sh.J[i][b];
      } else {
        const int a = lane - 36;
        for (int i = 0; i < m; ++i) s += sh.J[i][a] * sh.r[i];
      }
      sh.red[lane] = s;
    }
    __syncthreads();
#pragma unroll
    for (int e = 0; e < 36; ++e) JtJ[e] = sh.red[e];
#pragma unroll
    for (int a = 0; a < 6; ++a) JtErr[a] = sh.red[36 + a];
#pragma unroll
    for (int a = 0; a < 6; ++a) prev[a] = param[a];
    if (iters == 0) prevErrNorm = err_norm();
    __syncthreads();
    double errNorm;
    for (;;) {
      double lambda = det_pow10i(lambdaLg10);
      double S[36], dx[6];
#pragma unroll
      for (int e = 0; e < 36; ++e) S[e] = JtJ[e];
#pragma unroll
      for (int i = 0; i < 6; ++i) S[i * 6 + i] *= 1. + lambda;
      solve6_wave(sh, S, JtErr, dx, lane);
#pragma unroll
      for (int i = 0; i < 6; ++i) param[i] = prev[i] - dx[i];
      rows(param, false);
      errNorm = err_norm();
      __syncthreads();
      if (errNorm > prevErrNorm && ++lambdaLg10 <= 16) continue;
      break;
    }
    lambdaLg10 = lambdaLg10 - 1 > -16 ? lambdaLg10 - 1 : -16;
    double dn = 0, pn = 0;
#pragma unroll
    for (int i = 0; i < 6; ++i) { dn += (param[i] - prev[i]) * (param[i] - prev[i]); pn += prev[i] * prev[i]; }
    double rel = sqrt(dn) / (sqrt(pn) + DBL_EPSILON);
    if (++iters >= 20 || rel < FLT_EPSILON) break;
    prevErrNorm = errNorm;
    rows(param, true);
  }
  for (int c = 0; c < 3; ++c) { rvec[c] = param[c]; tvec[c] = param[3 + c]; }
}

// the pose on lane 0 (epnp_solve_wave / the RANSAC replay) -> every lane
__device__ void bcast_pose(LmShared& sh, double* rvec, double* tvec, int lane) {
  if (lane == 0)
    for (int c = 0; c < 3; ++c) { sh.x[c] = rvec[c]; sh.x[3 + c] = tvec[c]; }
  __syncthreads();
  for (int c = 0; c < 3; ++c) { rvec[c] = sh.x[c]; tvec[c] = sh.x[3 + c]; }
  __syncthreads();
}

// float32 reprojection error of correspondence `lane` under (rvec, t) into err[lane]; returns the
// np.sum of err[0 .. nl) on every lane (pose uniform across lanes)
__device__ float repro_errors_wave(float* err, const cam_t* k, const float* img_f, const float* wld_f, int nl,
                                   const double* rvec, const double* t, int lane) {
  __syncthreads();
  if (lane < nl) {
    double R[9];
    rodrigues_r2R(rvec, R);
    float uv[2];
    project_f(k, R, t, wld_f + 3 * lane, uv);
    err[lane] = repro_err_f(img_f + 2 * lane, uv);
  }
  __syncthreads();
  return np_sum_f32(err, nl);
}

// sigma_lm (pnp_math.h) over the selected correspondences, all lanes; result uniform
__device__ void sigma_lm_wave(LmShared& sh, const cam_t* k, const LmPoint& pt, int n, double delta, double* rvec,
                              double* tvec, int lane) {
  const int m = 2 * n;
  double xn[2] = {0, 0}, w[2] = {0, 0};
  float w1[2] = {0.f, 0.f};
  // weights in float32 like the reference's numpy on float32 sigmas (sigma_weights_f32)
  if (pt.row >= 0)
    for (int a = 0; a < 2; ++a) {
      xn[a] = (float)((pt.obs[a] - (a ? k->cy : k->cx)) * (1. / (a ? k->fy : k->fx)));
      w1[a] = 1.0f / (sqrtf((float)pt.sig[a]) + 1e-6f);
      sh.w[2 * pt.row + a] = w1[a];
    }
  __syncthreads();
  float sum[2] = {0.f, 0.f};
  for (int i = 0; i < n; ++i) { sum[0] = sum[0] + (float)sh.w[2 * i]; sum[1] = sum[1] + (float)sh.w[2 * i + 1]; }
  __syncthreads();
  if (pt.row >= 0)
    for (int a = 0; a < 2; ++a) { w[a] = (double)(w1[a] / sum[a]); sh.w[2 * pt.row + a] = w[a]; }
  const cam_t unit = {1, 1, 0, 0};
  double param[6] = {rvec[0], rvec[1], rvec[2], tvec[0], tvec[1], tvec[2]};
  double mu = 1e-4, nu = 2;
  double cost_prev = 0;
  const double d2 = delta * delta;
  for (int it = 0; it < 20; ++it) {
    {
      double R[9], dRdr[27], proj[2], J[2][6];
      rodrigues_r2R(param, R);
      rodrigues_jac(param, dRdr);
      if (pt.row >= 0) {
        lm_project(&unit, R, dRdr, param + 3, pt, proj, J);
        for (int a = 0; a < 2; ++a) {
          sh.r[2 * pt.row + a] = w[a] * (proj[a] - xn[a]);
          for (int c = 0; c < 6; ++c) sh.J[2 * pt.row + a][c] = J[a][c];
        }
      }
    }
    __syncthreads();
    if (lane < 43) {          // H[a][b] (36, not symmetric bitwise), g[a] (6), cost: serial row order
      double s = 0;
      for (int i = 0; i < m; ++i) {
        const double r = sh.r[i], r2 = r * r, wi = sh.w[i];
        double rho1 = 1;
        if (r2 > d2) {
          double q = sqrt(r2);
          rho1 = delta / q;
          if (lane == 42) s += 2 * delta * q - d2;
        } else if (lane == 42) {
          s += r2;
        }
        if (lane < 36) {
          const int a = lane / 6, b = lane % 6;
          const double ja = wi * sh.J[i][a];
          s += rho1 * ja * wi * sh.J[i][b];
        } else if (lane < 42) {
          const double ja = wi * sh.J[i][lane - 36];
          s += rho1 * ja * r;
        }
      }
      sh.red[lane] = s;
    }
    __syncthreads();
    double H[36], g[6], cost;
#pragma unroll
    for (int e = 0; e < 36; ++e) H[e] = sh.red[e];
#pragma unroll
    for (int a = 0; a < 6; ++a) g[a] = sh.red[36 + a];
    cost = sh.red[42];
    __syncthreads();
    if (it == 0) cost_prev = cost;
    double S[36], dx[6], trial[6];
#pragma unroll
    for (int e = 0; e < 36; ++e) S[e] = H[e];
#pragma unroll
    for (int a = 0; a < 6; ++a) S[a * 6 + a] += mu * (H[a * 6 + a] > 1e-12 ? H[a * 6 + a] : 1e-12);
    solve6_wave(sh, S, g, dx, lane);
#pragma unroll
    for (int a = 0; a < 6; ++a) trial[a] = param[a] - dx[a];
    {
      double R[9], proj[2];
      rodrigues_r2R(trial, R);
      if (pt.row >= 0) {
        lm_project(&unit, R, nullptr, trial + 3, pt, proj, nullptr);
        for (int a = 0; a < 2; ++a) sh.r[2 * pt.row + a] = w[a] * (proj[a] - xn[a]);
      }
    }
    __syncthreads();
    double cost_new = 0;
    for (int i = 0; i < m; ++i) {
      double r = sh.r[i], r2 = r * r;
      cost_new += r2 > d2 ? 2 * delta * sqrt(r2) - d2 : r2;
    }
    __syncthreads();
    if (cost_new < cost_prev) {
#pragma unroll
      for (int a = 0; a < 6; ++a) param[a] = trial[a];
      double dn = 0, pn = 0;
#pragma unroll
      for (int a = 0; a < 6; ++a) { dn += dx[a] * dx[a]; pn += param[a] * param[a]; }
      mu *= 1. / 3.; nu = 2;
      if (cost_prev - cost_new < 1e-6 * cost_prev || sqrt(dn) < 1e-8 * (sqrt(pn) + 1e-8)) { cost_prev = cost_new; break; }
      cost_prev = cost_new;
    } else {
      mu *= nu; nu *= 2;
    }
  }
  for (int c = 0; c < 3; ++c) { rvec[c] = param[c]; tvec[c] = param[3 + c]; }
}

// The cv::RNG((uint64)-1) subset stream of OpenCV's RANSACPointSetRegistrator: `mp` distinct
// indices in [0, nl) per iteration, rejection-sampled, iterations drawn in order.
__device__ void draw_subset(rng_t* rng, int nl, int mp, int* idx) {
  for (int i = 0; i < mp; ++i) {
    for (;;) {
      int v = rng_uniform(rng, 0, nl), j;
      idx[i] = v;
      for (j = 0; j < i; ++j) if (v == idx[j]) break;
      if (j == i) break;
    }
  }
}

// RANSAC uses EPnP hypotheses (5-point model): sigma mode with more than 5 correspondences
SPE_DEV bool epnp_ransac_path(const PnpArgs& a, int nl) { return a.mode == SPE_PNP_EPNP_RANSAC_SIGMA && nl > 5; }

// EPnP-RANSAC hypotheses, one wave per (image, iteration): the 12x12 eigen-decomposition of a
// 5-point EPnP runs wave-cooperatively (jacobi12_rr_wave) instead of serially on one lane of the
// image's wave, so the ~100 hypotheses of an image run concurrently across the chip.  Same IEEE
// operation sequence as the serial per-lane form (jacobi12_rr == the oracle's), so inlier sets
// stay bit-identical.  Results go to a[b][it] records; pnp_kernel replays the adaptive loop.
__global__ __launch_bounds__(WAVE) void pnp_hyp_kernel(PnpArgs a, int iters) {
  const int b = blockIdx.x / iters, it = blockIdx.x - b * iters;
  const int lane = threadIdx.x;
  __shared__ SelShared sel;
  __shared__ float h_img[10], h_wld[15];
  __shared__ double h_rt[6];
  __shared__ EpnpShared s_ep;
  select_correspondences(a, b, lane, sel);
  const int nl = sel.nl;
  if (!epnp_ransac_path(a, nl)) return;              // wave-uniform
  if (lane == 0) {
    rng_t rng = {(uint64_t)-1};
    int idx[5];
    for (int j = 0; j <= it; ++j) draw_subset(&rng, nl, 5, idx);
    for (int i = 0; i < 5; ++i) {
      h_img[2 * i] = sel.img[2 * idx[i]]; h_img[2 * i + 1] = sel.img[2 * idx[i] + 1];
      for (int c = 0; c < 3; ++c) h_wld[3 * i + c] = sel.wld[3 * idx[i] + c];
    }
  }
  __syncthreads();
  const cam_t k = {a.K[0], a.K[4], a.K[2], a.K[5]};
  double r[3], tt[3];
  epnp_solve_wave(s_ep, &k, h_img, h_wld, 5, 0x1Fu, 1, r, tt, lane);
  if (lane == 0) for (int c = 0; c < 3; ++c) { h_rt[c] = r[c]; h_rt[3 + c] = tt[c]; }
  __syncthreads();
  for (int c = 0; c < 3; ++c) { r[c] = h_rt[c]; tt[c] = h_rt[3 + c]; }
  const float thr2 = (float)((double)a.repro * (double)a.repro);
  bool in = false;
  if (lane < nl) {
    double R[9];
    rodrigues_r2R(r, R);
    float uv[2];
    project_f(&k, R, tt, sel.wld + 3 * lane, uv);
    in = sq_err_f(sel.img + 2 * lane, uv) <= thr2;
  }
  const uint64_t m = __ballot(in);
  if (lane == 0) {
    HypRec& h = a.hyp[(size_t)b * a.hyp_stride + it];
    for (int c = 0; c < 6; ++c) h.rt[c] = h_rt[c];
    h.mask = (uint32_t)m;
    h.good = __popcll(m);
    h.ok = 1;
  }
}

__global__ __launch_bounds__(WAVE) void pnp_kernel(PnpArgs a) {
  const int b = blockIdx.x;
  const int lane = threadIdx.x;
  __shared__ SelShared sel;
  float* const s_img = sel.img;
  float* const s_wld = sel.wld;
  float* const s_sig = sel.sig;
  __shared__ unsigned char s_idx[MAXIT][5];
  __shared__ int s_ok[MAXIT], s_good[MAXIT];
  __shared__ uint32_t s_mask[MAXIT];
  __shared__ double s_rt[MAXIT][6];
  __shared__ EpnpShared s_ep;
  __shared__ LmShared s_lm;
  __shared__ float s_err[MAXN];

  const cam_t k = {a.K[0], a.K[4], a.K[2], a.K[5]};

  select_correspondences(a, b, lane, sel);
  const int nl = sel.nl;
  const uint32_t all = nl >= 32 ? 0xffffffffu : ((1u << nl) - 1);

  double rvec[3] = {0, 0, 0}, t[3] = {0, 0, 0};
  int status = SPE_PNP_OK;
  uint32_t inl = 0;
  bool have_pose = false;

  if (nl == 0) {
    status = SPE_PNP_NO_FG;
  } else if (nl < 4) {
    status = SPE_PNP_CV_ERROR;
  } else if (a.mode == SPE_PNP_EPNP || a.mode == SPE_PNP_EPNP_LM || a.mode == SPE_PNP_EPNP_CERES) {
    epnp_solve_wave(s_ep, &k, s_img, s_wld, nl, all, 1, rvec, t, lane);
    bcast_pose(s_lm, rvec, t, lane);
    if (a.mode == SPE_PNP_EPNP_LM) {
      lm_refine_wave(s_lm, &k, lm_point(s_img, s_wld, nullptr, nl, all, lane), nl, rvec, t, lane);
      inl = all;
    } else {
      // epnp_init (UNC/utils/speed_eval_ceres.py:153-169): float32 reprojection errors of every
      // correspondence, inliers err < th, and their np.sum
      const float th = a.repro_img ? a.repro_img[b] : a.repro;
      const float before = repro_errors_wave(s_err, &k, s_img, s_wld, nl, rvec, t, lane);
      inl = (uint32_t)__ballot(lane < nl && (double)s_err[lane] < (double)th);
      const int m = __popc(inl);
      if (a.mode == SPE_PNP_EPNP_CERES && m == 1) {
        status = SPE_PNP_NO_FG;                    // obj_pts[idx, 0] on a squeezed 1-D array: IndexError
      } else if (a.mode == SPE_PNP_EPNP_CERES && m >= 2) {
        // ceres_pnp (:172-243) on the inliers, weights normalised over them, HuberLoss(0.001);
        // keep the EPnP pose if the refined error sum over all points is larger (:142-146)
        double r2[3] = {rvec[0], rvec[1], rvec[2]}, t2[3] = {t[0], t[1], t[2]};
        sigma_lm_wave(s_lm, &k, lm_point(s_img, s_wld, s_sig, nl, inl, lane), m, 0.001, r2, t2, lane);
        const float after = repro_errors_wave(s_err, &k, s_img, s_wld, nl, r2, t2, lane);
        if (!(after > before))
          for (int c = 0; c < 3; ++c) { rvec[c] = r2[c]; t[c] = t2[c]; }
      }
    }
    have_pose = status == SPE_PNP_OK;
  } else {
    const int kernel = (a.mode == SPE_PNP_RANSAC_P3P_LM || nl == 4) ? 0 : 1;
    const int mp = kernel == 0 ? 4 : 5;
    bool ok = false;
    if (nl == mp) {
      // model_points == npoints: direct solve on all points (solvepnp.cpp)
      if (kernel == 0) {
        if (lane == 0) s_ok[0] = p3p_solve4(&k, s_img, s_wld, rvec, t) != 0;
      } else {
        epnp_solve_wave(s_ep, &k, s_img, s_wld, nl, all, 1, rvec, t, lane);
        if (lane == 0) s_ok[0] = 1;
      }
      __syncthreads();
      ok = s_ok[0];
      if (!ok) status = SPE_PNP_UNPINNED;
      inl = all;
    } else {
      const int iters = a.ransac_iters < MAXIT ? a.ransac_iters : MAXIT;
      // 1. subset stream of cv::RNG((uint64)-1), drawn in order
      const bool pre = kernel == 1 && a.hyp != nullptr;   // hypotheses precomputed by pnp_hyp_kernel
      if (lane == 0 && !pre) {
        rng_t rng = {(uint64_t)-1};
        for (int it = 0; it < iters; ++it) {
          int idx[5];
          draw_subset(&rng, nl, mp, idx);
          for (int i = 0; i < mp; ++i) s_idx[it][i] = (unsigned char)idx[i];
        }
      }
      __syncthreads();
      // 2. hypotheses + float32 inlier sets, lane-parallel
      const float thr2 = (float)((double)a.repro * (double)a.repro);
      if (pre) {
        for (int it = lane; it < iters; it += WAVE) {
          const HypRec& h = a.hyp[(size_t)b * a.hyp_stride + it];
          s_ok[it] = h.ok;
          s_good[it] = h.good;
          s_mask[it] = h.mask;
          for (int c = 0; c < 6; ++c) s_rt[it][c] = h.rt[c];
        }
      }
      for (int it = pre ? iters : lane; it < iters; it += WAVE) {
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
      // 3. serial replay of the adaptive loop (lane 0)
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
          s_mask[MAXIT - 1] = s_mask[best];
          s_ok[MAXIT - 1] = 1;
        } else if (last >= 0) {
          for (int c = 0; c < 3; ++c) { rvec[c] = s_rt[last][c]; t[c] = s_rt[last][3 + c]; }
          s_ok[MAXIT - 1] = 2;
        } else {
          s_ok[MAXIT - 1] = 0;
        }
      }
      __syncthreads();
      const int verdict = s_ok[MAXIT - 1];
      ok = verdict == 1;
      if (ok) {
        inl = s_mask[MAXIT - 1];
        epnp_solve_wave(s_ep, &k, s_img, s_wld, nl, inl, 0, rvec, t, lane);   // refit on the consensus set
      }
      if (verdict == 2) status = SPE_PNP_RANSAC_FALLBACK;
      if (verdict == 0) status = SPE_PNP_UNPINNED;
    }
    if (ok) {                                     // wave-uniform
      bcast_pose(s_lm, rvec, t, lane);
      const LmPoint pt = lm_point(s_img, s_wld, s_sig, nl, inl, lane);
      const int m = __popc(inl);
      if (a.mode == SPE_PNP_RANSAC_P3P_LM) lm_refine_wave(s_lm, &k, pt, m, rvec, t, lane);
      else sigma_lm_wave(s_lm, &k, pt, m, 0.005, rvec, t, lane);
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
  if (a.corr_label) for (int j = 0; j < MAXN; ++j) a.corr_label[MAXN * b + j] = j < nl ? sel.order[j] : -1;
}

// SPEED score (REV/utils/speed_eval.py:245-262): q sign-normalised, s_t = |dt|/|t_gt|,
// s_q = 2 acos(min(|q.q_gt|, 1)), NaN poses score NaN as on the host; failures arrive as zero poses (REV/datasets/speed.py:355-363).
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
  // Python's min(d, 1) keeps its first argument unless 1 < d, so a NaN dot product stays NaN
  s_q[b] = 2 * acos(1 < d ? 1.0 : d);
}

// Self-assessment filter (BASELINE config 4).  The reference has no code for it: the UNC README
// (ROOT/README.md:15-20) describes a mechanism that "filters out unreliable pose estimation
// results" from the predicted keypoint sigmas, and the only code trace is the commented per-
// keypoint gate `s_ > 0.5 and sig.mean() < 5` (UNC/utils/speed_eval_ceres.py:110-114).  Defined
// here (parity unpinned): with the solver's correspondence selection
// re-derived from probs (same argmax / first-on-ties rule as pnp_kernel), over the RANSAC
// inliers j of image b:
//     mean_sigma[b] = mean over inliers and both axes of sigma[sel(j)]
//     confident(j)  = score(sel(j)) > score_th  and  mean(sigma[sel(j)]) < sigma_th
//     reliable[b]   = status in {0, 3} and #confident inliers >= min_inliers and mean_sigma < sigma_th
// One thread per image (Q <= 64, C <= 17): the whole pass is a few hundred loads.
__global__ void self_assess_kernel(SelfAssessArgs a) {
  const int b = blockIdx.x * blockDim.x + threadIdx.x;
  if (b >= a.B) return;
  const int Q = a.Q, C = a.C;
  int best_q[MAXN];
  float best_s[MAXN];
  for (int l = 0; l < MAXN; ++l) { best_q[l] = -1; best_s[l] = 0.f; }
  for (int q = 0; q < Q; ++q) {
    const float* p = a.probs + ((size_t)b * Q + q) * C;
    int lab = 0;
    float sc = p[0];
    for (int c = 1; c < C; ++c)
      if (p[c] > sc) { sc = p[c]; lab = c; }
    if (lab == C - 1) continue;
    if (best_q[lab] < 0 || sc > best_s[lab]) { best_q[lab] = q; best_s[lab] = sc; }
  }
  const int st = a.status[b];
  const uint32_t inl = (st == SPE_PNP_OK || st == SPE_PNP_RANSAC_FALLBACK) ? a.inlier_mask[b] : 0u;
  float ssum = 0.f;
  int n = 0, nconf = 0;
  for (int j = 0; j < MAXN; ++j) {
    if (!(inl & (1u << j))) continue;
    const int lab = a.corr_label[MAXN * b + j];
    if (lab < 0 || lab >= MAXN || best_q[lab] < 0) continue;
    const int q = best_q[lab];
    const float sx = a.sigmas[((size_t)b * Q + q) * 2], sy = a.sigmas[((size_t)b * Q + q) * 2 + 1];
    ssum += sx + sy;
    n++;
    if (best_s[lab] > a.score_th && 0.5f * (sx + sy) < a.sigma_th) nconf++;
  }
  const float ms = n ? ssum / (2.f * n) : INFINITY;
  a.mean_sigma[b] = ms;
  a.n_confident[b] = nconf;
  a.reliable[b] = (n > 0 && nconf >= a.min_inliers && ms < a.sigma_th) ? 1 : 0;
}

}  // namespace

int spe_launch_self_assess(const SelfAssessArgs& a, hipStream_t s) {
  if (a.B <= 0) return 0;
  if (a.Q > WAVE || a.C < 2 || a.C - 1 > MAXN) return -7;
  hipLaunchKernelGGL(self_assess_kernel, dim3((a.B + 127) / 128), dim3(128), 0, s, a);
  return (int)hipGetLastError();
}

int spe_launch_pnp(const PnpArgs& a, hipStream_t s) {
  if (a.B <= 0) return 0;
  if (a.Q > WAVE || a.C < 2 || a.C - 1 > MAXN || a.ransac_iters > MAXIT - 1) return -7;
  if (a.hyp) {
    if (a.hyp_stride < a.ransac_iters) return -7;
    hipLaunchKernelGGL(pnp_hyp_kernel, dim3(a.B * a.ransac_iters), dim3(WAVE), 0, s, a, a.ransac_iters);
  }
  hipLaunchKernelGGL(pnp_kernel, dim3(a.B), dim3(WAVE), 0, s, a);
  return (int)hipGetLastError();
}

int spe_launch_score(const float* quat, const double* tvec, const double* q_gt, const double* t_gt, int B, double* s_t,
                     double* s_q, hipStream_t s) {
  if (B <= 0) return 0;
  hipLaunchKernelGGL(score_kernel, dim3((B + 127) / 128), dim3(128), 0, s, quat, tvec, q_gt, t_gt, B, s_t, s_q);
  return (int)hipGetLastError();
}
