// Device-side pose-solver arithmetic (OpenCV 4.4 p3p / epnp / LevMarq restated, Blender
// mat3_to_quat, deterministic transcendental helpers) used by pnp.hip.  Same published
// algorithms and the same IEEE operation sequence as the CPU checker oracle/pnp_ref.c (a
// separate copy: the product never links the oracle); both are compiled with
// -ffp-contract=off so integer / index outputs (inlier sets, iteration counts) agree bit for bit.
// Every function here runs on one lane; pnp.hip provides the wave-level parallelism
// (lane-parallel RANSAC hypotheses, wave-cooperative M^T M and 12x12 Jacobi for EPnP).
#pragma once
#include <hip/hip_runtime.h>
#include <stdint.h>
#include <float.h>
#define PNP_FN __device__ static inline
#define MAXN 16
typedef struct { double fx, fy, cx, cy; } cam_t;
/* ------------------------------------------------------------------ cv::RNG */
typedef struct { uint64_t state; } rng_t;
PNP_FN unsigned rng_next(rng_t* r) {
  r->state = (uint64_t)(unsigned)r->state * 4164903690U + (unsigned)(r->state >> 32);
  return (unsigned)r->state;
}
PNP_FN int rng_uniform(rng_t* r, int a, int b) { return a == b ? a : (int)(rng_next(r) % (unsigned)(b - a) + a); }

/* ------------------------------------------------------------------ deterministic math
 * The inlier decisions and the RANSAC iteration count are index outputs that must agree bit for
 * bit between this checker and the device solver.  libm (glibc) and the GPU's device library
 * round transcendental functions differently in the last ulp, so every transcendental on the
 * decision path is evaluated here with a fixed sequence of IEEE add/mul/div/sqrt (and the file
 * is compiled with -ffp-contract=off on both sides).  Accuracy is ~1 ulp; OpenCV itself uses
 * libm, so agreement with OpenCV stays at rounding level (unpinned there anyway). */
PNP_FN double det_rint(double x) { return rint(x); } /* exact IEEE operation */

PNP_FN void det_sincos(double x, double* s_out, double* c_out) {
  const double INV_PIO2 = 6.36619772367581382433e-01;
  const double PIO2_1 = 1.57079632673412561417e+00, PIO2_1T = 6.07710050650619224932e-11;
  double k = det_rint(x * INV_PIO2);
  double r = (x - k * PIO2_1) - k * PIO2_1T;
  double z = r * r;
  /* Taylor coefficients (-1)^n / (2n+1)!  and  (-1)^n / (2n)!, Horner in z = r^2 */
  const double SC[10] = {1.0, -1.0 / 6.0, 1.0 / 120.0, -1.0 / 5040.0, 1.0 / 362880.0, -1.0 / 39916800.0,
                                1.0 / 6227020800.0, -1.0 / 1307674368000.0, 1.0 / 355687428096000.0,
                                -1.0 / 121645100408832000.0};
  const double CC[10] = {1.0, -1.0 / 2.0, 1.0 / 24.0, -1.0 / 720.0, 1.0 / 40320.0, -1.0 / 3628800.0,
                                1.0 / 479001600.0, -1.0 / 87178291200.0, 1.0 / 20922789888000.0,
                                -1.0 / 6402373705728000.0};
  double s = SC[9], c = CC[9];
  for (int i = 8; i >= 0; --i) { s = s * z + SC[i]; c = c * z + CC[i]; }
  s *= r;
  long q = ((long)k) & 3;
  if (q == 0) { *s_out = s; *c_out = c; }
  else if (q == 1) { *s_out = c; *c_out = -s; }
  else if (q == 2) { *s_out = -s; *c_out = -c; }
  else { *s_out = -c; *c_out = s; }
}
PNP_FN double det_sin(double x) { double s, c; det_sincos(x, &s, &c); return s; }
PNP_FN double det_cos(double x) { double s, c; det_sincos(x, &s, &c); return c; }

/* asin for |y| <= 0.5 by its Taylor series (terms decrease faster than 4^-n) */
PNP_FN double det_asin_small(double y) {
  double y2 = y * y, term = y, sum = y;
  for (int n = 1; n < 30; ++n) {
    term = term * y2 * ((2.0 * n - 1.0) * (2.0 * n - 1.0)) / ((2.0 * n) * (2.0 * n + 1.0));
    sum += term;
  }
  return sum;
}

PNP_FN double det_acos(double x) {
  const double PI = 3.14159265358979311600e+00, PIO2 = 1.57079632679489655800e+00;
  if (x >= 1.0) return 0.0;
  if (x <= -1.0) return PI;
  if (x <= 0.5 && x >= -0.5) return PIO2 - det_asin_small(x);
  if (x > 0.5) return 2.0 * det_asin_small(sqrt((1.0 - x) * 0.5));
  return PI - 2.0 * det_asin_small(sqrt((1.0 + x) * 0.5));
}

PNP_FN double det_cbrt(double x) {
  if (x == 0.0) return 0.0;
  double a = fabs(x);
  int e;
  double m = frexp(a, &e); /* a = m 2^e, m in [0.5, 1) */
  int r = ((e % 3) + 3) % 3;
  m = ldexp(m, r);         /* m in [0.5, 4) */
  e -= r;
  double y = 0.75 + 0.25 * m;
  for (int i = 0; i < 10; ++i) y = y - (y * y * y - m) / (3.0 * y * y);
  y = ldexp(y, e / 3);
  return x < 0 ? -y : y;
}

PNP_FN double det_log(double x) { /* x > 0 */
  const double LN2_HI = 6.93147180369123816490e-01, LN2_LO = 1.90821492927058770002e-10;
  int e;
  double m = frexp(x, &e);
  if (m < 7.07106781186547524401e-01) { m *= 2.0; e -= 1; }
  double s = (m - 1.0) / (m + 1.0), s2 = s * s, term = s, sum = s;
  for (int n = 1; n < 14; ++n) { term *= s2; sum += term / (2.0 * n + 1.0); }
  return (double)e * LN2_HI + ((double)e * LN2_LO + 2.0 * sum);
}

PNP_FN double det_pow10i(int k) {
  double v = 1.0;
  for (int i = 0; i < (k > 0 ? k : -k); ++i) v *= 10.0;
  return k >= 0 ? v : 1.0 / v;
}

/* ------------------------------------------------------------------ small linear algebra */
/* cyclic Jacobi eigen-decomposition of a symmetric n x n matrix (row-major, destroyed).
 * evec[i*n + k] = component i of eigenvector k.  Eigenvalues returned unsorted. */
PNP_FN void jacobi_eig(int n, double* a, double* ev, double* evec) {
  for (int i = 0; i < n; ++i)
    for (int j = 0; j < n; ++j) evec[i * n + j] = (i == j);
  for (int sweep = 0; sweep < 60; ++sweep) {
    double off = 0, diag = 0;
    for (int i = 0; i < n; ++i) {
      diag += a[i * n + i] * a[i * n + i];
      for (int j = i + 1; j < n; ++j) off += a[i * n + j] * a[i * n + j];
    }
    if (off <= 1e-30 * diag || off == 0) break;
    for (int p = 0; p < n - 1; ++p)
      for (int q = p + 1; q < n; ++q) {
        double apq = a[p * n + q];
        if (fabs(apq) < 1e-300) continue;
        double app = a[p * n + p], aqq = a[q * n + q];
        double theta = (aqq - app) / (2 * apq);
        double t = (theta >= 0 ? 1.0 : -1.0) / (fabs(theta) + sqrt(theta * theta + 1));
        double c = 1 / sqrt(t * t + 1), s = t * c;
        for (int k = 0; k < n; ++k) {
          double akp = a[k * n + p], akq = a[k * n + q];
          a[k * n + p] = c * akp - s * akq;
          a[k * n + q] = s * akp + c * akq;
        }
        for (int k = 0; k < n; ++k) {
          double apk = a[p * n + k], aqk = a[q * n + k];
          a[p * n + k] = c * apk - s * aqk;
          a[q * n + k] = s * apk + c * aqk;
        }
        for (int k = 0; k < n; ++k) {
          double vkp = evec[k * n + p], vkq = evec[k * n + q];
          evec[k * n + p] = c * vkp - s * vkq;
          evec[k * n + q] = s * vkp + c * vkq;
        }
      }
  }
  for (int i = 0; i < n; ++i) ev[i] = a[i * n + i];
}

/* eigen-decomposition sorted by descending eigenvalue; vt[k*n + i] = component i of vector k
 * (the row layout of OpenCV's cvSVD(..., CV_SVD_U_T) on a symmetric PSD matrix). */
/* Jacobi rotation angle for pivot (p, q); identity when a_pq vanishes */
PNP_FN void jacobi_cs(double app, double aqq, double apq, double* c, double* s) {
  if (fabs(apq) < 1e-300) { *c = 1.0; *s = 0.0; return; }
  double theta = (aqq - app) / (2 * apq);
  double t = (theta >= 0 ? 1.0 : -1.0) / (fabs(theta) + sqrt(theta * theta + 1));
  *c = 1 / sqrt(t * t + 1);
  *s = t * *c;
}

/* round r of the 12-player round-robin: 6 disjoint pivot pairs (p < q) covering 0..11 */
PNP_FN void rr_pairs(int r, int* P, int* Q) {
  int a = 11, b = r;
  P[0] = b < a ? b : a; Q[0] = b < a ? a : b;
  for (int i = 1; i < 6; ++i) {
    a = (r + i) % 11; b = (r + 11 - i) % 11;
    P[i] = a < b ? a : b; Q[i] = a < b ? b : a;
  }
}

/* Round-parallel cyclic Jacobi for the 12x12 EPnP normal matrix M^T M: the 6 rotations of a
 * round are computed from one snapshot and applied as a column pass then a row pass.  This
 * is the order the device solver runs with 64 lanes cooperating (csrc/pnp.hip), and the
 * sequential form here performs exactly the same IEEE operations.  evec: column k = vector k. */
PNP_FN void jacobi12_rr(double* a, double* ev, double* evec) {
  const int n = 12;
  double tmp[144];
  for (int i = 0; i < n; ++i)
    for (int j = 0; j < n; ++j) evec[i * n + j] = (i == j);
  for (int sweep = 0; sweep < 60; ++sweep) {
    double off = 0, diag = 0;
    for (int i = 0; i < n; ++i) {
      diag += a[i * n + i] * a[i * n + i];
      for (int j = i + 1; j < n; ++j) off += a[i * n + j] * a[i * n + j];
    }
    if (off <= 1e-30 * diag || off == 0) break;
    for (int r = 0; r < 11; ++r) {
      int P[6], Q[6];
      double C[6], S[6];
      rr_pairs(r, P, Q);
      for (int k = 0; k < 6; ++k) jacobi_cs(a[P[k] * n + P[k]], a[Q[k] * n + Q[k]], a[P[k] * n + Q[k]], &C[k], &S[k]);
      memcpy(tmp, a, sizeof tmp);
      for (int k = 0; k < 6; ++k)
        for (int i = 0; i < n; ++i) {
          const double x = a[i * n + P[k]], y = a[i * n + Q[k]];
          tmp[i * n + P[k]] = C[k] * x - S[k] * y;
          tmp[i * n + Q[k]] = S[k] * x + C[k] * y;
        }
      for (int k = 0; k < 6; ++k)
        for (int j = 0; j < n; ++j) {
          const double x = tmp[P[k] * n + j], y = tmp[Q[k] * n + j];
          a[P[k] * n + j] = C[k] * x - S[k] * y;
          a[Q[k] * n + j] = S[k] * x + C[k] * y;
        }
      for (int k = 0; k < 6; ++k)
        for (int i = 0; i < n; ++i) {
          const double x = evec[i * n + P[k]], y = evec[i * n + Q[k]];
          evec[i * n + P[k]] = C[k] * x - S[k] * y;
          evec[i * n + Q[k]] = S[k] * x + C[k] * y;
        }
    }
  }
  for (int i = 0; i < n; ++i) ev[i] = a[i * n + i];
}

/* sort an eigen-decomposition by descending eigenvalue into vt rows (stable insertion sort) */
PNP_FN void eig_sort_desc(int n, const double* ev, const double* evec, double* w, double* vt) {
  int idx[12];
  for (int i = 0; i < n; ++i) idx[i] = i;
  for (int i = 1; i < n; ++i)
    for (int j = i; j > 0 && ev[idx[j - 1]] < ev[idx[j]]; --j) { int t = idx[j]; idx[j] = idx[j - 1]; idx[j - 1] = t; }
  for (int k = 0; k < n; ++k) {
    w[k] = ev[idx[k]];
    for (int i = 0; i < n; ++i) vt[k * n + i] = evec[i * n + idx[k]];
  }
}

PNP_FN void sym_eig_desc(int n, const double* A, double* w, double* vt) {
  double a[144], ev[12], evec[144];
  memcpy(a, A, sizeof(double) * n * n);
  if (n == 12) {
    jacobi12_rr(a, ev, evec);
    eig_sort_desc(n, ev, evec, w, vt);
    return;
  }
  jacobi_eig(n, a, ev, evec);
  int idx[12];
  for (int i = 0; i < n; ++i) idx[i] = i;
  for (int i = 1; i < n; ++i)
    for (int j = i; j > 0 && ev[idx[j - 1]] < ev[idx[j]]; --j) { int t = idx[j]; idx[j] = idx[j - 1]; idx[j - 1] = t; }
  for (int k = 0; k < n; ++k) {
    w[k] = ev[idx[k]];
    for (int i = 0; i < n; ++i) vt[k * n + i] = evec[i * n + idx[k]];
  }
}

/* minimum-norm least squares x = pinv(A) b, A is m x n (n <= 6), via eig of A^T A */
PNP_FN void lstsq_pinv(int m, int n, const double* A, const double* b, double* x) {
  double ata[36], atb[6], w[6], vt[36];
  for (int i = 0; i < n; ++i) {
    atb[i] = 0;
    for (int k = 0; k < m; ++k) atb[i] += A[k * n + i] * b[k];
    for (int j = 0; j < n; ++j) {
      double s = 0;
      for (int k = 0; k < m; ++k) s += A[k * n + i] * A[k * n + j];
      ata[i * n + j] = s;
    }
  }
  sym_eig_desc(n, ata, w, vt);
  double thr = w[0] * DBL_EPSILON * 16;
  for (int i = 0; i < n; ++i) x[i] = 0;
  for (int k = 0; k < n; ++k) {
    if (w[k] <= thr) continue;
    double c = 0;
    for (int i = 0; i < n; ++i) c += vt[k * n + i] * atb[i];
    c /= w[k];
    for (int i = 0; i < n; ++i) x[i] += c * vt[k * n + i];
  }
}

/* solve symmetric system S x = r (pseudo-inverse; S n x n, n <= 6) */
PNP_FN void sym_solve(int n, const double* S, const double* r, double* x) {
  double w[6], vt[36];
  sym_eig_desc(n, S, w, vt);
  double thr = fabs(w[0]) * DBL_EPSILON * 16;
  for (int i = 0; i < n; ++i) x[i] = 0;
  for (int k = 0; k < n; ++k) {
    if (fabs(w[k]) <= thr) continue;
    double c = 0;
    for (int i = 0; i < n; ++i) c += vt[k * n + i] * r[i];
    c /= w[k];
    for (int i = 0; i < n; ++i) x[i] += c * vt[k * n + i];
  }
}

/* 3x3 SVD A = U diag(s) V^T (one-sided Jacobi on columns); U, V row-major 3x3 */
PNP_FN void svd3(const double* A, double* U, double* s, double* V) {
  double a[9];
  memcpy(a, A, sizeof a);
  for (int i = 0; i < 9; ++i) V[i] = (i % 4 == 0);
  for (int sweep = 0; sweep < 60; ++sweep) {
    double conv = 0;
    for (int p = 0; p < 2; ++p)
      for (int q = p + 1; q < 3; ++q) {
        double alpha = 0, beta = 0, gamma = 0;
        for (int k = 0; k < 3; ++k) {
          alpha += a[k * 3 + p] * a[k * 3 + p];
          beta += a[k * 3 + q] * a[k * 3 + q];
          gamma += a[k * 3 + p] * a[k * 3 + q];
        }
        if (gamma == 0) continue;
        double c0 = fabs(gamma) / sqrt(alpha * beta);
        if (c0 > conv) conv = c0;
        double zeta = (beta - alpha) / (2 * gamma);
        double t = (zeta >= 0 ? 1.0 : -1.0) / (fabs(zeta) + sqrt(1 + zeta * zeta));
        double c = 1 / sqrt(1 + t * t), sn = c * t;
        for (int k = 0; k < 3; ++k) {
          double x = a[k * 3 + p], y = a[k * 3 + q];
          a[k * 3 + p] = c * x - sn * y;
          a[k * 3 + q] = sn * x + c * y;
          x = V[k * 3 + p]; y = V[k * 3 + q];
          V[k * 3 + p] = c * x - sn * y;
          V[k * 3 + q] = sn * x + c * y;
        }
      }
    if (conv < 1e-15) break;
  }
  for (int j = 0; j < 3; ++j) {
    double nrm = sqrt(a[j] * a[j] + a[3 + j] * a[3 + j] + a[6 + j] * a[6 + j]);
    s[j] = nrm;
    for (int k = 0; k < 3; ++k) U[k * 3 + j] = nrm > 1e-300 ? a[k * 3 + j] / nrm : 0;
  }
  /* sort descending */
  for (int i = 0; i < 2; ++i)
    for (int j = 0; j < 2 - i; ++j)
      if (s[j] < s[j + 1]) {
        double t = s[j]; s[j] = s[j + 1]; s[j + 1] = t;
        for (int k = 0; k < 3; ++k) {
          t = U[k * 3 + j]; U[k * 3 + j] = U[k * 3 + j + 1]; U[k * 3 + j + 1] = t;
          t = V[k * 3 + j]; V[k * 3 + j] = V[k * 3 + j + 1]; V[k * 3 + j + 1] = t;
        }
      }
  if (s[2] <= 1e-14 * (s[0] > 0 ? s[0] : 1)) { /* complete a null left vector */
    U[2] = U[3] * U[7] - U[6] * U[4];
    U[5] = U[6] * U[1] - U[0] * U[7];
    U[8] = U[0] * U[4] - U[3] * U[1];
  }
}

/* ------------------------------------------------------------------ Rodrigues */
PNP_FN void rodrigues_r2R(const double* r, double* R) {
  double th = sqrt(r[0] * r[0] + r[1] * r[1] + r[2] * r[2]);
  if (th < DBL_EPSILON) {
    for (int i = 0; i < 9; ++i) R[i] = (i % 4 == 0);
    return;
  }
  double c, s;
  det_sincos(th, &s, &c);
  double c1 = 1. - c, it = 1. / th;
  double x = r[0] * it, y = r[1] * it, z = r[2] * it;
  double rrt[9] = {x * x, x * y, x * z, x * y, y * y, y * z, x * z, y * z, z * z};
  double rx[9] = {0, -z, y, z, 0, -x, -y, x, 0};
  for (int k = 0; k < 9; ++k) R[k] = c * (k % 4 == 0) + c1 * rrt[k] + s * rx[k];
}

/* dR/dr: J[i*9 + k] = d R_k / d r_i (cvRodrigues2 jacobian) */
PNP_FN void rodrigues_jac(const double* r, double* J) {
  double th = sqrt(r[0] * r[0] + r[1] * r[1] + r[2] * r[2]);
  if (th < DBL_EPSILON) {
    const double J0[27] = {0, 0, 0, 0, 0, 1, 0, -1, 0, 0, 0, -1, 0, 0, 0, 1, 0, 0, 0, 1, 0, -1, 0, 0, 0, 0, 0};
    memcpy(J, J0, sizeof J0);
    return;
  }
  double c, s;
  det_sincos(th, &s, &c);
  double c1 = 1. - c, it = 1. / th;
  double x = r[0] * it, y = r[1] * it, z = r[2] * it;
  double rrt[9] = {x * x, x * y, x * z, x * y, y * y, y * z, x * z, y * z, z * z};
  double rx[9] = {0, -z, y, z, 0, -x, -y, x, 0};
  double drrt[27] = {x + x, y, z, y, 0, 0, z, 0, 0, 0, x, 0, x, y + y, z, 0, z, 0, 0, 0, x, 0, 0, y, x, y, z + z};
  double drx[27] = {0, 0, 0, 0, 0, -1, 0, 1, 0, 0, 0, 1, 0, 0, 0, -1, 0, 0, 0, -1, 0, 1, 0, 0, 0, 0, 0};
  for (int i = 0; i < 3; ++i) {
    double ri = i == 0 ? x : (i == 1 ? y : z);
    double a0 = -s * ri, a1 = (s - 2 * c1 * it) * ri, a2 = c1 * it, a3 = (c - s * it) * ri, a4 = s * it;
    for (int k = 0; k < 9; ++k)
      J[i * 9 + k] = a0 * (k % 4 == 0) + a1 * rrt[k] + a2 * drrt[i * 9 + k] + a3 * rx[k] + a4 * drx[i * 9 + k];
  }
}

PNP_FN void rodrigues_R2r(const double* R, double* r) {
  double rx = R[7] - R[5], ry = R[2] - R[6], rz = R[3] - R[1];
  double s = sqrt((rx * rx + ry * ry + rz * rz) * 0.25);
  double c = (R[0] + R[4] + R[8] - 1) * 0.5;
  c = c > 1. ? 1. : (c < -1. ? -1. : c);
  double theta = det_acos(c);
  if (s < 1e-5) {
    if (c > 0) {
      r[0] = r[1] = r[2] = 0;
    } else {
      double t;
      t = (R[0] + 1) * 0.5; rx = sqrt(t > 0 ? t : 0);
      t = (R[4] + 1) * 0.5; ry = sqrt(t > 0 ? t : 0) * (R[1] < 0 ? -1. : 1.);
      t = (R[8] + 1) * 0.5; rz = sqrt(t > 0 ? t : 0) * (R[2] < 0 ? -1. : 1.);
      if (fabs(rx) < fabs(ry) && fabs(rx) < fabs(rz) && (R[5] > 0) != (ry * rz > 0)) rz = -rz;
      double nr = sqrt(rx * rx + ry * ry + rz * rz);
      theta /= nr;
      r[0] = rx * theta; r[1] = ry * theta; r[2] = rz * theta;
    }
  } else {
    double vth = 1 / (2 * s);
    vth *= theta;
    r[0] = rx * vth; r[1] = ry * vth; r[2] = rz * vth;
  }
}

/* ------------------------------------------------------------------ projections */
/* cv::projectPoints with zero distortion, float output (RANSAC error path) */
PNP_FN void project_f(const cam_t* k, const double* R, const double* t, const float* w, float* uv) {
  double X = R[0] * w[0] + R[1] * w[1] + R[2] * w[2] + t[0];
  double Y = R[3] * w[0] + R[4] * w[1] + R[5] * w[2] + t[1];
  double Z = R[6] * w[0] + R[7] * w[1] + R[8] * w[2] + t[2];
  double z = Z ? 1. / Z : 1.;
  uv[0] = (float)(X * z * k->fx + k->cx);
  uv[1] = (float)(Y * z * k->fy + k->cy);
}

PNP_FN float sq_err_f(const float* obs, const float* proj) {
  float dx = obs[0] - proj[0], dy = obs[1] - proj[1];
  return dx * dx + dy * dy;
}

/* np.linalg.norm(projected - observed, axis=-1) of one float32 point (UNC/utils/speed_eval_ceres.py
 * :143,164): float32 difference, squares, sum and root */
PNP_FN float repro_err_f(const float* obs, const float* proj) {
  const float dx = proj[0] - obs[0], dy = proj[1] - obs[1];
  const float dx2 = dx * dx, dy2 = dy * dy;
  return sqrtf(dx2 + dy2);
}

/* np.sum of a contiguous float32 vector: numpy's pairwise summation (sequential below 8
 * elements, 8 accumulators combined pairwise above), float32 throughout */
PNP_FN float np_sum_f32(const float* a, int n) {
  if (n < 8) {
    float r = 0.f;
    for (int i = 0; i < n; ++i) r += a[i];
    return r;
  }
  float r[8];
  for (int j = 0; j < 8; ++j) r[j] = a[j];
  int i = 8;
  for (; i < n - (n % 8); i += 8)
    for (int j = 0; j < 8; ++j) r[j] += a[i + j];
  float res = ((r[0] + r[1]) + (r[2] + r[3])) + ((r[4] + r[5]) + (r[6] + r[7]));
  for (; i < n; ++i) res += a[i];
  return res;
}

/* ------------------------------------------------------------------ polynomial roots */
PNP_FN int solve_deg2(double a, double b, double c, double* x1, double* x2) {
  double delta = b * b - 4 * a * c;
  if (delta < 0) return 0;
  double inv_2a = 0.5 / a;
  if (delta == 0) { *x1 = -b * inv_2a; *x2 = *x1; return 1; }
  double sd = sqrt(delta);
  *x1 = (-b + sd) * inv_2a;
  *x2 = (-b - sd) * inv_2a;
  return 2;
}

PNP_FN int solve_deg3(double a, double b, double c, double d, double* x0, double* x1, double* x2) {
  if (a == 0) {
    if (b == 0) {
      if (c == 0) return 0;
      *x0 = -d / c;
      return 1;
    }
    *x2 = 0;
    return solve_deg2(b, c, d, x0, x1);
  }
  double inv_a = 1. / a, b_a = inv_a * b, b_a2 = b_a * b_a, c_a = inv_a * c, d_a = inv_a * d;
  double Q = (3 * c_a - b_a2) / 9;
  double R = (9 * b_a * c_a - 27 * d_a - 2 * b_a * b_a2) / 54;
  double Q3 = Q * Q * Q, D = Q3 + R * R, b_a_3 = (1. / 3.) * b_a;
  if (Q == 0) {
    if (R == 0) { *x0 = *x1 = *x2 = -b_a_3; return 3; }
    *x0 = (2 * R >= 0 ? det_cbrt(2 * R) : NAN) - b_a_3; /* pow(<0, 1/3.) is NaN in OpenCV's code */
    return 1;
  }
  if (D <= 0) {
    double theta = det_acos(R / sqrt(-Q3)), sq = sqrt(-Q);
    *x0 = 2 * sq * det_cos(theta / 3.0) - b_a_3;
    *x1 = 2 * sq * det_cos((theta + 2 * 3.14159265358979323846) / 3.0) - b_a_3;
    *x2 = 2 * sq * det_cos((theta + 4 * 3.14159265358979323846) / 3.0) - b_a_3;
    return 3;
  }
  double AD = det_cbrt(fabs(R) + sqrt(D)) * (R > 0 ? 1 : (R < 0 ? -1 : 0));
  double BD = (AD == 0) ? 0 : -Q / AD;
  *x0 = AD + BD - b_a_3;
  return 1;
}

PNP_FN int solve_deg4(double a, double b, double c, double d, double e, double* x) {
  if (a == 0) { x[3] = 0; return solve_deg3(b, c, d, e, &x[0], &x[1], &x[2]); }
  double inv_a = 1. / a;
  b *= inv_a; c *= inv_a; d *= inv_a; e *= inv_a;
  double b2 = b * b, bc = b * c, b3 = b2 * b;
  double r0, r1, r2;
  int n = solve_deg3(1, -c, d * b - 4 * e, 4 * c * e - d * d - b2 * e, &r0, &r1, &r2);
  if (n == 0) return 0;
  double R2 = 0.25 * b2 - c + r0;
  if (R2 < 0) return 0;
  double R = sqrt(R2), inv_R = 1. / R;
  int nr = 0;
  double D2, E2;
  if (R < 10E-12) {
    double temp = r0 * r0 - 4 * e;
    if (temp < 0) D2 = E2 = -1;
    else {
      double st = sqrt(temp);
      D2 = 0.75 * b2 - 2 * c + 2 * st;
      E2 = D2 - 4 * st;
    }
  } else {
    double u = 0.75 * b2 - 2 * c - R2, v = 0.25 * inv_R * (4 * bc - 8 * d - b3);
    D2 = u + v;
    E2 = u - v;
  }
  double b_4 = 0.25 * b, R_2 = 0.5 * R;
  if (D2 >= 0) {
    double D = sqrt(D2), D_2 = 0.5 * D;
    nr = 2;
    x[0] = R_2 + D_2 - b_4;
    x[1] = x[0] - D;
  }
  if (E2 >= 0) {
    double E = sqrt(E2), E_2 = 0.5 * E;
    if (nr == 0) { x[0] = -R_2 + E_2 - b_4; x[1] = x[0] - E; nr = 2; }
    else { x[2] = -R_2 + E_2 - b_4; x[3] = x[2] - E; nr = 4; }
  }
  return nr;
}

/* ------------------------------------------------------------------ P3P (Gao, OpenCV p3p.cpp) */
PNP_FN int p3p_lengths(double lengths[4][3], const double dist[3], const double cosv[3]) {
  double p = cosv[0] * 2, q = cosv[1] * 2, r = cosv[2] * 2;
  double inv_d22 = 1. / (dist[2] * dist[2]);
  double a = inv_d22 * (dist[0] * dist[0]), b = inv_d22 * (dist[1] * dist[1]);
  double a2 = a * a, b2 = b * b, p2 = p * p, q2 = q * q, r2 = r * r;
  double pr = p * r, pqr = q * pr;
  if (p2 + q2 + r2 - pqr - 1 == 0) return 0;
  double ab = a * b, a_2 = 2 * a;
  double A = -2 * b + b2 + a2 + 1 + ab * (2 - r2) - a_2;
  if (A == 0) return 0;
  double a_4 = 4 * a;
  double B = q * (-2 * (ab + a2 + 1 - b) + r2 * ab + a_4) + pr * (b - b2 + ab);
  double C = q2 + b2 * (r2 + p2 - 2) - b * (p2 + pqr) - ab * (r2 + pqr) + (a2 - a_2) * (2 + q2) + 2;
  double D = pr * (ab - b2 + b) + q * ((p2 - 2) * b + 2 * (ab - a2) + a_4 - 2);
  double E = 1 + 2 * (b - a - ab) + b2 - b * p2 + a2;
  double temp = (p2 * (a - 1 + b) + r2 * (a - 1 - b) + pqr - a * pqr);
  double b0 = b * temp * temp;
  if (b0 == 0) return 0;
  double roots[4];
  int n = solve_deg4(A, B, C, D, E, roots);
  if (n == 0) return 0;
  int ns = 0;
  double r3 = r2 * r, pr2 = p * r2, r3q = r3 * q, inv_b0 = 1. / b0;
  for (int i = 0; i < n; ++i) {
    double x = roots[i];
    if (x <= 0) continue;
    double x2 = x * x;
    double b1 = ((1 - a - b) * x2 + (q * a - q) * x + 1 - a + b) *
                (((r3 * (a2 + ab * (2 - r2) - a_2 + b2 - 2 * b + 1)) * x +
                  (r3q * (2 * (b - a2) + a_4 + ab * (r2 - 2) - 2) + pr2 * (1 + a2 + 2 * (ab - a - b) + r2 * (b - b2) + b2))) * x2 +
                 (r3 * (q2 * (1 - 2 * a + a2) + r2 * (b2 - ab) - a_4 + 2 * (a2 - b2) + 2) + r * p2 * (b2 + 2 * (ab - b - a) + 1 + a2) +
                  pr2 * q * (a_4 + 2 * (b - ab - a2) - 2 - r2 * b)) * x +
                 2 * r3q * (a_2 - b - a2 + ab - 1) + pr2 * (q2 - a_4 + 2 * (a2 - b2) + r2 * b + q2 * (a2 - a_2) + 2) +
                 p2 * (p * (2 * (ab - a - b) + a2 + b2 + 1) + 2 * q * r * (b + a_2 - a2 - ab - 1)));
    if (b1 <= 0) continue;
    double y = inv_b0 * b1;
    double v = x2 + y * y - x * y * r;
    if (v <= 0) continue;
    double Z = dist[2] / sqrt(v);
    lengths[ns][0] = x * Z;
    lengths[ns][1] = y * Z;
    lengths[ns][2] = Z;
    ns++;
  }
  return ns;
}

/* Horn absolute orientation of 3 camera points M[i] onto world points w[i] */
PNP_FN void p3p_align(const double M[3][3], const double w[3][3], double R[9], double T[3]) {
  double Ce[3], Cs[3];
  for (int i = 0; i < 3; ++i) Ce[i] = (M[0][i] + M[1][i] + M[2][i]) / 3;
  for (int i = 0; i < 3; ++i) Cs[i] = (w[0][i] + w[1][i] + w[2][i]) / 3;
  double s[9];
  for (int j = 0; j < 3; ++j)
    for (int i = 0; i < 3; ++i)
      s[i * 3 + j] = (w[0][i] * M[0][j] + w[1][i] * M[1][j] + w[2][i] * M[2][j]) / 3 - Ce[j] * Cs[i];
  double Qs[16];
  Qs[0] = s[0] + s[4] + s[8];
  Qs[5] = s[0] - s[4] - s[8];
  Qs[10] = s[4] - s[8] - s[0];
  Qs[15] = s[8] - s[0] - s[4];
  Qs[4] = Qs[1] = s[5] - s[7];
  Qs[8] = Qs[2] = s[6] - s[2];
  Qs[12] = Qs[3] = s[1] - s[3];
  Qs[9] = Qs[6] = s[3] + s[1];
  Qs[13] = Qs[7] = s[6] + s[2];
  Qs[14] = Qs[11] = s[7] + s[5];
  double ev[4], U[16];
  jacobi_eig(4, Qs, ev, U);
  int ie = 0;
  for (int i = 1; i < 4; ++i) if (ev[i] > ev[ie]) ie = i;
  double q0 = U[0 * 4 + ie], q1 = U[1 * 4 + ie], q2 = U[2 * 4 + ie], q3 = U[3 * 4 + ie];
  R[0] = q0 * q0 + q1 * q1 - q2 * q2 - q3 * q3;
  R[1] = 2. * (q1 * q2 - q0 * q3);
  R[2] = 2. * (q1 * q3 + q0 * q2);
  R[3] = 2. * (q1 * q2 + q0 * q3);
  R[4] = q0 * q0 + q2 * q2 - q1 * q1 - q3 * q3;
  R[5] = 2. * (q2 * q3 - q0 * q1);
  R[6] = 2. * (q1 * q3 - q0 * q2);
  R[7] = 2. * (q2 * q3 + q0 * q1);
  R[8] = q0 * q0 + q3 * q3 - q1 * q1 - q2 * q2;
  for (int i = 0; i < 3; ++i) T[i] = Ce[i] - (R[i * 3] * Cs[0] + R[i * 3 + 1] * Cs[1] + R[i * 3 + 2] * Cs[2]);
}

/* solveP3P on exactly 4 points (p4p): best of up to 4 solutions by the 4th point.
 * img: float pixel points; wld: float world points.  Returns 1 and rvec/tvec, or 0. */
PNP_FN int p3p_solve4(const cam_t* k, const float* img, const float* wld, double* rvec, double* tvec) {
  /* undistortPoints (float output) then back to pixels in double (p3p::extract_points) */
  double mu[4], mv[4], X[4][3];
  for (int i = 0; i < 4; ++i) {
    float un = (float)((img[2 * i] - k->cx) * (1. / k->fx));
    float vn = (float)((img[2 * i + 1] - k->cy) * (1. / k->fy));
    mu[i] = un * k->fx + k->cx;
    mv[i] = vn * k->fy + k->cy;
    for (int j = 0; j < 3; ++j) X[i][j] = wld[3 * i + j];
  }
  double inv_fx = 1. / k->fx, inv_fy = 1. / k->fy, cx_fx = k->cx / k->fx, cy_fy = k->cy / k->fy;
  double ray[3][3];
  for (int i = 0; i < 3; ++i) {
    double u = inv_fx * mu[i] - cx_fx, v = inv_fy * mv[i] - cy_fy;
    double nrm = sqrt(u * u + v * v + 1), mk = 1. / nrm;
    ray[i][0] = u * mk; ray[i][1] = v * mk; ray[i][2] = mk;
  }
  double dist[3], cosv[3];
  dist[0] = sqrt((X[1][0] - X[2][0]) * (X[1][0] - X[2][0]) + (X[1][1] - X[2][1]) * (X[1][1] - X[2][1]) + (X[1][2] - X[2][2]) * (X[1][2] - X[2][2]));
  dist[1] = sqrt((X[0][0] - X[2][0]) * (X[0][0] - X[2][0]) + (X[0][1] - X[2][1]) * (X[0][1] - X[2][1]) + (X[0][2] - X[2][2]) * (X[0][2] - X[2][2]));
  dist[2] = sqrt((X[0][0] - X[1][0]) * (X[0][0] - X[1][0]) + (X[0][1] - X[1][1]) * (X[0][1] - X[1][1]) + (X[0][2] - X[1][2]) * (X[0][2] - X[1][2]));
  cosv[0] = ray[1][0] * ray[2][0] + ray[1][1] * ray[2][1] + ray[1][2] * ray[2][2];
  cosv[1] = ray[0][0] * ray[2][0] + ray[0][1] * ray[2][1] + ray[0][2] * ray[2][2];
  cosv[2] = ray[0][0] * ray[1][0] + ray[0][1] * ray[1][1] + ray[0][2] * ray[1][2];
  double lengths[4][3];
  int n = p3p_lengths(lengths, dist, cosv);
  if (n == 0) return 0;
  double Rs[4][9], ts[4][3];
  for (int i = 0; i < n; ++i) {
    double M[3][3];
    for (int j = 0; j < 3; ++j)
      for (int c = 0; c < 3; ++c) M[j][c] = lengths[i][j] * ray[j][c];
    p3p_align(M, X, Rs[i], ts[i]);
  }
  int best = 0;
  double minr = 0;
  for (int i = 0; i < n; ++i) {
    const double* R = Rs[i];
    double X3 = R[0] * X[3][0] + R[1] * X[3][1] + R[2] * X[3][2] + ts[i][0];
    double Y3 = R[3] * X[3][0] + R[4] * X[3][1] + R[5] * X[3][2] + ts[i][1];
    double Z3 = R[6] * X[3][0] + R[7] * X[3][1] + R[8] * X[3][2] + ts[i][2];
    double u3 = k->cx + k->fx * X3 / Z3, v3 = k->cy + k->fy * Y3 / Z3;
    double re = (u3 - mu[3]) * (u3 - mu[3]) + (v3 - mv[3]) * (v3 - mv[3]);
    if (i == 0 || minr > re) { best = i; minr = re; }
  }
  rodrigues_R2r(Rs[best], rvec);
  memcpy(tvec, ts[best], sizeof(double) * 3);
  return 1;
}

/* ------------------------------------------------------------------ EPnP (OpenCV epnp.cpp) */
typedef struct {
  int n;
  double fu, fv, uc, vc;
  double pws[3 * MAXN], us[2 * MAXN], alphas[4 * MAXN], pcs[3 * MAXN];
  double cws[4][3], ccs[4][3];
} epnp_t;

PNP_FN double dot3(const double* a, const double* b) { return a[0] * b[0] + a[1] * b[1] + a[2] * b[2]; }
PNP_FN double dist2(const double* a, const double* b) {
  return (a[0] - b[0]) * (a[0] - b[0]) + (a[1] - b[1]) * (a[1] - b[1]) + (a[2] - b[2]) * (a[2] - b[2]);
}

PNP_FN void epnp_control_points(epnp_t* e) {
  for (int j = 0; j < 3; ++j) e->cws[0][j] = 0;
  for (int i = 0; i < e->n; ++i)
    for (int j = 0; j < 3; ++j) e->cws[0][j] += e->pws[3 * i + j];
  for (int j = 0; j < 3; ++j) e->cws[0][j] /= e->n;
  double m[9] = {0};
  for (int i = 0; i < e->n; ++i) {
    double d[3];
    for (int j = 0; j < 3; ++j) d[j] = e->pws[3 * i + j] - e->cws[0][j];
    for (int a = 0; a < 3; ++a)
      for (int b = 0; b < 3; ++b) m[a * 3 + b] += d[a] * d[b];
  }
  double dc[3], uct[9];
  sym_eig_desc(3, m, dc, uct);
  for (int i = 1; i < 4; ++i) {
    double kk = sqrt((dc[i - 1] > 0 ? dc[i - 1] : 0) / e->n);
    for (int j = 0; j < 3; ++j) e->cws[i][j] = e->cws[0][j] + kk * uct[3 * (i - 1) + j];
  }
}

PNP_FN void inv3_pinv(const double* A, double* Ai) {
  double U[9], s[3], V[9];
  svd3(A, U, s, V);
  double thr = s[0] * DBL_EPSILON * 8;
  for (int i = 0; i < 3; ++i)
    for (int j = 0; j < 3; ++j) {
      double acc = 0;
      for (int k = 0; k < 3; ++k)
        if (s[k] > thr) acc += V[i * 3 + k] * U[j * 3 + k] / s[k];
      Ai[i * 3 + j] = acc;
    }
}

PNP_FN void epnp_barycentric(epnp_t* e) {
  double cc[9], ci[9];
  for (int i = 0; i < 3; ++i)
    for (int j = 1; j < 4; ++j) cc[3 * i + j - 1] = e->cws[j][i] - e->cws[0][i];
  inv3_pinv(cc, ci);
  for (int i = 0; i < e->n; ++i) {
    const double* pi = e->pws + 3 * i;
    double* a = e->alphas + 4 * i;
    for (int j = 0; j < 3; ++j)
      a[1 + j] = ci[3 * j] * (pi[0] - e->cws[0][0]) + ci[3 * j + 1] * (pi[1] - e->cws[0][1]) + ci[3 * j + 2] * (pi[2] - e->cws[0][2]);
    a[0] = 1.0f - a[1] - a[2] - a[3];
  }
}

PNP_FN void epnp_ccs(epnp_t* e, const double* betas, const double* ut) {
  for (int i = 0; i < 4; ++i) e->ccs[i][0] = e->ccs[i][1] = e->ccs[i][2] = 0.0f;
  for (int i = 0; i < 4; ++i) {
    const double* v = ut + 12 * (11 - i);
    for (int j = 0; j < 4; ++j)
      for (int k = 0; k < 3; ++k) e->ccs[j][k] += betas[i] * v[3 * j + k];
  }
  for (int i = 0; i < e->n; ++i) {
    const double* a = e->alphas + 4 * i;
    double* pc = e->pcs + 3 * i;
    for (int j = 0; j < 3; ++j) pc[j] = a[0] * e->ccs[0][j] + a[1] * e->ccs[1][j] + a[2] * e->ccs[2][j] + a[3] * e->ccs[3][j];
  }
}

PNP_FN double epnp_R_and_t(epnp_t* e, const double* ut, const double* betas, double* R, double* t) {
  epnp_ccs(e, betas, ut);
  if (e->pcs[2] < 0.0) {
    for (int i = 0; i < 4; ++i)
      for (int j = 0; j < 3; ++j) e->ccs[i][j] = -e->ccs[i][j];
    for (int i = 0; i < 3 * e->n; ++i) e->pcs[i] = -e->pcs[i];
  }
  double pc0[3] = {0, 0, 0}, pw0[3] = {0, 0, 0};
  for (int i = 0; i < e->n; ++i)
    for (int j = 0; j < 3; ++j) { pc0[j] += e->pcs[3 * i + j]; pw0[j] += e->pws[3 * i + j]; }
  for (int j = 0; j < 3; ++j) { pc0[j] /= e->n; pw0[j] /= e->n; }
  double abt[9] = {0};
  for (int i = 0; i < e->n; ++i) {
    const double* pc = e->pcs + 3 * i;
    const double* pw = e->pws + 3 * i;
    for (int j = 0; j < 3; ++j) {
      abt[3 * j] += (pc[j] - pc0[j]) * (pw[0] - pw0[0]);
      abt[3 * j + 1] += (pc[j] - pc0[j]) * (pw[1] - pw0[1]);
      abt[3 * j + 2] += (pc[j] - pc0[j]) * (pw[2] - pw0[2]);
    }
  }
  double U[9], s[3], V[9];
  svd3(abt, U, s, V);
  for (int i = 0; i < 3; ++i)
    for (int j = 0; j < 3; ++j) R[i * 3 + j] = U[i * 3] * V[j * 3] + U[i * 3 + 1] * V[j * 3 + 1] + U[i * 3 + 2] * V[j * 3 + 2];
  double det = R[0] * R[4] * R[8] + R[1] * R[5] * R[6] + R[2] * R[3] * R[7] - R[2] * R[4] * R[6] - R[1] * R[3] * R[8] - R[0] * R[5] * R[7];
  if (det < 0) { R[6] = -R[6]; R[7] = -R[7]; R[8] = -R[8]; }
  for (int i = 0; i < 3; ++i) t[i] = pc0[i] - dot3(R + 3 * i, pw0);
  double sum2 = 0;
  for (int i = 0; i < e->n; ++i) {
    const double* pw = e->pws + 3 * i;
    double Xc = dot3(R, pw) + t[0], Yc = dot3(R + 3, pw) + t[1], iz = 1.0 / (dot3(R + 6, pw) + t[2]);
    double ue = e->uc + e->fu * Xc * iz, ve = e->vc + e->fv * Yc * iz;
    double u = e->us[2 * i], v = e->us[2 * i + 1];
    sum2 += sqrt((u - ue) * (u - ue) + (v - ve) * (v - ve));
  }
  return sum2 / e->n;
}

PNP_FN void epnp_qr_solve(double* A, double* b, double* X) {
  const int nr = 6, nc = 4;
  double A1[6], A2[6];
  double* pA = A;
  for (int k = 0; k < nc; ++k) {
    double* ppAkk = pA + k * nc + k;
    double eta = fabs(*ppAkk);
    for (int i = k + 1; i < nr; ++i) { double elt = fabs(pA[i * nc + k]); if (eta < elt) eta = elt; }
    if (eta == 0) return; /* singular: X keeps its previous content (OpenCV) */
    double sum2 = 0, inv_eta = 1. / eta;
    for (int i = k; i < nr; ++i) { pA[i * nc + k] *= inv_eta; sum2 += pA[i * nc + k] * pA[i * nc + k]; }
    double sigma = sqrt(sum2);
    if (*ppAkk < 0) sigma = -sigma;
    *ppAkk += sigma;
    A1[k] = sigma * *ppAkk;
    A2[k] = -eta * sigma;
    for (int j = k + 1; j < nc; ++j) {
      double sum = 0;
      for (int i = k; i < nr; ++i) sum += pA[i * nc + k] * pA[i * nc + j];
      double tau = sum / A1[k];
      for (int i = k; i < nr; ++i) pA[i * nc + j] -= tau * pA[i * nc + k];
    }
  }
  for (int j = 0; j < nc; ++j) {
    double tau = 0;
    for (int i = j; i < nr; ++i) tau += pA[i * nc + j] * b[i];
    tau /= A1[j];
    for (int i = j; i < nr; ++i) b[i] -= tau * pA[i * nc + j];
  }
  X[nc - 1] = b[nc - 1] / A2[nc - 1];
  for (int i = nc - 2; i >= 0; --i) {
    double sum = 0;
    for (int j = i + 1; j < nc; ++j) sum += pA[i * nc + j] * X[j];
    X[i] = (b[i] - sum) / A2[i];
  }
}

PNP_FN void epnp_gauss_newton(const double* L, const double* rho, double* betas) {
  double x[4] = {0, 0, 0, 0};
  for (int it = 0; it < 5; ++it) {
    double A[24], b[6];
    for (int i = 0; i < 6; ++i) {
      const double* l = L + 10 * i;
      A[i * 4 + 0] = 2 * l[0] * betas[0] + l[1] * betas[1] + l[3] * betas[2] + l[6] * betas[3];
      A[i * 4 + 1] = l[1] * betas[0] + 2 * l[2] * betas[1] + l[4] * betas[2] + l[7] * betas[3];
      A[i * 4 + 2] = l[3] * betas[0] + l[4] * betas[1] + 2 * l[5] * betas[2] + l[8] * betas[3];
      A[i * 4 + 3] = l[6] * betas[0] + l[7] * betas[1] + l[8] * betas[2] + 2 * l[9] * betas[3];
      b[i] = rho[i] - (l[0] * betas[0] * betas[0] + l[1] * betas[0] * betas[1] + l[2] * betas[1] * betas[1] +
                       l[3] * betas[0] * betas[2] + l[4] * betas[1] * betas[2] + l[5] * betas[2] * betas[2] +
                       l[6] * betas[0] * betas[3] + l[7] * betas[1] * betas[3] + l[8] * betas[2] * betas[3] +
                       l[9] * betas[3] * betas[3]);
    }
    epnp_qr_solve(A, b, x);
    for (int i = 0; i < 4; ++i) betas[i] += x[i];
  }
}

/* EPnP pose from n >= 4 correspondences (pixel points given as double, OpenCV us[] convention) */
/* EPnP in three stages (setup -> M^T M + 12x12 eigen-decomposition -> betas / pose) so the
 * device solver can run the middle stage with a whole wave (csrc/pnp.hip) on the same math. */
PNP_FN void epnp_setup(epnp_t* e, const cam_t* k, int n, const double* wld, const double* img_norm) {
  e->n = n;
  e->fu = k->fx; e->fv = k->fy; e->uc = k->cx; e->vc = k->cy;
  for (int i = 0; i < n; ++i) {
    for (int j = 0; j < 3; ++j) e->pws[3 * i + j] = wld[3 * i + j];
    e->us[2 * i] = img_norm[2 * i] * e->fu + e->uc;
    e->us[2 * i + 1] = img_norm[2 * i + 1] * e->fv + e->vc;
  }
  epnp_control_points(e);
  epnp_barycentric(e);
}

/* one entry (a, b) of M^T M, accumulated over the correspondences in order */
PNP_FN double epnp_mtm_entry(const epnp_t* e, int a, int b) {
  double acc = 0;
  for (int i = 0; i < e->n; ++i) {
    const double* as = e->alphas + 4 * i;
    const double u = e->us[2 * i], v = e->us[2 * i + 1];
    const int ja = a / 3, ca = a % 3, jb = b / 3, cb = b % 3;
    const double m1a = ca == 0 ? as[ja] * e->fu : (ca == 1 ? 0.0 : as[ja] * (e->uc - u));
    const double m1b = cb == 0 ? as[jb] * e->fu : (cb == 1 ? 0.0 : as[jb] * (e->uc - u));
    const double m2a = ca == 0 ? 0.0 : (ca == 1 ? as[ja] * e->fv : as[ja] * (e->vc - v));
    const double m2b = cb == 0 ? 0.0 : (cb == 1 ? as[jb] * e->fv : as[jb] * (e->vc - v));
    acc += m1a * m1b + m2a * m2b;
  }
  return acc;
}

PNP_FN void epnp_finish(epnp_t* e, const double* ut, double* R, double* t);

PNP_FN void epnp_pose(const cam_t* k, int n, const double* wld, const double* img_norm, double* R, double* t) {
  epnp_t e;
  epnp_setup(&e, k, n, wld, img_norm);
  double mtm[144];
  for (int a = 0; a < 12; ++a)
    for (int b = 0; b < 12; ++b) mtm[a * 12 + b] = epnp_mtm_entry(&e, a, b);
  double d[12], ut[144];
  sym_eig_desc(12, mtm, d, ut);
  epnp_finish(&e, ut, R, t);
}

/* L_6x10 and rho from the four null-space vectors (OpenCV compute_L_6x10 / compute_rho) */
PNP_FN void epnp_L_rho(const epnp_t* ep, const double* ut, double* L, double* rho) {
  const double(*cws)[3] = ep->cws;
  const double* v[4] = {ut + 12 * 11, ut + 12 * 10, ut + 12 * 9, ut + 12 * 8};
  double dv[4][6][3];
  for (int i = 0; i < 4; ++i) {
    int a = 0, b = 1;
    for (int j = 0; j < 6; ++j) {
      for (int c = 0; c < 3; ++c) dv[i][j][c] = v[i][3 * a + c] - v[i][3 * b + c];
      b++;
      if (b > 3) { a++; b = a + 1; }
    }
  }
  for (int i = 0; i < 6; ++i) {
    double* row = L + 10 * i;
    row[0] = dot3(dv[0][i], dv[0][i]);
    row[1] = 2.0f * dot3(dv[0][i], dv[1][i]);
    row[2] = dot3(dv[1][i], dv[1][i]);
    row[3] = 2.0f * dot3(dv[0][i], dv[2][i]);
    row[4] = 2.0f * dot3(dv[1][i], dv[2][i]);
    row[5] = dot3(dv[2][i], dv[2][i]);
    row[6] = 2.0f * dot3(dv[0][i], dv[3][i]);
    row[7] = 2.0f * dot3(dv[1][i], dv[3][i]);
    row[8] = 2.0f * dot3(dv[2][i], dv[3][i]);
    row[9] = dot3(dv[3][i], dv[3][i]);
  }
  rho[0] = dist2(cws[0], cws[1]); rho[1] = dist2(cws[0], cws[2]); rho[2] = dist2(cws[0], cws[3]);
  rho[3] = dist2(cws[1], cws[2]); rho[4] = dist2(cws[1], cws[3]); rho[5] = dist2(cws[2], cws[3]);
}

/* beta approximation `which` (1: [B11 B12 B13 B14], 2: [B11 B12 B22], 3: [B11 B12 B22 B13 B23]),
 * Gauss-Newton refinement, pose and mean reprojection error.  The three are independent, so the
 * device solver runs them on three lanes. */
PNP_FN double epnp_approx(const epnp_t* e0, const double* ut, const double* L, const double* rho, int which, double* R,
                          double* t) {
  epnp_t e = *e0;
  double bb[4] = {0, 0, 0, 0};
  if (which == 1) {
    double A[24], x[4];
    for (int i = 0; i < 6; ++i) { A[i * 4] = L[10 * i]; A[i * 4 + 1] = L[10 * i + 1]; A[i * 4 + 2] = L[10 * i + 3]; A[i * 4 + 3] = L[10 * i + 6]; }
    lstsq_pinv(6, 4, A, rho, x);
    if (x[0] < 0) { bb[0] = sqrt(-x[0]); bb[1] = -x[1] / bb[0]; bb[2] = -x[2] / bb[0]; bb[3] = -x[3] / bb[0]; }
    else { bb[0] = sqrt(x[0]); bb[1] = x[1] / bb[0]; bb[2] = x[2] / bb[0]; bb[3] = x[3] / bb[0]; }
  } else if (which == 2) {
    double A[18], x[3];
    for (int i = 0; i < 6; ++i) { A[i * 3] = L[10 * i]; A[i * 3 + 1] = L[10 * i + 1]; A[i * 3 + 2] = L[10 * i + 2]; }
    lstsq_pinv(6, 3, A, rho, x);
    if (x[0] < 0) { bb[0] = sqrt(-x[0]); bb[1] = (x[2] < 0) ? sqrt(-x[2]) : 0.0; }
    else { bb[0] = sqrt(x[0]); bb[1] = (x[2] > 0) ? sqrt(x[2]) : 0.0; }
    if (x[1] < 0) bb[0] = -bb[0];
    bb[2] = 0.0; bb[3] = 0.0;
  } else {
    double A[30], x[5];
    for (int i = 0; i < 6; ++i)
      for (int c = 0; c < 5; ++c) A[i * 5 + c] = L[10 * i + c];
    lstsq_pinv(6, 5, A, rho, x);
    if (x[0] < 0) { bb[0] = sqrt(-x[0]); bb[1] = (x[2] < 0) ? sqrt(-x[2]) : 0.0; }
    else { bb[0] = sqrt(x[0]); bb[1] = (x[2] > 0) ? sqrt(x[2]) : 0.0; }
    if (x[1] < 0) bb[0] = -bb[0];
    bb[2] = x[3] / bb[0];
    bb[3] = 0.0;
  }
  epnp_gauss_newton(L, rho, bb);
  return epnp_R_and_t(&e, ut, bb, R, t);
}

/* OpenCV's choice among the three: N = 1; if err2 < err1 N = 2; if err3 < errN N = 3 */
PNP_FN int epnp_pick(const double* err /* [1..3] */) {
  int N = 1;
  if (err[2] < err[1]) N = 2;
  if (err[3] < err[N]) N = 3;
  return N;
}

PNP_FN void epnp_finish(epnp_t* e, const double* ut, double* R, double* t) {
  double L[60], rho[6], err[4] = {0, 0, 0, 0}, Rs[4][9], ts[4][3];
  epnp_L_rho(e, ut, L, rho);
  for (int w = 1; w <= 3; ++w) err[w] = epnp_approx(e, ut, L, rho, w, Rs[w], ts[w]);
  const int N = epnp_pick(err);
  memcpy(R, Rs[N], sizeof(double) * 9);
  memcpy(t, ts[N], sizeof(double) * 3);
}

/* solvePnPGeneric(EPNP): float (or double) inputs -> rvec/tvec.  `img_is_float` selects the
 * float32 rounding of undistortPoints' output (OpenCV keeps the input depth). */
PNP_FN void epnp_solve(const cam_t* k, int n, const double* wld, const double* img, int img_is_float, double* rvec,
                       double* tvec) {
  double nrm[2 * MAXN], R[9];
  for (int i = 0; i < n; ++i) {
    double un = (img[2 * i] - k->cx) * (1. / k->fx), vn = (img[2 * i + 1] - k->cy) * (1. / k->fy);
    if (img_is_float) { un = (float)un; vn = (float)vn; }
    nrm[2 * i] = un; nrm[2 * i + 1] = vn;
  }
  epnp_pose(k, n, wld, nrm, R, tvec);
  rodrigues_R2r(R, rvec);
}

/* ------------------------------------------------------------------ LM refinement */
/* cvFindExtrinsicCameraParams2(useExtrinsicGuess=1) with CvLevMarq, pixel residuals */
PNP_FN void project_jac(const cam_t* k, const double* p, int n, const double* wld, double* proj, double* J) {
  double R[9], dRdr[27];
  rodrigues_r2R(p, R);
  rodrigues_jac(p, dRdr);
  const double* t = p + 3;
  for (int i = 0; i < n; ++i) {
    const double* M = wld + 3 * i;
    double X = R[0] * M[0] + R[1] * M[1] + R[2] * M[2] + t[0];
    double Y = R[3] * M[0] + R[4] * M[1] + R[5] * M[2] + t[1];
    double Z = R[6] * M[0] + R[7] * M[1] + R[8] * M[2] + t[2];
    double z = Z ? 1. / Z : 1;
    double x = X * z, y = Y * z;
    proj[2 * i] = x * k->fx + k->cx;
    proj[2 * i + 1] = y * k->fy + k->cy;
    if (!J) continue;
    double* Ju = J + (2 * i) * 6;
    double* Jv = J + (2 * i + 1) * 6;
    for (int j = 0; j < 3; ++j) {
      const double* d = dRdr + 9 * j;
      double dX = d[0] * M[0] + d[1] * M[1] + d[2] * M[2];
      double dY = d[3] * M[0] + d[4] * M[1] + d[5] * M[2];
      double dZ = d[6] * M[0] + d[7] * M[1] + d[8] * M[2];
      Ju[j] = k->fx * (z * dX - x * z * dZ);
      Jv[j] = k->fy * (z * dY - y * z * dZ);
    }
    Ju[3] = k->fx * z; Ju[4] = 0; Ju[5] = -k->fx * x * z;
    Jv[3] = 0; Jv[4] = k->fy * z; Jv[5] = -k->fy * y * z;
  }
}

PNP_FN void lm_refine(const cam_t* k, int n, const double* wld, const double* img, double* rvec, double* tvec) {
  double param[6] = {rvec[0], rvec[1], rvec[2], tvec[0], tvec[1], tvec[2]}, prev[6];
  double J[2 * MAXN * 6], proj[2 * MAXN], err[2 * MAXN];
  double JtJ[36], JtErr[6];
  int lambdaLg10 = -3, iters = 0;
  double prevErrNorm = DBL_MAX;
  const int m = 2 * n;
  /* state CALC_J */
  project_jac(k, param, n, wld, proj, J);
  for (;;) {
    for (int i = 0; i < m; ++i) err[i] = proj[i] - img[i];
    for (int a = 0; a < 6; ++a) {
      double s = 0;
      for (int i = 0; i < m; ++i) s += J[i * 6 + a] * err[i];
      JtErr[a] = s;
      for (int b = 0; b < 6; ++b) {
        double q = 0;
        for (int i = 0; i < m; ++i) q += J[i * 6 + a] * J[i * 6 + b];
        JtJ[a * 6 + b] = q;
      }
    }
    memcpy(prev, param, sizeof prev);
    if (iters == 0) {
      double s = 0;
      for (int i = 0; i < m; ++i) s += err[i] * err[i];
      prevErrNorm = sqrt(s);
    }
    double errNorm;
    for (;;) { /* step + CHECK_ERR, retrying with larger lambda */
      double lambda = det_pow10i(lambdaLg10);
      double S[36], dx[6];
      memcpy(S, JtJ, sizeof S);
      for (int i = 0; i < 6; ++i) S[i * 6 + i] *= 1. + lambda;
      sym_solve(6, S, JtErr, dx);
      for (int i = 0; i < 6; ++i) param[i] = prev[i] - dx[i];
      project_jac(k, param, n, wld, proj, NULL);
      double s = 0;
      for (int i = 0; i < m; ++i) { double r = proj[i] - img[i]; s += r * r; }
      errNorm = sqrt(s);
      if (errNorm > prevErrNorm && ++lambdaLg10 <= 16) continue;
      break;
    }
    lambdaLg10 = lambdaLg10 - 1 > -16 ? lambdaLg10 - 1 : -16;
    double dn = 0, pn = 0;
    for (int i = 0; i < 6; ++i) { dn += (param[i] - prev[i]) * (param[i] - prev[i]); pn += prev[i] * prev[i]; }
    double rel = sqrt(dn) / (sqrt(pn) + DBL_EPSILON);
    if (++iters >= 20 || rel < FLT_EPSILON) break;
    prevErrNorm = errNorm;
    project_jac(k, param, n, wld, proj, J);
  }
  memcpy(rvec, param, sizeof(double) * 3);
  memcpy(tvec, param + 3, sizeof(double) * 3);
}

/* sigma-weighted Huber LM in normalised coordinates (UNC ceres_pnp restatement, UNPINNED):
 * residual_i = w_i * (x_obs - x_proj) per axis, Huber(delta) robust loss, <= 20 LM iterations. */
PNP_FN void sigma_lm(const cam_t* k, int n, const double* wld, const double* img, const double* sig, double delta,
                     double* rvec, double* tvec) {
  double xn[2 * MAXN], w[2 * MAXN];
  float w1[2 * MAXN], sum[2] = {0.f, 0.f};
  /* the reference computes the weights with numpy on the float32 sigmas (UNC/utils/speed_eval.py
   * :283-288): float32 sqrt, + 1e-6 and 1 / x in float32, the axis-0 sum row by row in float32,
   * the division in float32 (pinned by tests/golden/solver_front_ref.npz sig_cost) */
  for (int i = 0; i < n; ++i) {
    xn[2 * i] = (float)((img[2 * i] - k->cx) * (1. / k->fx));
    xn[2 * i + 1] = (float)((img[2 * i + 1] - k->cy) * (1. / k->fy));
    for (int a = 0; a < 2; ++a) {
      w1[2 * i + a] = 1.0f / (sqrtf((float)sig[2 * i + a]) + 1e-6f);
      sum[a] = sum[a] + w1[2 * i + a];
    }
  }
  for (int i = 0; i < n; ++i) for (int a = 0; a < 2; ++a) w[2 * i + a] = (double)(w1[2 * i + a] / sum[a]);
  cam_t unit = {1, 1, 0, 0};
  double param[6] = {rvec[0], rvec[1], rvec[2], tvec[0], tvec[1], tvec[2]};
  double mu = 1e-4, nu = 2;
  double J[2 * MAXN * 6], proj[2 * MAXN];
  const int m = 2 * n;
  double cost_prev = 0;
  for (int it = 0; it < 20; ++it) {
    project_jac(&unit, param, n, wld, proj, J);
    double g[6] = {0}, H[36] = {0}, cost = 0;
    for (int i = 0; i < m; ++i) {
      double r = w[i] * (proj[i] - xn[i]);
      double r2 = r * r, rho1 = 1;
      if (r2 > delta * delta) { double s = sqrt(r2); cost += 2 * delta * s - delta * delta; rho1 = delta / s; }
      else cost += r2;
      for (int a = 0; a < 6; ++a) {
        double ja = w[i] * J[i * 6 + a];
        g[a] += rho1 * ja * r;
        for (int b = 0; b < 6; ++b) H[a * 6 + b] += rho1 * ja * w[i] * J[i * 6 + b];
      }
    }
    if (it == 0) cost_prev = cost;
    double S[36], dx[6], trial[6];
    memcpy(S, H, sizeof S);
    for (int a = 0; a < 6; ++a) S[a * 6 + a] += mu * (H[a * 6 + a] > 1e-12 ? H[a * 6 + a] : 1e-12);
    sym_solve(6, S, g, dx);
    for (int a = 0; a < 6; ++a) trial[a] = param[a] - dx[a];
    project_jac(&unit, trial, n, wld, proj, NULL);
    double cost_new = 0;
    for (int i = 0; i < m; ++i) {
      double r = w[i] * (proj[i] - xn[i]), r2 = r * r;
      cost_new += r2 > delta * delta ? 2 * delta * sqrt(r2) - delta * delta : r2;
    }
    if (cost_new < cost_prev) {
      memcpy(param, trial, sizeof param);
      double dn = 0, pn = 0;
      for (int a = 0; a < 6; ++a) { dn += dx[a] * dx[a]; pn += param[a] * param[a]; }
      mu *= 1. / 3.; nu = 2;
      if (cost_prev - cost_new < 1e-6 * cost_prev || sqrt(dn) < 1e-8 * (sqrt(pn) + 1e-8)) { cost_prev = cost_new; break; }
      cost_prev = cost_new;
    } else {
      mu *= nu; nu *= 2;
    }
  }
  memcpy(rvec, param, sizeof(double) * 3);
  memcpy(tvec, param + 3, sizeof(double) * 3);
}

/* ------------------------------------------------------------------ RANSAC */
PNP_FN double ransac_update(double p, double ep, int mp, int maxIters) {
  p = p > 0 ? p : 0; p = p < 1 ? p : 1;
  ep = ep > 0 ? ep : 0; ep = ep < 1 ? ep : 1;
  double num = 1. - p > DBL_MIN ? 1. - p : DBL_MIN;
  double pw = 1.0;
  for (int i = 0; i < mp; ++i) pw *= 1. - ep;
  double denom = 1. - pw;
  if (denom < DBL_MIN) return 0;
  num = det_log(num);
  denom = det_log(denom);
  return (denom >= 0 || -num >= maxIters * (-denom)) ? maxIters : (int)det_rint(num / denom);
}

/* ------------------------------------------------------------------ Blender 2.81 mat3_to_quat */
PNP_FN void blender_quat(const double* Rd, float* q) {
  float m[3][3]; /* Blender column-major: m[col][row] */
  for (int r = 0; r < 3; ++r)
    for (int c = 0; c < 3; ++c) m[c][r] = (float)Rd[r * 3 + c];
  for (int c = 0; c < 3; ++c) { /* normalize_m3: normalise each axis (column) */
    float d = m[c][0] * m[c][0] + m[c][1] * m[c][1] + m[c][2] * m[c][2];
    if (d > 1.0e-35f) { d = sqrtf(d); m[c][0] /= d; m[c][1] /= d; m[c][2] /= d; }
    else { m[c][0] = m[c][1] = m[c][2] = 0.f; }
  }
  double tr = 0.25 * (double)(1.0f + m[0][0] + m[1][1] + m[2][2]), s;
  if (tr > (double)1e-4f) {
    s = sqrt(tr);
    q[0] = (float)s;
    s = 1.0 / (4.0 * s);
    q[1] = (float)((double)(m[1][2] - m[2][1]) * s);
    q[2] = (float)((double)(m[2][0] - m[0][2]) * s);
    q[3] = (float)((double)(m[0][1] - m[1][0]) * s);
  } else if (m[0][0] > m[1][1] && m[0][0] > m[2][2]) {
    s = 2.0f * sqrtf(1.0f + m[0][0] - m[1][1] - m[2][2]);
    q[1] = (float)(0.25 * s);
    s = 1.0 / s;
    q[0] = (float)((double)(m[1][2] - m[2][1]) * s);
    q[2] = (float)((double)(m[1][0] + m[0][1]) * s);
    q[3] = (float)((double)(m[2][0] + m[0][2]) * s);
  } else if (m[1][1] > m[2][2]) {
    s = 2.0f * sqrtf(1.0f - m[0][0] + m[1][1] - m[2][2]);
    q[2] = (float)(0.25 * s);
    s = 1.0 / s;
    q[0] = (float)((double)(m[2][0] - m[0][2]) * s);
    q[1] = (float)((double)(m[1][0] + m[0][1]) * s);
    q[3] = (float)((double)(m[2][1] + m[1][2]) * s);
  } else {
    s = 2.0f * sqrtf(1.0f - m[0][0] - m[1][1] + m[2][2]);
    q[3] = (float)(0.25 * s);
    s = 1.0 / s;
    q[0] = (float)((double)(m[0][1] - m[1][0]) * s);
    q[1] = (float)((double)(m[2][0] + m[0][2]) * s);
    q[2] = (float)((double)(m[2][1] + m[1][2]) * s);
  }
  float len = sqrtf(q[0] * q[0] + q[1] * q[1] + q[2] * q[2] + q[3] * q[3]);
  if (len != 0.0f) { float f = 1.0f / len; q[0] *= f; q[1] *= f; q[2] *= f; q[3] *= f; }
  else { q[1] = 1.0f; q[0] = q[2] = q[3] = 0.0f; }
}

