// Batched PnP-RANSAC for Trainer.get_pose (tools/trainer.py:383-438): one workgroup per crop.
//
//   obj[i] = float( xyz[b, :, choose[b, sel[b, i]]] * extent[b] + lfborder[b] )   (f64 math, then
//            f32 like cv::solvePnPRansac's CV_32F conversion of objectPoints)
//   img[i] = (x_map_choosed[b, sel[b, i]], y_map_choosed[b, sel[b, i]])
//   H hypotheses: EPnP on 5 correspondences each (one thread per hypothesis, f64),
//   score: #{ i : ||proj(R_h, t_h, obj_i) - img_i||^2 <= thr^2 } (f32, FMA-free, the same
//   expression as oracle/pnp_ref.c), best = most inliers / lowest h, accepted with >= 5
//   inliers (ptsetreg.cpp: goodCount > max(maxGoodCount, modelPoints - 1)),
//   refine: EPnP on every inlier of the best hypothesis; R as a rotation matrix (the
//   reference's Rodrigues round trip rvec -> kornia R is the identity map on R).
// Subsets come from the caller (krrn_ransac_subsets or explicit test inputs) so the GPU and
// the CPU oracle score identical hypotheses.
#include <math.h>

#include "krrn_common.h"

namespace {

constexpr int kPnpThreads = 128;
constexpr int kPnpMaxP = 1024;

struct Cam {
  double fu, fv, uc, vc;
};

__device__ void jacobi_eig(double* A, int n, double* w, double* V) {
  for (int i = 0; i < n; ++i)
    for (int j = 0; j < n; ++j) V[i * n + j] = (i == j) ? 1.0 : 0.0;
  for (int sweep = 0; sweep < 40; ++sweep) {
    double off = 0.0, tot = 0.0;
    for (int p = 0; p < n; ++p)
      for (int q = 0; q < n; ++q) {
        const double a2 = A[p * n + q] * A[p * n + q];
        tot += a2;
        if (p != q) off += a2;
      }
    if (off <= 1e-30 * tot || off < 1e-300) break;
    for (int p = 0; p < n; ++p) {
      for (int q = p + 1; q < n; ++q) {
        const double apq = A[p * n + q];
        if (fabs(apq) < 1e-300) continue;
        const double app = A[p * n + p], aqq = A[q * n + q];
        const double theta = (aqq - app) / (2.0 * apq);
        const double t = (theta >= 0 ? 1.0 : -1.0) / (fabs(theta) + sqrt(theta * theta + 1.0));
        const double c = 1.0 / sqrt(t * t + 1.0), s = t * c;
        for (int k = 0; k < n; ++k) {
          const double akp = A[k * n + p], akq = A[k * n + q];
          A[k * n + p] = c * akp - s * akq;
          A[k * n + q] = s * akp + c * akq;
        }
        for (int k = 0; k < n; ++k) {
          const double apk = A[p * n + k], aqk = A[q * n + k];
          A[p * n + k] = c * apk - s * aqk;
          A[q * n + k] = s * apk + c * aqk;
        }
        for (int k = 0; k < n; ++k) {
          const double vkp = V[k * n + p], vkq = V[k * n + q];
          V[k * n + p] = c * vkp - s * vkq;
          V[k * n + q] = s * vkp + c * vkq;
        }
      }
    }
  }
  // selection sort (descending) of eigenpairs; eigenvectors become rows of V
  for (int i = 0; i < n; ++i) w[i] = A[i * n + i];
  for (int i = 0; i < n; ++i) {
    int m = i;
    for (int j = i + 1; j < n; ++j)
      if (w[j] > w[m]) m = j;
    if (m != i) {
      const double tw = w[i]; w[i] = w[m]; w[m] = tw;
      for (int k = 0; k < n; ++k) {
        const double tv = V[k * n + i]; V[k * n + i] = V[k * n + m]; V[k * n + m] = tv;
      }
    }
  }
  for (int i = 0; i < n; ++i)
    for (int j = i + 1; j < n; ++j) {
      const double tv = V[i * n + j]; V[i * n + j] = V[j * n + i]; V[j * n + i] = tv;
    }
}

__device__ void lsq_solve(const double* A, int m, int n, const double* b, double* x) {
  double AtA[25], w[5], V[25], Atb[5];
  for (int i = 0; i < n; ++i) {
    for (int j = 0; j < n; ++j) {
      double s = 0.0;
      for (int k = 0; k < m; ++k) s += A[k * n + i] * A[k * n + j];
      AtA[i * n + j] = s;
    }
    double s = 0.0;
    for (int k = 0; k < m; ++k) s += A[k * n + i] * b[k];
    Atb[i] = s;
  }
  jacobi_eig(AtA, n, w, V);
  const double tol = (w[0] > 0 ? w[0] : 0.0) * 1e-24;
  for (int j = 0; j < n; ++j) x[j] = 0.0;
  for (int i = 0; i < n; ++i) {
    if (w[i] <= tol) continue;
    double proj = 0.0;
    for (int k = 0; k < n; ++k) proj += V[i * n + k] * Atb[k];
    proj /= w[i];
    for (int k = 0; k < n; ++k) x[k] += proj * V[i * n + k];
  }
}

// 3x3 pseudo-inverse (OpenCV inverts CC with CV_SVD): planar point sets make CC singular and
// the pseudo-inverse gives the 4th control point zero weight (EPnP's planar case).
__device__ void pinv3(const double* a, double* r) {
  double AtA[9], w[3], V[9];
  for (int i = 0; i < 3; ++i)
    for (int j = 0; j < 3; ++j) AtA[i * 3 + j] = a[i] * a[j] + a[3 + i] * a[3 + j] + a[6 + i] * a[6 + j];
  jacobi_eig(AtA, 3, w, V);
  const double tol = (w[0] > 0 ? w[0] : 0.0) * 1e-20;
  double P[9] = {0, 0, 0, 0, 0, 0, 0, 0, 0};
  for (int k = 0; k < 3; ++k) {
    if (w[k] <= tol) continue;
    for (int i = 0; i < 3; ++i)
      for (int j = 0; j < 3; ++j) P[i * 3 + j] += V[k * 3 + i] * V[k * 3 + j] / w[k];
  }
  for (int i = 0; i < 3; ++i)
    for (int j = 0; j < 3; ++j) r[i * 3 + j] = P[i * 3] * a[j * 3] + P[i * 3 + 1] * a[j * 3 + 1] + P[i * 3 + 2] * a[j * 3 + 2];
}

__device__ __forceinline__ double dot3(const double* a, const double* b) { return a[0] * b[0] + a[1] * b[1] + a[2] * b[2]; }

// Point accessor: correspondences live in LDS; `list` (optional) selects a subset.
struct Pts {
  const float* obj;  // [P][3]
  const float* img;  // [P][2]
  const int* list;   // nullptr -> identity
  int n;
  __device__ __forceinline__ int id(int i) const { return list ? list[i] : i; }
  __device__ __forceinline__ void pw(int i, double* p) const {
    const float* o = obj + 3 * id(i);
    p[0] = o[0]; p[1] = o[1]; p[2] = o[2];
  }
  __device__ __forceinline__ void uv(int i, double* q) const {
    const float* o = img + 2 * id(i);
    q[0] = o[0]; q[1] = o[1];
  }
};

__device__ void alphas_of(const double* p, const double cws[4][3], const double* ci, double a[4]) {
  const double d0 = p[0] - cws[0][0], d1 = p[1] - cws[0][1], d2 = p[2] - cws[0][2];
  a[1] = ci[0] * d0 + ci[1] * d1 + ci[2] * d2;
  a[2] = ci[3] * d0 + ci[4] * d1 + ci[5] * d2;
  a[3] = ci[6] * d0 + ci[7] * d1 + ci[8] * d2;
  a[0] = 1.0 - a[1] - a[2] - a[3];
}

__device__ void gauss_newton(const double* L, const double* rho, double betas[4]) {
  for (int it = 0; it < 5; ++it) {
    double A[24], b[6], x[4];
    for (int i = 0; i < 6; ++i) {
      const double* l = L + 10 * i;
      double* a = A + 4 * i;
      a[0] = 2 * l[0] * betas[0] + l[1] * betas[1] + l[3] * betas[2] + l[6] * betas[3];
      a[1] = l[1] * betas[0] + 2 * l[2] * betas[1] + l[4] * betas[2] + l[7] * betas[3];
      a[2] = l[3] * betas[0] + l[4] * betas[1] + 2 * l[5] * betas[2] + l[8] * betas[3];
      a[3] = l[6] * betas[0] + l[7] * betas[1] + l[8] * betas[2] + 2 * l[9] * betas[3];
      b[i] = rho[i] - (l[0] * betas[0] * betas[0] + l[1] * betas[0] * betas[1] + l[2] * betas[1] * betas[1] +
                       l[3] * betas[0] * betas[2] + l[4] * betas[1] * betas[2] + l[5] * betas[2] * betas[2] +
                       l[6] * betas[0] * betas[3] + l[7] * betas[1] * betas[3] + l[8] * betas[2] * betas[3] +
                       l[9] * betas[3] * betas[3]);
    }
    lsq_solve(A, 6, 4, b, x);
    for (int k = 0; k < 4; ++k) betas[k] += x[k];
  }
}

// Kabsch: R, t minimising sum ||R pw + t - pc||^2 for the camera-frame points pcs(i).
__device__ void procrustes(const Pts& P, const double ccs[4][3], const double cws[4][3], const double* ci,
                           bool flip, double* R, double* t) {
  double cw[3] = {0, 0, 0}, cc[3] = {0, 0, 0};
  const int n = P.n;
  for (int i = 0; i < n; ++i) {
    double p[3], a[4];
    P.pw(i, p);
    alphas_of(p, cws, ci, a);
    for (int k = 0; k < 3; ++k) {
      double pc = a[0] * ccs[0][k] + a[1] * ccs[1][k] + a[2] * ccs[2][k] + a[3] * ccs[3][k];
      cc[k] += flip ? -pc : pc;
      cw[k] += p[k];
    }
  }
  for (int k = 0; k < 3; ++k) { cw[k] /= n; cc[k] /= n; }
  double H[9] = {0, 0, 0, 0, 0, 0, 0, 0, 0};
  for (int i = 0; i < n; ++i) {
    double p[3], a[4], pc[3];
    P.pw(i, p);
    alphas_of(p, cws, ci, a);
    for (int k = 0; k < 3; ++k) {
      const double v = a[0] * ccs[0][k] + a[1] * ccs[1][k] + a[2] * ccs[2][k] + a[3] * ccs[3][k];
      pc[k] = flip ? -v : v;
    }
    for (int r = 0; r < 3; ++r)
      for (int c = 0; c < 3; ++c) H[r * 3 + c] += (pc[r] - cc[r]) * (p[c] - cw[c]);
  }
  double HtH[9], w[3], V[9];
  for (int i = 0; i < 3; ++i)
    for (int j = 0; j < 3; ++j) {
      double s = 0;
      for (int k = 0; k < 3; ++k) s += H[k * 3 + i] * H[k * 3 + j];
      HtH[i * 3 + j] = s;
    }
  jacobi_eig(HtH, 3, w, V);
  double U[9];
  for (int i = 0; i < 2; ++i) {
    double u[3];
    for (int r = 0; r < 3; ++r) u[r] = H[r * 3 + 0] * V[i * 3 + 0] + H[r * 3 + 1] * V[i * 3 + 1] + H[r * 3 + 2] * V[i * 3 + 2];
    double nr = sqrt(u[0] * u[0] + u[1] * u[1] + u[2] * u[2]);
    if (nr < 1e-300) nr = 1e-300;
    for (int r = 0; r < 3; ++r) U[i * 3 + r] = u[r] / nr;
  }
  {
    const double d = U[0] * U[3] + U[1] * U[4] + U[2] * U[5];
    for (int r = 0; r < 3; ++r) U[3 + r] -= d * U[r];
    double nr = sqrt(U[3] * U[3] + U[4] * U[4] + U[5] * U[5]);
    if (nr < 1e-300) nr = 1e-300;
    for (int r = 0; r < 3; ++r) U[3 + r] /= nr;
  }
  U[6] = U[1] * U[5] - U[2] * U[4];
  U[7] = U[2] * U[3] - U[0] * U[5];
  U[8] = U[0] * U[4] - U[1] * U[3];
  const double v2[3] = {V[1] * V[5] - V[2] * V[4], V[2] * V[3] - V[0] * V[5], V[0] * V[4] - V[1] * V[3]};
  for (int r = 0; r < 3; ++r)
    for (int c = 0; c < 3; ++c) R[r * 3 + c] = U[r] * V[c] + U[3 + r] * V[3 + c] + U[6 + r] * v2[c];
  for (int r = 0; r < 3; ++r) t[r] = cc[r] - (R[r * 3 + 0] * cw[0] + R[r * 3 + 1] * cw[1] + R[r * 3 + 2] * cw[2]);
}

__device__ double r_and_t(const double* ut, const double betas[4], const Pts& P, const double cws[4][3],
                          const double* ci, const Cam& cam, double* R, double* t) {
  double ccs[4][3];
  for (int j = 0; j < 4; ++j)
    for (int k = 0; k < 3; ++k) ccs[j][k] = 0.0;
  for (int i = 0; i < 4; ++i) {
    const double* v = ut + 12 * (11 - i);
    for (int j = 0; j < 4; ++j)
      for (int k = 0; k < 3; ++k) ccs[j][k] += betas[i] * v[3 * j + k];
  }
  // solve_for_sign: the first point must lie in front of the camera
  double p0[3], a0[4];
  P.pw(0, p0);
  alphas_of(p0, cws, ci, a0);
  const double z0 = a0[0] * ccs[0][2] + a0[1] * ccs[1][2] + a0[2] * ccs[2][2] + a0[3] * ccs[3][2];
  procrustes(P, ccs, cws, ci, z0 < 0.0, R, t);
  double err = 0.0;
  for (int i = 0; i < P.n; ++i) {
    double X[3], q[2];
    P.pw(i, X);
    P.uv(i, q);
    const double Xc = dot3(R, X) + t[0], Yc = dot3(R + 3, X) + t[1], Zc = dot3(R + 6, X) + t[2];
    const double iz = 1.0 / Zc;
    const double du = q[0] - (cam.uc + cam.fu * Xc * iz), dv = q[1] - (cam.vc + cam.fv * Yc * iz);
    err += sqrt(du * du + dv * dv);
  }
  return err / P.n;
}

// EPnP (Lepetit et al. 2009) on the points of P; result R (row-major), t.
__device__ void epnp(const Pts& P, const Cam& cam, double* Rout, double* tout) {
  const int n = P.n;
  double cws[4][3], ci[9];
  {
    double c0[3] = {0, 0, 0};
    for (int i = 0; i < n; ++i) {
      double p[3];
      P.pw(i, p);
      c0[0] += p[0]; c0[1] += p[1]; c0[2] += p[2];
    }
    for (int j = 0; j < 3; ++j) c0[j] /= n;
    double C[9] = {0, 0, 0, 0, 0, 0, 0, 0, 0};
    for (int i = 0; i < n; ++i) {
      double p[3];
      P.pw(i, p);
      for (int r = 0; r < 3; ++r)
        for (int c = 0; c < 3; ++c) C[r * 3 + c] += (p[r] - c0[r]) * (p[c] - c0[c]);
    }
    double w[3], V[9];
    jacobi_eig(C, 3, w, V);
    for (int j = 0; j < 3; ++j) cws[0][j] = c0[j];
    for (int i = 0; i < 3; ++i) {
      const double k = sqrt((w[i] > 0 ? w[i] : 0.0) / n);
      for (int j = 0; j < 3; ++j) cws[i + 1][j] = c0[j] + k * V[i * 3 + j];
    }
    double CC[9];
    for (int i = 0; i < 3; ++i)
      for (int j = 1; j < 4; ++j) CC[i * 3 + j - 1] = cws[j][i] - cws[0][i];
    pinv3(CC, ci);
  }
  double MtM[144];
  for (int i = 0; i < 144; ++i) MtM[i] = 0.0;
  for (int p = 0; p < n; ++p) {
    double X[3], q[2], a[4];
    P.pw(p, X);
    P.uv(p, q);
    alphas_of(X, cws, ci, a);
    double r1[12], r2[12];
    for (int j = 0; j < 4; ++j) {
      r1[3 * j] = a[j] * cam.fu;
      r1[3 * j + 1] = 0.0;
      r1[3 * j + 2] = a[j] * (cam.uc - q[0]);
      r2[3 * j] = 0.0;
      r2[3 * j + 1] = a[j] * cam.fv;
      r2[3 * j + 2] = a[j] * (cam.vc - q[1]);
    }
    for (int i = 0; i < 12; ++i)
      for (int j = i; j < 12; ++j) MtM[i * 12 + j] += r1[i] * r1[j] + r2[i] * r2[j];
  }
  for (int i = 0; i < 12; ++i)
    for (int j = 0; j < i; ++j) MtM[i * 12 + j] = MtM[j * 12 + i];
  double w12[12], ut[144];
  jacobi_eig(MtM, 12, w12, ut);
  double L[60], rho[6];
  {
    double dv[4][6][3];
    for (int i = 0; i < 4; ++i) {
      const double* v = ut + 12 * (11 - i);
      int a = 0, b = 1;
      for (int j = 0; j < 6; ++j) {
        for (int k = 0; k < 3; ++k) dv[i][j][k] = v[3 * a + k] - v[3 * b + k];
        if (++b > 3) { ++a; b = a + 1; }
      }
    }
    for (int i = 0; i < 6; ++i) {
      double* r = L + 10 * i;
      r[0] = dot3(dv[0][i], dv[0][i]);
      r[1] = 2.0 * dot3(dv[0][i], dv[1][i]);
      r[2] = dot3(dv[1][i], dv[1][i]);
      r[3] = 2.0 * dot3(dv[0][i], dv[2][i]);
      r[4] = 2.0 * dot3(dv[1][i], dv[2][i]);
      r[5] = dot3(dv[2][i], dv[2][i]);
      r[6] = 2.0 * dot3(dv[0][i], dv[3][i]);
      r[7] = 2.0 * dot3(dv[1][i], dv[3][i]);
      r[8] = 2.0 * dot3(dv[2][i], dv[3][i]);
      r[9] = dot3(dv[3][i], dv[3][i]);
    }
    int a = 0, b = 1;
    for (int j = 0; j < 6; ++j) {
      const double d0 = cws[a][0] - cws[b][0], d1 = cws[a][1] - cws[b][1], d2 = cws[a][2] - cws[b][2];
      rho[j] = d0 * d0 + d1 * d1 + d2 * d2;
      if (++b > 3) { ++a; b = a + 1; }
    }
  }
  double bestR[9], bestt[3], best_err = 1e300;
  for (int approx = 1; approx <= 3; ++approx) {
    double betas[4] = {0, 0, 0, 0};
    if (approx == 1) {
      double A[24], x[4];
      const int cols[4] = {0, 1, 3, 6};
      for (int i = 0; i < 6; ++i)
        for (int j = 0; j < 4; ++j) A[4 * i + j] = L[10 * i + cols[j]];
      lsq_solve(A, 6, 4, rho, x);
      if (x[0] < 0) {
        betas[0] = sqrt(-x[0]);
        for (int k = 1; k < 4; ++k) betas[k] = -x[k] / betas[0];
      } else {
        betas[0] = sqrt(x[0]);
        for (int k = 1; k < 4; ++k) betas[k] = betas[0] > 0 ? x[k] / betas[0] : 0.0;
      }
    } else if (approx == 2) {
      double A[18], x[3];
      for (int i = 0; i < 6; ++i)
        for (int j = 0; j < 3; ++j) A[3 * i + j] = L[10 * i + j];
      lsq_solve(A, 6, 3, rho, x);
      if (x[0] < 0) {
        betas[0] = sqrt(-x[0]);
        betas[1] = (x[2] < 0) ? sqrt(-x[2]) : 0.0;
      } else {
        betas[0] = sqrt(x[0]);
        betas[1] = (x[2] > 0) ? sqrt(x[2]) : 0.0;
      }
      if (x[1] < 0) betas[0] = -betas[0];
    } else {
      double A[30], x[5];
      for (int i = 0; i < 6; ++i)
        for (int j = 0; j < 5; ++j) A[5 * i + j] = L[10 * i + j];
      lsq_solve(A, 6, 5, rho, x);
      if (x[0] < 0) {
        betas[0] = sqrt(-x[0]);
        betas[1] = (x[2] < 0) ? sqrt(-x[2]) : 0.0;
      } else {
        betas[0] = sqrt(x[0]);
        betas[1] = (x[2] > 0) ? sqrt(x[2]) : 0.0;
      }
      if (x[1] < 0) betas[0] = -betas[0];
      betas[2] = betas[0] != 0.0 ? x[3] / betas[0] : 0.0;
    }
    gauss_newton(L, rho, betas);
    double R[9], t[3];
    const double err = r_and_t(ut, betas, P, cws, ci, cam, R, t);
    if (approx == 1 || err < best_err) {
      best_err = err;
      for (int i = 0; i < 9; ++i) bestR[i] = R[i];
      for (int i = 0; i < 3; ++i) bestt[i] = t[i];
    }
  }
  for (int i = 0; i < 9; ++i) Rout[i] = bestR[i];
  for (int i = 0; i < 3; ++i) tout[i] = bestt[i];
}

// FMA-free f32 inlier test (same expression order as oracle/pnp_ref.c)
__device__ __forceinline__ bool is_inlier(const float* Rf, const float* tf, const float* o, const float* q,
                                          const Cam& cam, float thr2) {
#pragma clang fp contract(off)
  const float X = o[0], Y = o[1], Z = o[2];
  const float xc = Rf[0] * X + Rf[1] * Y + Rf[2] * Z + tf[0];
  const float yc = Rf[3] * X + Rf[4] * Y + Rf[5] * Z + tf[1];
  const float zc = Rf[6] * X + Rf[7] * Y + Rf[8] * Z + tf[2];
  const float iz = 1.0f / zc;
  const float du = q[0] - ((float)cam.fu * xc * iz + (float)cam.uc);
  const float dv = q[1] - ((float)cam.fv * yc * iz + (float)cam.vc);
  return du * du + dv * dv <= thr2;
}

__global__ __launch_bounds__(kPnpThreads) void pnp_ransac_kernel(
    const float* __restrict__ xyz, int HW, const long long* __restrict__ choose, int N, const int* __restrict__ sel,
    int P, const float* __restrict__ xmap, const float* __restrict__ ymap, const float* __restrict__ K4,
    const double* __restrict__ extent, const double* __restrict__ lfb, const int* __restrict__ subsets, int H,
    float thr, float* __restrict__ Rout, float* __restrict__ tout, int* __restrict__ inl_out,
    unsigned char* __restrict__ mask_out) {
  __shared__ float sobj[kPnpMaxP * 3];
  __shared__ float simg[kPnpMaxP * 2];
  __shared__ int slist[kPnpMaxP];
  __shared__ int sbest[kPnpThreads];
  __shared__ float sRt[12];
  const int b = blockIdx.x;
  const Cam cam = {K4[4 * b + 0], K4[4 * b + 1], K4[4 * b + 2], K4[4 * b + 3]};
  const double e0 = extent[3 * b], e1 = extent[3 * b + 1], e2 = extent[3 * b + 2];
  const double l0 = lfb[3 * b], l1 = lfb[3 * b + 1], l2 = lfb[3 * b + 2];
  for (int i = threadIdx.x; i < P; i += kPnpThreads) {
    const int ci = sel[(long long)b * P + i];
    const long long pix = choose[(long long)b * N + ci];
    const float* xb = xyz + (long long)b * 3 * HW + pix;
    sobj[3 * i + 0] = (float)((double)xb[0] * e0 + l0);
    sobj[3 * i + 1] = (float)((double)xb[HW] * e1 + l1);
    sobj[3 * i + 2] = (float)((double)xb[2 * HW] * e2 + l2);
    simg[2 * i + 0] = xmap[(long long)b * N + ci];
    simg[2 * i + 1] = ymap[(long long)b * N + ci];
  }
  __syncthreads();
  const float thr2 = thr * thr;
  // ---- hypotheses (one per thread) --------------------------------------------------------
  int my_cnt = -1;
  for (int h = threadIdx.x; h < H; h += kPnpThreads) {
    int ids[5];
    for (int i = 0; i < 5; ++i) ids[i] = subsets[((long long)b * H + h) * 5 + i];
    Pts sub{sobj, simg, ids, 5};
    double R[9], t[3];
    epnp(sub, cam, R, t);
    float Rf[9], tf[3];
    for (int i = 0; i < 9; ++i) Rf[i] = (float)R[i];
    for (int i = 0; i < 3; ++i) tf[i] = (float)t[i];
    int cnt = 0;
    for (int p = 0; p < P; ++p) cnt += is_inlier(Rf, tf, sobj + 3 * p, simg + 2 * p, cam, thr2) ? 1 : 0;
    // encode (count, -h) so that max picks most inliers, then lowest h
    const int key = cnt * 4096 + (4095 - h);
    my_cnt = max(my_cnt, key);
  }
  sbest[threadIdx.x] = my_cnt;
  __syncthreads();
  for (int s = kPnpThreads / 2; s > 0; s >>= 1) {
    if (threadIdx.x < s) sbest[threadIdx.x] = max(sbest[threadIdx.x], sbest[threadIdx.x + s]);
    __syncthreads();
  }
  const int key = sbest[0];
  const int best_cnt = key >= 0 ? key / 4096 : 0;
  const int best_h = key >= 0 ? 4095 - (key % 4096) : -1;
  const bool ok = best_h >= 0 && best_cnt >= 5;
  if (threadIdx.x == 0) {
    double R[9] = {1, 0, 0, 0, 1, 0, 0, 0, 1}, t[3] = {0, 0, 0};
    if (best_h >= 0) {
      int ids[5];
      for (int i = 0; i < 5; ++i) ids[i] = subsets[((long long)b * H + best_h) * 5 + i];
      Pts sub{sobj, simg, ids, 5};
      epnp(sub, cam, R, t);
    }
    for (int i = 0; i < 9; ++i) sRt[i] = (float)R[i];
    for (int i = 0; i < 3; ++i) sRt[9 + i] = (float)t[i];
  }
  __syncthreads();
  // ---- inlier set of the best hypothesis (ordered compaction) -------------------------------
  if (threadIdx.x == 0) {
    int n = 0;
    for (int p = 0; p < P; ++p) {
      const bool in = ok && is_inlier(sRt, sRt + 9, sobj + 3 * p, simg + 2 * p, cam, thr2);
      if (mask_out) mask_out[(long long)b * P + p] = in ? 1 : 0;
      if (in) slist[n++] = p;
    }
    double R[9], t[3];
    for (int i = 0; i < 9; ++i) R[i] = sRt[i];
    for (int i = 0; i < 3; ++i) t[i] = sRt[9 + i];
    if (ok && n >= 5) {
      Pts inl{sobj, simg, slist, n};
      epnp(inl, cam, R, t);
      for (int i = 0; i < 9; ++i) Rout[9 * b + i] = (float)R[i];
      for (int i = 0; i < 3; ++i) tout[3 * b + i] = (float)t[i];
    } else {
      // RANSAC failed (< 5 inliers): cv::solvePnPRansac returns false with rvec = tvec = 0,
      // i.e. R = I, t = 0 after the Rodrigues step of trainer.py:429-435
      for (int i = 0; i < 9; ++i) Rout[9 * b + i] = (i % 4 == 0) ? 1.f : 0.f;
      for (int i = 0; i < 3; ++i) tout[3 * b + i] = 0.f;
    }
    inl_out[b] = ok ? best_cnt : 0;
  }
}

}  // namespace

KRRN_API int krrn_pnp_ransac_f32(const float* xyz, int HW, const long long* choose, int N, const int* sel, int P,
                                 const float* xmap, const float* ymap, const float* K4, const double* extent,
                                 const double* lfborder, const int* subsets, int H, float thr, float* R, float* t,
                                 int* inliers, unsigned char* inlier_mask, int B, void* stream) {
  if (!xyz || !choose || !sel || !xmap || !ymap || !K4 || !extent || !lfborder || !subsets || !R || !t || !inliers)
    return KRRN_EARG;
  if (B < 1 || P < 5 || P > kPnpMaxP || H < 1 || H > 4095 || N < 1 || HW < 1) return KRRN_ESHAPE;
  hipLaunchKernelGGL(pnp_ransac_kernel, dim3(B), dim3(kPnpThreads), 0, (hipStream_t)stream, xyz, HW, choose, N, sel,
                     P, xmap, ymap, K4, extent, lfborder, subsets, H, thr, R, t, inliers, inlier_mask);
  return krrn_launch_status();
}
