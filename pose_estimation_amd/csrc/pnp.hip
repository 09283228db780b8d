// Batched PnP-RANSAC for Trainer.get_pose (tools/trainer.py:383-438).
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
//
// Latency design: a 5-point EPnP is ~100 small dense solves. Every 3x3 / 4x4 / 5x5 symmetric
// eigen-solve is a fully unrolled cyclic Jacobi whose indices are all compile-time constants,
// so the matrices live in VGPRs; the one 12x12 solve (M^T M) runs on a per-thread LDS arena
// with runtime (p, q) but unrolled rows, so each rotation issues its loads back to back.
// (A dynamically indexed private array lives in scratch: the first version spent 2.8 ms per
// 64-crop batch there.)
#include <math.h>

#include "krrn_common.h"

namespace {

constexpr int kPnpMaxP = 1024;
constexpr int kArena = 300;  // doubles per 12x12 solve: A 144, U 144, w 12

struct Cam {
  double fu, fv, uc, vc;
};

// ---- small symmetric eigen-solves in registers --------------------------------------------
// A (destroyed) -> eigenvalues w (descending) and eigenvectors as ROWS of V.
template <int N>
__device__ __forceinline__ void eig_small(double (&A)[N * N], double (&w)[N], double (&V)[N * N]) {
  double U[N * N];  // columns = eigenvectors during the sweeps
#pragma unroll
  for (int i = 0; i < N; ++i)
#pragma unroll
    for (int j = 0; j < N; ++j) U[i * N + j] = (i == j) ? 1.0 : 0.0;
  for (int sweep = 0; sweep < 40; ++sweep) {
    double off = 0.0, tot = 0.0;
#pragma unroll
    for (int p = 0; p < N; ++p)
#pragma unroll
      for (int q = 0; q < N; ++q) {
        const double a2 = A[p * N + q] * A[p * N + q];
        tot += a2;
        if (p != q) off += a2;
      }
    if (off <= 1e-30 * tot || off < 1e-300) break;
#pragma unroll
    for (int p = 0; p < N; ++p) {
#pragma unroll
      for (int q = p + 1; q < N; ++q) {
        const double apq = A[p * N + q];
        const double app = A[p * N + p], aqq = A[q * N + q];
        const bool rot = fabs(apq) >= 1e-300;
        const double theta = (aqq - app) / (2.0 * (rot ? apq : 1.0));
        const double tt = (theta >= 0 ? 1.0 : -1.0) / (fabs(theta) + sqrt(theta * theta + 1.0));
        const double c = rot ? 1.0 / sqrt(tt * tt + 1.0) : 1.0;
        const double s = rot ? tt * c : 0.0;
#pragma unroll
        for (int k = 0; k < N; ++k) {
          const double akp = A[k * N + p], akq = A[k * N + q];
          A[k * N + p] = c * akp - s * akq;
          A[k * N + q] = s * akp + c * akq;
        }
#pragma unroll
        for (int k = 0; k < N; ++k) {
          const double apk = A[p * N + k], aqk = A[q * N + k];
          A[p * N + k] = c * apk - s * aqk;
          A[q * N + k] = s * apk + c * aqk;
        }
#pragma unroll
        for (int k = 0; k < N; ++k) {
          const double ukp = U[k * N + p], ukq = U[k * N + q];
          U[k * N + p] = c * ukp - s * ukq;
          U[k * N + q] = s * ukp + c * ukq;
        }
      }
    }
  }
#pragma unroll
  for (int i = 0; i < N; ++i) w[i] = A[i * N + i];
  // descending order by compare-exchange (every index compile-time)
#pragma unroll
  for (int i = 0; i < N; ++i)
#pragma unroll
    for (int j = i + 1; j < N; ++j) {
      const bool sw = w[j] > w[i];
      const double wi = w[i], wj = w[j];
      w[i] = sw ? wj : wi;
      w[j] = sw ? wi : wj;
#pragma unroll
      for (int k = 0; k < N; ++k) {
        const double ui = U[k * N + i], uj = U[k * N + j];
        U[k * N + i] = sw ? uj : ui;
        U[k * N + j] = sw ? ui : uj;
      }
    }
#pragma unroll
  for (int i = 0; i < N; ++i)
#pragma unroll
    for (int k = 0; k < N; ++k) V[i * N + k] = U[k * N + i];
}

// 12x12 symmetric eigen-solve on an LDS arena (element e at arena[e * S]); returns the four
// eigenvectors of the SMALLEST eigenvalues, smallest first: v4[r * 12 + k].
__device__ void eig12_arena(double* ar, int S, double (&v4)[48]) {
  double* A = ar;
  double* U = ar + 144 * S;
  double* w = ar + 288 * S;
#define AA(i) A[(i) * S]
#define UU(i) U[(i) * S]
  for (int i = 0; i < 144; ++i) UU(i) = (i % 13 == 0) ? 1.0 : 0.0;
  for (int sweep = 0; sweep < 40; ++sweep) {
    double off = 0.0, tot = 0.0;
#pragma unroll 12
    for (int e = 0; e < 144; ++e) {
      const double a = AA(e);
      tot += a * a;
      if (e % 13 != 0) off += a * a;
    }
    if (off <= 1e-30 * tot || off < 1e-300) break;
    for (int p = 0; p < 12; ++p) {
      for (int q = p + 1; q < 12; ++q) {
        const double apq = AA(p * 12 + q);
        const double app = AA(p * 13), aqq = AA(q * 13);
        // negligible against both diagonal entries (below their f64 resolution): skip
        if (fabs(apq) < 1e-300 || fabs(apq) < 1e-18 * sqrt(fabs(app * aqq))) continue;
        const double theta = (aqq - app) / (2.0 * apq);
        const double tt = (theta >= 0 ? 1.0 : -1.0) / (fabs(theta) + sqrt(theta * theta + 1.0));
        const double c = 1.0 / sqrt(tt * tt + 1.0), s = tt * c;
        double cp[12], cq[12];
#pragma unroll
        for (int k = 0; k < 12; ++k) { cp[k] = AA(k * 12 + p); cq[k] = AA(k * 12 + q); }
#pragma unroll
        for (int k = 0; k < 12; ++k) {
          AA(k * 12 + p) = c * cp[k] - s * cq[k];
          AA(k * 12 + q) = s * cp[k] + c * cq[k];
        }
#pragma unroll
        for (int k = 0; k < 12; ++k) { cp[k] = AA(p * 12 + k); cq[k] = AA(q * 12 + k); }
#pragma unroll
        for (int k = 0; k < 12; ++k) {
          AA(p * 12 + k) = c * cp[k] - s * cq[k];
          AA(q * 12 + k) = s * cp[k] + c * cq[k];
        }
#pragma unroll
        for (int k = 0; k < 12; ++k) { cp[k] = UU(k * 12 + p); cq[k] = UU(k * 12 + q); }
#pragma unroll
        for (int k = 0; k < 12; ++k) {
          UU(k * 12 + p) = c * cp[k] - s * cq[k];
          UU(k * 12 + q) = s * cp[k] + c * cq[k];
        }
      }
    }
  }
  for (int i = 0; i < 12; ++i) w[i * S] = AA(i * 13);
  // the 4 smallest eigenvalues in ascending order (ties: lower column first)
  unsigned used = 0;
  for (int r = 0; r < 4; ++r) {
    int m = -1;
    double wm = 0.0;
    for (int j = 0; j < 12; ++j) {
      if (used & (1u << j)) continue;
      const double wj = w[j * S];
      if (m < 0 || wj < wm) { m = j; wm = wj; }
    }
    used |= 1u << m;
#pragma unroll
    for (int k = 0; k < 12; ++k) v4[r * 12 + k] = UU(k * 12 + m);
  }
#undef AA
#undef UU
}

// least squares min ||A x - b|| (A is 6 x N) through the pseudo-inverse from eig(A^T A)
template <int N>
__device__ __forceinline__ void lsq_solve(const double (&A)[6 * N], const double (&b)[6], double (&x)[N]) {
  double AtA[N * N], w[N], V[N * N], Atb[N];
#pragma unroll
  for (int i = 0; i < N; ++i) {
#pragma unroll
    for (int j = 0; j < N; ++j) {
      double s = 0.0;
#pragma unroll
      for (int k = 0; k < 6; ++k) s += A[k * N + i] * A[k * N + j];
      AtA[i * N + j] = s;
    }
    double s = 0.0;
#pragma unroll
    for (int k = 0; k < 6; ++k) s += A[k * N + i] * b[k];
    Atb[i] = s;
  }
  // Full column rank (the usual case): Cholesky of the normal equations, ~N^3/6 flops.
  double C[N * N];
  double dmax = 0.0;
#pragma unroll
  for (int i = 0; i < N; ++i) dmax = fmax(dmax, AtA[i * N + i]);
  bool spd = dmax > 0.0;
#pragma unroll
  for (int j = 0; j < N; ++j) {
    double d = AtA[j * N + j];
#pragma unroll
    for (int k = 0; k < j; ++k) d -= C[j * N + k] * C[j * N + k];
    spd = spd && d > 1e-14 * dmax;
    const double cjj = sqrt(fmax(d, 1e-300));
    C[j * N + j] = cjj;
#pragma unroll
    for (int i = j + 1; i < N; ++i) {
      double s = AtA[i * N + j];
#pragma unroll
      for (int k = 0; k < j; ++k) s -= C[i * N + k] * C[j * N + k];
      C[i * N + j] = s / cjj;
    }
  }
  if (spd) {
    double y[N];
#pragma unroll
    for (int i = 0; i < N; ++i) {
      double s = Atb[i];
#pragma unroll
      for (int k = 0; k < i; ++k) s -= C[i * N + k] * y[k];
      y[i] = s / C[i * N + i];
    }
#pragma unroll
    for (int i = N - 1; i >= 0; --i) {
      double s = y[i];
#pragma unroll
      for (int k = i + 1; k < N; ++k) s -= C[k * N + i] * x[k];
      x[i] = s / C[i * N + i];
    }
    return;
  }
  // rank deficient: pseudo-inverse (OpenCV solves these with CV_SVD)
  eig_small<N>(AtA, w, V);
  const double tol = (w[0] > 0 ? w[0] : 0.0) * 1e-24;
#pragma unroll
  for (int j = 0; j < N; ++j) x[j] = 0.0;
#pragma unroll
  for (int i = 0; i < N; ++i) {
    double proj = 0.0;
#pragma unroll
    for (int k = 0; k < N; ++k) proj += V[i * N + k] * Atb[k];
    proj = (w[i] > tol) ? proj / w[i] : 0.0;
#pragma unroll
    for (int k = 0; k < N; ++k) x[k] += proj * V[i * N + k];
  }
}

// 3x3 pseudo-inverse (OpenCV inverts CC with CV_SVD): planar point sets make CC singular and
// the pseudo-inverse gives the 4th control point zero weight (EPnP's planar case).
__device__ __forceinline__ void pinv3(const double (&a)[9], double (&r)[9]) {
  double AtA[9], w[3], V[9];
#pragma unroll
  for (int i = 0; i < 3; ++i)
#pragma unroll
    for (int j = 0; j < 3; ++j) AtA[i * 3 + j] = a[i] * a[j] + a[3 + i] * a[3 + j] + a[6 + i] * a[6 + j];
  eig_small<3>(AtA, w, V);
  const double tol = (w[0] > 0 ? w[0] : 0.0) * 1e-20;
  double Pm[9] = {0, 0, 0, 0, 0, 0, 0, 0, 0};
#pragma unroll
  for (int k = 0; k < 3; ++k) {
    const double iw = (w[k] > tol) ? 1.0 / w[k] : 0.0;
#pragma unroll
    for (int i = 0; i < 3; ++i)
#pragma unroll
      for (int j = 0; j < 3; ++j) Pm[i * 3 + j] += V[k * 3 + i] * V[k * 3 + j] * iw;
  }
#pragma unroll
  for (int i = 0; i < 3; ++i)
#pragma unroll
    for (int j = 0; j < 3; ++j) r[i * 3 + j] = Pm[i * 3] * a[j * 3] + Pm[i * 3 + 1] * a[j * 3 + 1] + Pm[i * 3 + 2] * a[j * 3 + 2];
}

__device__ __forceinline__ double dot3(const double* a, const double* b) { return a[0] * b[0] + a[1] * b[1] + a[2] * b[2]; }

// Correspondences in LDS; `list` (optional) selects a subset.
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

// Point-loop sums and the 12x12 solve of EPnP, evaluated either by one thread (a RANSAC
// hypothesis, SerialSum) or by one wave with the points spread over the 64 lanes and a
// butterfly reduction (the refinement on all inliers, WaveSum). The small dense algebra
// between the sums is replicated in every lane, which costs one wave's time.
struct SerialSum {
  double* arena;  // this thread's arena (stride S)
  int S;
  template <int NV, class F>
  __device__ __forceinline__ void operator()(int n, F f, double (&acc)[NV]) const {
#pragma unroll
    for (int k = 0; k < NV; ++k) acc[k] = 0.0;
    for (int i = 0; i < n; ++i) f(i, acc);
  }
  __device__ __forceinline__ void eig12(const double (&m)[78], double (&v4)[48]) const {
    int e = 0;
#pragma unroll
    for (int i = 0; i < 12; ++i)
#pragma unroll
      for (int j = i; j < 12; ++j, ++e) {
        arena[(i * 12 + j) * S] = m[e];
        arena[(j * 12 + i) * S] = m[e];
      }
    eig12_arena(arena, S, v4);
  }
};

struct WaveSum {
  int lane;
  double* arena;  // one shared arena (stride 1), solved by lane 0
  template <int NV, class F>
  __device__ __forceinline__ void operator()(int n, F f, double (&acc)[NV]) const {
#pragma unroll
    for (int k = 0; k < NV; ++k) acc[k] = 0.0;
    for (int i = lane; i < n; i += 64) f(i, acc);
#pragma unroll
    for (int k = 0; k < NV; ++k) {
      double v = acc[k];
#pragma unroll
      for (int off = 32; off > 0; off >>= 1) v += __shfl_xor(v, off);
      acc[k] = v;
    }
  }
  __device__ __forceinline__ void eig12(const double (&m)[78], double (&v4)[48]) const {
    __syncthreads();
    if (lane == 0) {
      int e = 0;
      for (int i = 0; i < 12; ++i)
        for (int j = i; j < 12; ++j, ++e) {
          arena[i * 12 + j] = m[e];
          arena[j * 12 + i] = m[e];
        }
      double r[48];
      eig12_arena(arena, 1, r);
      for (int k = 0; k < 48; ++k) arena[k] = r[k];
    }
    __syncthreads();
#pragma unroll
    for (int k = 0; k < 48; ++k) v4[k] = arena[k];
  }
};

__device__ __forceinline__ void alphas_of(const double* p, const double cws[4][3], const double* ci, double a[4]) {
  const double d0 = p[0] - cws[0][0], d1 = p[1] - cws[0][1], d2 = p[2] - cws[0][2];
  a[1] = ci[0] * d0 + ci[1] * d1 + ci[2] * d2;
  a[2] = ci[3] * d0 + ci[4] * d1 + ci[5] * d2;
  a[3] = ci[6] * d0 + ci[7] * d1 + ci[8] * d2;
  a[0] = 1.0 - a[1] - a[2] - a[3];
}

__device__ __forceinline__ void gauss_newton(const double (&L)[60], const double (&rho)[6], double (&betas)[4]) {
  for (int it = 0; it < 5; ++it) {
    double A[24], b[6], x[4];
#pragma unroll
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
    lsq_solve<4>(A, b, x);
#pragma unroll
    for (int k = 0; k < 4; ++k) betas[k] += x[k];
  }
}

// Kabsch on the 3x3 correlation H = sum (pc - cc)(pw - cw)^T: R = U diag(1,1,det) V^T.
__device__ __forceinline__ void kabsch(const double (&H)[9], double (&R)[9]) {
  double HtH[9], w[3], V[9];
#pragma unroll
  for (int i = 0; i < 3; ++i)
#pragma unroll
    for (int j = 0; j < 3; ++j) HtH[i * 3 + j] = H[i] * H[j] + H[3 + i] * H[3 + j] + H[6 + i] * H[6 + j];
  eig_small<3>(HtH, w, V);
  double U[9];
#pragma unroll
  for (int i = 0; i < 2; ++i) {
    double u[3];
#pragma unroll
    for (int r = 0; r < 3; ++r) u[r] = H[r * 3 + 0] * V[i * 3 + 0] + H[r * 3 + 1] * V[i * 3 + 1] + H[r * 3 + 2] * V[i * 3 + 2];
    double nr = sqrt(u[0] * u[0] + u[1] * u[1] + u[2] * u[2]);
    if (nr < 1e-300) nr = 1e-300;
#pragma unroll
    for (int r = 0; r < 3; ++r) U[i * 3 + r] = u[r] / nr;
  }
  {
    const double d = U[0] * U[3] + U[1] * U[4] + U[2] * U[5];
#pragma unroll
    for (int r = 0; r < 3; ++r) U[3 + r] -= d * U[r];
    double nr = sqrt(U[3] * U[3] + U[4] * U[4] + U[5] * U[5]);
    if (nr < 1e-300) nr = 1e-300;
#pragma unroll
    for (int r = 0; r < 3; ++r) U[3 + r] /= nr;
  }
  U[6] = U[1] * U[5] - U[2] * U[4];
  U[7] = U[2] * U[3] - U[0] * U[5];
  U[8] = U[0] * U[4] - U[1] * U[3];
  const double v2[3] = {V[1] * V[5] - V[2] * V[4], V[2] * V[3] - V[0] * V[5], V[0] * V[4] - V[1] * V[3]};
#pragma unroll
  for (int r = 0; r < 3; ++r)
#pragma unroll
    for (int c = 0; c < 3; ++c) R[r * 3 + c] = U[r] * V[c] + U[3 + r] * V[3 + c] + U[6 + r] * v2[c];
}

template <class SUM>
__device__ double r_and_t(const SUM& sum, const double (&v4)[48], const double (&betas)[4], const Pts& P,
                          const double cws[4][3], const double* ci, const double* cw, const Cam& cam, double (&R)[9],
                          double (&t)[3]) {
  double ccs[4][3];
#pragma unroll
  for (int j = 0; j < 4; ++j)
#pragma unroll
    for (int k = 0; k < 3; ++k) ccs[j][k] = 0.0;
#pragma unroll
  for (int i = 0; i < 4; ++i)
#pragma unroll
    for (int j = 0; j < 4; ++j)
#pragma unroll
      for (int k = 0; k < 3; ++k) ccs[j][k] += betas[i] * v4[12 * i + 3 * j + k];
  // solve_for_sign: the first point must lie in front of the camera
  double p0[3], a0[4];
  P.pw(0, p0);
  alphas_of(p0, cws, ci, a0);
  const double z0 = a0[0] * ccs[0][2] + a0[1] * ccs[1][2] + a0[2] * ccs[2][2] + a0[3] * ccs[3][2];
  const double sg = z0 < 0.0 ? -1.0 : 1.0;
  const int n = P.n;
  double cc[3];
  sum(n, [&](int i, double (&acc)[3]) {
        double p[3], a[4];
        P.pw(i, p);
        alphas_of(p, cws, ci, a);
#pragma unroll
        for (int k = 0; k < 3; ++k) acc[k] += sg * (a[0] * ccs[0][k] + a[1] * ccs[1][k] + a[2] * ccs[2][k] + a[3] * ccs[3][k]);
      }, cc);
#pragma unroll
  for (int k = 0; k < 3; ++k) cc[k] /= n;
  double H[9];
  sum(n, [&](int i, double (&acc)[9]) {
        double p[3], a[4], pc[3];
        P.pw(i, p);
        alphas_of(p, cws, ci, a);
#pragma unroll
        for (int k = 0; k < 3; ++k) pc[k] = sg * (a[0] * ccs[0][k] + a[1] * ccs[1][k] + a[2] * ccs[2][k] + a[3] * ccs[3][k]);
#pragma unroll
        for (int r = 0; r < 3; ++r)
#pragma unroll
          for (int c = 0; c < 3; ++c) acc[r * 3 + c] += (pc[r] - cc[r]) * (p[c] - cw[c]);
      }, H);
  kabsch(H, R);
#pragma unroll
  for (int r = 0; r < 3; ++r) t[r] = cc[r] - (R[r * 3 + 0] * cw[0] + R[r * 3 + 1] * cw[1] + R[r * 3 + 2] * cw[2]);
  double err[1];
  sum(n, [&](int i, double (&acc)[1]) {
        double X[3], q[2];
        P.pw(i, X);
        P.uv(i, q);
        const double Xc = dot3(R, X) + t[0], Yc = dot3(R + 3, X) + t[1], Zc = dot3(R + 6, X) + t[2];
        const double iz = 1.0 / Zc;
        const double du = q[0] - (cam.uc + cam.fu * Xc * iz), dv = q[1] - (cam.vc + cam.fv * Yc * iz);
        acc[0] += sqrt(du * du + dv * dv);
      }, err);
  return err[0] / n;
}

// EPnP (Lepetit et al. 2009) on the points of P; result R (row-major), t.
template <class SUM>
__device__ void epnp(const SUM& sum, const Pts& P, const Cam& cam, double (&Rout)[9], double (&tout)[3]) {
  const int n = P.n;
  double cws[4][3], ci[9], cw[3];
  {
    sum(n, [&](int i, double (&acc)[3]) {
          double p[3];
          P.pw(i, p);
          acc[0] += p[0]; acc[1] += p[1]; acc[2] += p[2];
        }, cw);
#pragma unroll
    for (int j = 0; j < 3; ++j) cw[j] /= n;
    double C6[6];
    sum(n, [&](int i, double (&acc)[6]) {
          double p[3];
          P.pw(i, p);
          const double d0 = p[0] - cw[0], d1 = p[1] - cw[1], d2 = p[2] - cw[2];
          acc[0] += d0 * d0; acc[1] += d0 * d1; acc[2] += d0 * d2;
          acc[3] += d1 * d1; acc[4] += d1 * d2; acc[5] += d2 * d2;
        }, C6);
    double C[9] = {C6[0], C6[1], C6[2], C6[1], C6[3], C6[4], C6[2], C6[4], C6[5]};
    double w[3], V[9];
    eig_small<3>(C, w, V);
#pragma unroll
    for (int j = 0; j < 3; ++j) cws[0][j] = cw[j];
#pragma unroll
    for (int i = 0; i < 3; ++i) {
      const double k = sqrt((w[i] > 0 ? w[i] : 0.0) / n);
#pragma unroll
      for (int j = 0; j < 3; ++j) cws[i + 1][j] = cw[j] + k * V[i * 3 + j];
    }
    double CC[9], CI[9];
#pragma unroll
    for (int i = 0; i < 3; ++i)
#pragma unroll
      for (int j = 1; j < 4; ++j) CC[i * 3 + j - 1] = cws[j][i] - cws[0][i];
    pinv3(CC, CI);
#pragma unroll
    for (int i = 0; i < 9; ++i) ci[i] = CI[i];
  }
  // M^T M from the two rows per point: r1 = [a_j fu, 0, a_j (uc - u)], r2 = [0, a_j fv, a_j (vc - v)]
  double m[78];
  sum(n, [&](int p, double (&acc)[78]) {
        double X[3], q[2], a[4];
        P.pw(p, X);
        P.uv(p, q);
        alphas_of(X, cws, ci, a);
        double r1[12], r2[12];
#pragma unroll
        for (int j = 0; j < 4; ++j) {
          r1[3 * j] = a[j] * cam.fu;
          r1[3 * j + 1] = 0.0;
          r1[3 * j + 2] = a[j] * (cam.uc - q[0]);
          r2[3 * j] = 0.0;
          r2[3 * j + 1] = a[j] * cam.fv;
          r2[3 * j + 2] = a[j] * (cam.vc - q[1]);
        }
        int e = 0;
#pragma unroll
        for (int i = 0; i < 12; ++i)
#pragma unroll
          for (int j = i; j < 12; ++j, ++e) acc[e] += r1[i] * r1[j] + r2[i] * r2[j];
      }, m);
  double v4[48];
  sum.eig12(m, v4);
  double L[60], rho[6];
  {
    double dv[4][6][3];
#pragma unroll
    for (int i = 0; i < 4; ++i) {
      const double* v = v4 + 12 * i;
      int a = 0, b = 1;
#pragma unroll
      for (int j = 0; j < 6; ++j) {
#pragma unroll
        for (int k = 0; k < 3; ++k) dv[i][j][k] = v[3 * a + k] - v[3 * b + k];
        if (++b > 3) { ++a; b = a + 1; }
      }
    }
#pragma unroll
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
#pragma unroll
    for (int j = 0; j < 6; ++j) {
      const double d0 = cws[a][0] - cws[b][0], d1 = cws[a][1] - cws[b][1], d2 = cws[a][2] - cws[b][2];
      rho[j] = d0 * d0 + d1 * d1 + d2 * d2;
      if (++b > 3) { ++a; b = a + 1; }
    }
  }
  double best_err = 1e300;
  for (int approx = 1; approx <= 3; ++approx) {
    double betas[4] = {0, 0, 0, 0};
    if (approx == 1) {
      double A[24], x[4];
      const int cols[4] = {0, 1, 3, 6};
#pragma unroll
      for (int i = 0; i < 6; ++i)
#pragma unroll
        for (int j = 0; j < 4; ++j) A[4 * i + j] = L[10 * i + cols[j]];
      lsq_solve<4>(A, rho, x);
      if (x[0] < 0) {
        betas[0] = sqrt(-x[0]);
#pragma unroll
        for (int k = 1; k < 4; ++k) betas[k] = -x[k] / betas[0];
      } else {
        betas[0] = sqrt(x[0]);
#pragma unroll
        for (int k = 1; k < 4; ++k) betas[k] = betas[0] > 0 ? x[k] / betas[0] : 0.0;
      }
    } else if (approx == 2) {
      double A[18], x[3];
#pragma unroll
      for (int i = 0; i < 6; ++i)
#pragma unroll
        for (int j = 0; j < 3; ++j) A[3 * i + j] = L[10 * i + j];
      lsq_solve<3>(A, rho, x);
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
#pragma unroll
      for (int i = 0; i < 6; ++i)
#pragma unroll
        for (int j = 0; j < 5; ++j) A[5 * i + j] = L[10 * i + j];
      lsq_solve<5>(A, rho, x);
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
    const double err = r_and_t(sum, v4, betas, P, cws, ci, cw, cam, R, t);
    if (approx == 1 || err < best_err) {
      best_err = err;
#pragma unroll
      for (int i = 0; i < 9; ++i) Rout[i] = R[i];
#pragma unroll
      for (int i = 0; i < 3; ++i) tout[i] = t[i];
    }
  }
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

// obj / img correspondences of crop b into LDS (see the file header)
__device__ void load_corr(int b, const float* xyz, int HW, const long long* choose, int N, const int* sel, int P,
                          const float* xmap, const float* ymap, const double* extent, const double* lfb,
                          float* sobj, float* simg) {
  const double e0 = extent[3 * b], e1 = extent[3 * b + 1], e2 = extent[3 * b + 2];
  const double l0 = lfb[3 * b], l1 = lfb[3 * b + 1], l2 = lfb[3 * b + 2];
  for (int i = threadIdx.x; i < P; i += blockDim.x) {
    const int ci = sel[(long long)b * P + i];
    const long long pix = choose[(long long)b * N + ci];
    const float* xb = xyz + (long long)b * 3 * HW + pix;
    sobj[3 * i + 0] = (float)((double)xb[0] * e0 + l0);
    sobj[3 * i + 1] = (float)((double)xb[HW] * e1 + l1);
    sobj[3 * i + 2] = (float)((double)xb[2 * HW] * e2 + l2);
    simg[2 * i + 0] = xmap[(long long)b * N + ci];
    simg[2 * i + 1] = ymap[(long long)b * N + ci];
  }
}

#ifndef KRRN_PNP_HPB
#define KRRN_PNP_HPB 50  // measured (ms/step): 16 -> 15.98, 25 -> 15.90, 32 -> 15.83, 50 -> 15.64-15.77, 64 -> 15.75
#endif
constexpr int kHypPerBlock = KRRN_PNP_HPB;

// Phase 1: one thread per RANSAC hypothesis; grid (B, ceil(H / kHypPerBlock)). The blocks are
// long-lived (~1 ms of serial f64 solves) and run beside the fusion / TBase launches: 50
// hypotheses per block (H = 100 -> 2 blocks per crop, 125 KB of LDS each, one per CU) confines
// the kernel to ~128 CUs and leaves the rest of the chip whole, which beats spreading 448
// quarter-wave blocks of 16 over every CU (15.7 vs 16.0 ms per step). Writes the f32 pose (R, t: the precision the inlier
// test uses) and the inlier count of every hypothesis.
__global__ __launch_bounds__(kHypPerBlock) void pnp_hyp_kernel(
    const float* __restrict__ xyz, int HW, const long long* __restrict__ choose, int N, const int* __restrict__ sel,
    int P, const float* __restrict__ xmap, const float* __restrict__ ymap, const float* __restrict__ K4,
    const double* __restrict__ extent, const double* __restrict__ lfb, const int* __restrict__ subsets, int H,
    float thr, float* __restrict__ hyp_pose, int* __restrict__ hyp_cnt) {
  // LDS sized by P (dynamic): the arena, then P object + P image points. At P = 256 this is
  // 43.5 KB instead of 58.9 KB for kPnpMaxP: the kernel's blocks live ~1 ms beside the fusion /
  // TBase launches, whose co-residency on those CUs the LDS footprint decides (16.42 -> 16.26
  // ms/step measured)
  extern __shared__ double pnp_dyn[];
  double* sarena = pnp_dyn;
  float* sobj = reinterpret_cast<float*>(pnp_dyn + kArena * kHypPerBlock);
  float* simg = sobj + 3 * P;
  const int b = blockIdx.x;
  const Cam cam = {K4[4 * b + 0], K4[4 * b + 1], K4[4 * b + 2], K4[4 * b + 3]};
  load_corr(b, xyz, HW, choose, N, sel, P, xmap, ymap, extent, lfb, sobj, simg);
  __syncthreads();
  const int h = blockIdx.y * kHypPerBlock + threadIdx.x;
  if (h >= H) return;
  int ids[5];
  for (int i = 0; i < 5; ++i) ids[i] = subsets[((long long)b * H + h) * 5 + i];
  Pts sub{sobj, simg, ids, 5};
  double R[9], t[3];
  epnp(SerialSum{sarena + threadIdx.x, kHypPerBlock}, sub, cam, R, t);
  float Rf[9], tf[3];
  for (int i = 0; i < 9; ++i) Rf[i] = (float)R[i];
  for (int i = 0; i < 3; ++i) tf[i] = (float)t[i];
  const float thr2 = thr * thr;
  int cnt = 0;
  for (int p = 0; p < P; ++p) cnt += is_inlier(Rf, tf, sobj + 3 * p, simg + 2 * p, cam, thr2) ? 1 : 0;
  float* o = hyp_pose + ((long long)b * H + h) * 12;
  for (int i = 0; i < 9; ++i) o[i] = Rf[i];
  for (int i = 0; i < 3; ++i) o[9 + i] = tf[i];
  hyp_cnt[(long long)b * H + h] = cnt;
}

// Phase 2: one wave per crop. Best hypothesis (most inliers, lowest index; accepted with >= 5
// inliers), its ordered inlier set, then EPnP on all inliers with the point sums spread over
// the 64 lanes.
__global__ __launch_bounds__(64) void pnp_refine_kernel(
    const float* __restrict__ xyz, int HW, const long long* __restrict__ choose, int N, const int* __restrict__ sel,
    int P, const float* __restrict__ xmap, const float* __restrict__ ymap, const float* __restrict__ K4,
    const double* __restrict__ extent, const double* __restrict__ lfb, int H, float thr,
    const float* __restrict__ hyp_pose, const int* __restrict__ hyp_cnt, float* __restrict__ Rout,
    float* __restrict__ tout, int* __restrict__ inl_out, unsigned char* __restrict__ mask_out) {
  __shared__ float sobj[kPnpMaxP * 3];
  __shared__ float simg[kPnpMaxP * 2];
  __shared__ int slist[kPnpMaxP];
  __shared__ double sarena[kArena];
  const int b = blockIdx.x;
  const int lane = threadIdx.x;
  const Cam cam = {K4[4 * b + 0], K4[4 * b + 1], K4[4 * b + 2], K4[4 * b + 3]};
  load_corr(b, xyz, HW, choose, N, sel, P, xmap, ymap, extent, lfb, sobj, simg);
  __syncthreads();
  int key = -1;
  for (int h = lane; h < H; h += 64) key = max(key, hyp_cnt[(long long)b * H + h] * 4096 + (4095 - h));
  for (int off = 32; off > 0; off >>= 1) key = max(key, __shfl_xor(key, off));
  const int best_cnt = key >= 0 ? key / 4096 : 0;
  const int best_h = key >= 0 ? 4095 - (key % 4096) : -1;
  const bool ok = best_h >= 0 && best_cnt >= 5;
  float Rf[9], tf[3];
  if (best_h >= 0) {
    const float* hp = hyp_pose + ((long long)b * H + best_h) * 12;
    for (int i = 0; i < 9; ++i) Rf[i] = hp[i];
    for (int i = 0; i < 3; ++i) tf[i] = hp[9 + i];
  }
  const float thr2 = thr * thr;
  // ordered compaction of the inliers: ballot per 64-point chunk + prefix popcount
  int n = 0;
  for (int p0 = 0; p0 < P; p0 += 64) {
    const int p = p0 + lane;
    const bool in = ok && p < P && is_inlier(Rf, tf, sobj + 3 * p, simg + 2 * p, cam, thr2);
    if (mask_out && p < P) mask_out[(long long)b * P + p] = in ? 1 : 0;
    const unsigned long long bal = __ballot(in);
    const int before = __popcll(bal & ((1ull << lane) - 1ull));
    if (in) slist[n + before] = p;
    n += __popcll(bal);
  }
  __syncthreads();
  if (ok && n >= 5) {
    Pts inl{sobj, simg, slist, n};
    double R[9], t[3];
    epnp(WaveSum{lane, sarena}, inl, cam, R, t);
    if (lane == 0) {
      for (int i = 0; i < 9; ++i) Rout[9 * b + i] = (float)R[i];
      for (int i = 0; i < 3; ++i) tout[3 * b + i] = (float)t[i];
    }
  } else if (lane == 0) {
    // RANSAC failed (< 5 inliers): cv::solvePnPRansac returns false with rvec = tvec = 0,
    // i.e. R = I, t = 0 after the Rodrigues step of trainer.py:429-435
    for (int i = 0; i < 9; ++i) Rout[9 * b + i] = (i % 4 == 0) ? 1.f : 0.f;
    for (int i = 0; i < 3; ++i) tout[3 * b + i] = 0.f;
  }
  if (lane == 0) inl_out[b] = ok ? best_cnt : 0;
}

}  // namespace

KRRN_API int krrn_pnp_ransac_f32(const float* xyz, int HW, const long long* choose, int N, const int* sel, int P,
                                 const float* xmap, const float* ymap, const float* K4, const double* extent,
                                 const double* lfborder, const int* subsets, int H, float thr, float* workspace,
                                 float* R, float* t, int* inliers, unsigned char* inlier_mask, int B, void* stream) {
  if (!xyz || !choose || !sel || !xmap || !ymap || !K4 || !extent || !lfborder || !subsets || !workspace || !R ||
      !t || !inliers)
    return KRRN_EARG;
  if (B < 1 || P < 5 || P > kPnpMaxP || H < 1 || H > 4095 || N < 1 || HW < 1) return KRRN_ESHAPE;
  hipStream_t s = (hipStream_t)stream;
  float* hyp_pose = workspace;
  int* hyp_cnt = reinterpret_cast<int*>(workspace + (size_t)B * H * 12);
  const size_t hyp_lds = sizeof(double) * kArena * kHypPerBlock + sizeof(float) * 5 * (size_t)P;
  hipLaunchKernelGGL(pnp_hyp_kernel, dim3(B, krrn_cdiv(H, kHypPerBlock)), dim3(kHypPerBlock), hyp_lds, s, xyz, HW, choose,
                     N, sel, P, xmap, ymap, K4, extent, lfborder, subsets, H, thr, hyp_pose, hyp_cnt);
  hipLaunchKernelGGL(pnp_refine_kernel, dim3(B), dim3(64), 0, s, xyz, HW, choose, N, sel, P, xmap, ymap, K4, extent,
                     lfborder, H, thr, hyp_pose, hyp_cnt, R, t, inliers, inlier_mask);
  return krrn_launch_status();
}
