// Batched PnP-RANSAC for Trainer.get_pose (tools/trainer.py:383-438):
//   cv2.solvePnPRansac(obj, img, K, None, flags=SOLVEPNP_EPNP, confidence=0.9999, reprojectionError=1)
//
//   obj[i] = float( xyz[b, :, choose[b, sel[b, i]]] * extent[b] + lfborder[b] )   (f64 math, then
//            f32 like cv::solvePnPRansac's CV_32F conversion of objectPoints)
//   img[i] = (x_map_choosed[b, sel[b, i]], y_map_choosed[b, sel[b, i]])
//   H hypotheses: EPnP on 5 correspondences each (f64), scored in parallel:
//   #{ i : ||proj(R_h, t_h, obj_i) - img_i||^2 <= thr^2 } (f32, FMA-free, the same expression as
//   oracle/pnp_ref.c); selection = ptsetreg.cpp's sequential loop over h < niters: a count above
//   max(best, modelPoints - 1) becomes the best and sets niters = RANSACUpdateNumIters(conf,
//   outlier ratio, 5, niters) (cv2's adaptive early exit, iterationsCount = H = 100);
//   refine: EPnP on every inlier of the best hypothesis; R as a rotation matrix (the
//   reference's Rodrigues round trip rvec -> kornia R is the identity map on R).
// Subsets come from the caller (krrn_ransac_subsets or explicit test inputs) so the GPU and
// the CPU oracle score identical hypotheses.
//
// Latency design: a 5-point EPnP is a chain of small dense f64 solves. Every 3x3 / 4x4 / 5x5
// symmetric eigen-solve is a fully unrolled cyclic Jacobi whose indices are all compile-time
// constants, so the matrices live in VGPRs. The 12x12 solve (M^T M), 90 % of the time when one
// thread ran it cyclically on an LDS arena (1.5 ms per 64-crop batch), is shared by a 16-lane
// group in registers with a parallel (round-robin) rotation order (eig12_group), so one
// hypothesis is one 16-lane group.
#include <math.h>

#include "krrn_common.h"

namespace {

constexpr int kPnpMaxP = 1024;

struct Cam {
  double fu, fv, uc, vc;
};

// Scheduling fence: the values are "rewritten" by an empty asm, so nothing computed after this
// point moves above it. Without these, LLVM moved the eigenvector updates (U <- U J, independent of
// the A chain) of many rotations together and held their intermediate values: the hypothesis kernel
// needed 446 registers (one wave per SIMD); with them 256 (two).
template <int N>
__device__ __forceinline__ void fence_regs(double (&v)[N]) {
#pragma unroll
  for (int i = 0; i < N; ++i) asm volatile("" : "+v"(v[i]));
}

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
        fence_regs(U);
        fence_regs(A);
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

// f64 lane shuffle (two ds_bpermute)
__device__ __forceinline__ double shfl_f64(double v, int src) {
  const unsigned long long b = __builtin_bit_cast(unsigned long long, v);
  const int lo = __shfl((int)(unsigned)b, src), hi = __shfl((int)(unsigned)(b >> 32), src);
  return __builtin_bit_cast(double, ((unsigned long long)(unsigned)hi << 32) | (unsigned)lo);
}

// v[i] for a per-lane i: select chain. Each element passes through an empty asm first: otherwise
// LLVM folds the chain back into a dynamically indexed load, which puts the array in scratch memory
// (the round-2 kernels' 1 KB / lane of scratch came from exactly this).
template <int N>
__device__ __forceinline__ double pick(const double (&v)[N], int i) {
  double r = v[0];
  asm volatile("" : "+v"(r));
#pragma unroll
  for (int j = 1; j < N; ++j) {
    double x = v[j];
    asm volatile("" : "+v"(x));
    r = (i == j) ? x : r;
  }
  return r;
}

// v[i] = x for a per-lane / runtime i (select chain, registers only)
template <int N>
__device__ __forceinline__ void put(double (&v)[N], int i, double x) {
#pragma unroll
  for (int j = 0; j < N; ++j) v[j] = (i == j) ? x : v[j];
}

// 12x12 symmetric eigen-solve (M^T M of EPnP) by the 16 lanes of an aligned lane group, lanes
// 12..15 idle: lane r < 12 holds row r of A and of U (eigenvectors as columns) in registers.
// Parallel-ordered Jacobi (round-robin / circle schedule): a sweep is 11 steps, each rotating 6
// disjoint pairs (p, q) at once -- lane r is in exactly one pair, so every lane computes its pair's
// rotation (the two lanes of a pair from identical inputs, a[p][q] taken from lane p), then
// A <- A J (each lane's own row, all 6 pairs' (c, s) shuffled in), A <- J^T A (row r combined with
// its partner's row), U <- U J. The cyclic one-rotation-at-a-time order had a dependent f64
// (theta, sqrt, division) chain per rotation, 66 per sweep; here 11 per sweep. oracle/pnp_ref.c
// (jacobi12_par) restates the same schedule and expressions. Convergence: off(A) <= 1e-30 |A|^2
// with the row sums reduced over the group by a fixed butterfly (identical in every lane).
// Rotation arithmetic without FMA contraction (as the gcc-built oracle).
__device__ __forceinline__ int rr_partner(int k, int r) {  // step k's partner of r (0 <= r < 12)
  return r == 11 ? k : (r == k ? 11 : (2 * k - r + 11) % 11);
}

__device__ __forceinline__ double group_sum16(double v) {
#pragma unroll
  for (int off = 8; off > 0; off >>= 1) v += __shfl_xor(v, off);
  return v;
}

typedef double pnp_d2 __attribute__((ext_vector_type(2)));

// In: lane r's row of M^T M (zero in lanes 12..15). Out: vq[q] = component r of the eigenvector of
// the q-th smallest eigenvalue (ascending, ties: lower column first) -- each lane keeps its own
// components only (the old form broadcast all 48 into every lane: 96 VGPRs).
// The per-step exchanges go through the group's LDS area xs (kPnpXs doubles, 16-B aligned): lane r
// writes its row at the step's start (then reads a[r][r], a[p][p], a[lo][hi] at per-lane addresses:
// two 12-way select chains before), its (c, s) (then reads the 6 pairs' (c, s)), and its row after
// A <- A J (then reads the partner's): 6 + 3 / 1 + 6 / 6 + 6 accesses per step where lane shuffles
// took 4 / 24 / 24 ds_bpermute. Lanes of one wave: the hardware keeps a wave's LDS accesses in
// order, and the wave barriers keep the compiler from moving them.
constexpr int kPnpXs = 16 * 12 + 16 * 2;
__device__ __forceinline__ void eig12_rows(const double (&row)[12], double (&vq)[4], double* xs) {
#pragma clang fp contract(off)
  const int lane = threadIdx.x & 63, r = lane & 15, base = lane & ~15;
  double* const xrow = xs;             // [16][12]
  double* const xcs = xs + 16 * 12;    // [16][2]: (c, s)
  const bool act = r < 12;
  double a[12], u[12];
#pragma unroll
  for (int j = 0; j < 12; ++j) {
    a[j] = row[j];
    u[j] = (r == j) ? 1.0 : 0.0;
  }
  for (int sweep = 0; sweep < 40; ++sweep) {
    double tot = 0.0, off = 0.0;
    if (act) {
#pragma unroll
      for (int j = 0; j < 12; ++j) {
        const double x2 = a[j] * a[j];
        tot += x2;
        if (j != r) off += x2;
      }
    }
    tot = group_sum16(tot);
    off = group_sum16(off);
    if (off <= 1e-30 * tot || off < 1e-300) break;
#pragma unroll
    for (int k = 0; k < 11; ++k) {
      const int pr = act ? rr_partner(k, r) : r;
      const int lo = r < pr ? r : pr;
      // the step's inputs from the rows in LDS (per-lane addresses instead of select chains over a[])
#pragma unroll
      for (int j = 0; j < 12; j += 2) *reinterpret_cast<pnp_d2*>(xrow + 12 * r + j) = pnp_d2{a[j], a[j + 1]};
      __builtin_amdgcn_wave_barrier();
      const int hi = r < pr ? pr : r;
      const int rc = act ? r : 11, pc = act ? pr : 11;        // idle lanes 12..15 read a valid slot
      const double d = xrow[13 * rc];                         // own diagonal
      const double dp = xrow[13 * pc];                        // partner's diagonal
      const double apq = act ? xrow[12 * lo + hi] : 0.0;      // a[lo][hi], lane lo's row
      __builtin_amdgcn_wave_barrier();
      const double app = r == lo ? d : dp, aqq = r == lo ? dp : d;
      double c = 1.0, sn = 0.0;
      if (act && !(fabs(apq) < 1e-300 || fabs(apq) < 1e-18 * sqrt(fabs(app * aqq)))) {
        const double theta = (aqq - app) / (2.0 * apq);
        const double tt = (theta >= 0 ? 1.0 : -1.0) / (fabs(theta) + sqrt(theta * theta + 1.0));
        c = 1.0 / sqrt(tt * tt + 1.0);
        sn = tt * c;
      }
      // the 6 pairs of step k: (k, 11) and ((k + i) % 11, (k - i) % 11), i = 1..5; (c, s) from the lower lane
      double cs[6], ss[6];
      int pp[6], qq[6];
      *reinterpret_cast<pnp_d2*>(xcs + 2 * r) = pnp_d2{c, sn};
      __builtin_amdgcn_wave_barrier();
#pragma unroll
      for (int i = 0; i < 6; ++i) {
        const int x = i == 0 ? k : (k + i) % 11, y = i == 0 ? 11 : (k - i + 11) % 11;
        pp[i] = x < y ? x : y;
        qq[i] = x < y ? y : x;
        const pnp_d2 v = *reinterpret_cast<const pnp_d2*>(xcs + 2 * pp[i]);
        cs[i] = v.x;
        ss[i] = v.y;
      }
      // A <- A J: own row, columns (p_i, q_i)
#pragma unroll
      for (int i = 0; i < 6; ++i) {
        const double xp = a[pp[i]], xq = a[qq[i]];
        a[pp[i]] = cs[i] * xp - ss[i] * xq;
        a[qq[i]] = ss[i] * xp + cs[i] * xq;
      }
      // A <- J^T A: row lo' = c row lo - s row hi, row hi' = s row lo + c row hi
#pragma unroll
      for (int j = 0; j < 12; j += 2) *reinterpret_cast<pnp_d2*>(xrow + 12 * r + j) = pnp_d2{a[j], a[j + 1]};
      __builtin_amdgcn_wave_barrier();
      // c a - s y (lane lo) and s y + c a (lane hi) as c a + s' y, s' = -s / s: the same IEEE results
      // (negation and the order of two addends are exact), no per-element select
      const double sgn_s = r == lo ? -sn : sn;
#pragma unroll
      for (int j = 0; j < 12; j += 2) {
        const pnp_d2 y = *reinterpret_cast<const pnp_d2*>(xrow + 12 * pr + j);
        a[j] = c * a[j] + sgn_s * y.x;
        a[j + 1] = c * a[j + 1] + sgn_s * y.y;
      }
      // U <- U J
#pragma unroll
      for (int i = 0; i < 6; ++i) {
        const double xp = u[pp[i]], xq = u[qq[i]];
        u[pp[i]] = cs[i] * xp - ss[i] * xq;
        u[qq[i]] = ss[i] * xp + cs[i] * xq;
      }
      fence_regs(u);
      fence_regs(a);
    }
  }
  double w[12];
  const double wd = pick(a, r);
#pragma unroll
  for (int i = 0; i < 12; ++i) w[i] = shfl_f64(wd, base + i);
  unsigned used = 0;
#pragma unroll
  for (int q4 = 0; q4 < 4; ++q4) {
    int mi = -1;
    double wm = 0.0;
#pragma unroll
    for (int j = 0; j < 12; ++j) {
      if (used & (1u << j)) continue;
      if (mi < 0 || w[j] < wm) { mi = j; wm = w[j]; }
    }
    used |= 1u << mi;
    vq[q4] = pick(u, mi);
  }
}

// Least squares min ||A x - b|| for the 6 x N system whose row k lives in lane k of the group
// (arow, brow; lanes >= 6 hold duplicates that are never read): the normal equations gathered row
// by row in order k = 0..5 (the expression order of oracle/pnp_ref.c), then replicated in every
// lane: Cholesky when A has full column rank (the usual case), else the pseudo-inverse from
// eig(A^T A) (OpenCV solves these with CV_SVD).
template <int N>
__device__ __forceinline__ void lsq_rows(const double (&arow)[N], double brow, double (&x)[N]) {
#pragma clang fp contract(off)
  const int base = (threadIdx.x & 63) & ~15;
  double AtA[N * N], Atb[N];
#pragma unroll
  for (int i = 0; i < N * N; ++i) AtA[i] = 0.0;
#pragma unroll
  for (int i = 0; i < N; ++i) Atb[i] = 0.0;
#pragma unroll
  for (int k = 0; k < 6; ++k) {
    double ak[N];
#pragma unroll
    for (int i = 0; i < N; ++i) ak[i] = shfl_f64(arow[i], base + k);
    const double bk = shfl_f64(brow, base + k);
#pragma unroll
    for (int i = 0; i < N; ++i) {
#pragma unroll
      for (int j = 0; j < N; ++j) AtA[i * N + j] += ak[i] * ak[j];
      Atb[i] += ak[i] * bk;
    }
    fence_regs(AtA);
  }
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
  double w[N], V[N * N];
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

__device__ __forceinline__ void alphas_of(const double* p, const double cws[4][3], const double* ci, double a[4]) {
  const double d0 = p[0] - cws[0][0], d1 = p[1] - cws[0][1], d2 = p[2] - cws[0][2];
  a[1] = ci[0] * d0 + ci[1] * d1 + ci[2] * d2;
  a[2] = ci[3] * d0 + ci[4] * d1 + ci[5] * d2;
  a[3] = ci[6] * d0 + ci[7] * d1 + ci[8] * d2;
  a[0] = 1.0 - a[1] - a[2] - a[3];
}

// Lane r's entries of row r of M^T M for one point: the two rows of M per point are
// r1 = [a_j fu, 0, a_j (uc - u)], r2 = [0, a_j fv, a_j (vc - v)] (j = 0..3).
__device__ __forceinline__ void mtm_row_add(const double* X, const double* q, const double cws[4][3], const double* ci,
                                            const Cam& cam, int r, double (&acc)[12]) {
  double a[4];
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
  // r1[r], r2[r] from a[r / 3] (a 4-way select, not two 12-way ones; the same products)
  const int jr = r / 3, tr = r - 3 * jr;
  const double aj = pick(a, jr);
  const double r1r = tr == 0 ? aj * cam.fu : (tr == 1 ? 0.0 : aj * (cam.uc - q[0]));
  const double r2r = tr == 0 ? 0.0 : (tr == 1 ? aj * cam.fv : aj * (cam.vc - q[1]));
#pragma unroll
  for (int j = 0; j < 12; ++j) acc[j] += r1r * r1[j] + r2r * r2[j];
}

// Point sums of EPnP. HypSum: one RANSAC hypothesis per aligned 16-lane group, its 5 points in
// order in every lane (the point indices are registers, so the loop is unrolled at compile time).
// WaveSum: the refinement on all inliers by one wave, points strided over the 64 lanes then a fixed
// butterfly (identical in every lane); M^T M rows strided over the 4 groups, then (g0 + g1) +
// (g2 + g3). oracle/pnp_ref.c restates both orders.
struct HypSum {
  const float* obj;  // LDS [P][3]
  const float* img;  // LDS [P][2]
  int ids[5];
  __device__ __forceinline__ void pt(int i, double* X, double* q) const {
    const float* o = obj + 3 * ids[i];
    X[0] = o[0]; X[1] = o[1]; X[2] = o[2];
    const float* u = img + 2 * ids[i];
    q[0] = u[0]; q[1] = u[1];
  }
  template <int NV, class F>
  __device__ __forceinline__ void operator()(F f, double (&acc)[NV]) const {
#pragma unroll
    for (int k = 0; k < NV; ++k) acc[k] = 0.0;
#pragma unroll
    for (int i = 0; i < 5; ++i) {
      double X[3], q[2];
      pt(i, X, q);
      f(X, q, acc);
    }
  }
  __device__ __forceinline__ int count() const { return 5; }
  __device__ __forceinline__ void rows(const double cws[4][3], const double* ci, const Cam& cam, double (&acc)[12]) const {
    const int r = threadIdx.x & 15;
#pragma unroll
    for (int j = 0; j < 12; ++j) acc[j] = 0.0;
#pragma unroll
    for (int i = 0; i < 5; ++i) {
      double X[3], q[2];
      pt(i, X, q);
      mtm_row_add(X, q, cws, ci, cam, r, acc);
    }
    if (r >= 12) {
#pragma unroll
      for (int j = 0; j < 12; ++j) acc[j] = 0.0;
    }
  }
};

struct WaveSum {
  const float* obj;
  const float* img;
  const int* list;  // LDS: the inlier indices
  int n;
  __device__ __forceinline__ void pt(int i, double* X, double* q) const {
    const int id = list[i];
    const float* o = obj + 3 * id;
    X[0] = o[0]; X[1] = o[1]; X[2] = o[2];
    const float* u = img + 2 * id;
    q[0] = u[0]; q[1] = u[1];
  }
  template <int NV, class F>
  __device__ __forceinline__ void operator()(F f, double (&acc)[NV]) const {
    const int lane = threadIdx.x & 63;
#pragma unroll
    for (int k = 0; k < NV; ++k) acc[k] = 0.0;
    for (int i = lane; i < n; i += 64) {
      double X[3], q[2];
      pt(i, X, q);
      f(X, q, acc);
    }
#pragma unroll
    for (int k = 0; k < NV; ++k) {
      double v = acc[k];
#pragma unroll
      for (int off = 32; off > 0; off >>= 1) v += __shfl_xor(v, off);
      acc[k] = v;
    }
  }
  __device__ __forceinline__ int count() const { return n; }
  __device__ __forceinline__ void rows(const double cws[4][3], const double* ci, const Cam& cam, double (&acc)[12]) const {
    const int lane = threadIdx.x & 63, r = lane & 15, g = lane >> 4;
#pragma unroll
    for (int j = 0; j < 12; ++j) acc[j] = 0.0;
    for (int i = g; i < n; i += 4) {
      double X[3], q[2];
      pt(i, X, q);
      mtm_row_add(X, q, cws, ci, cam, r, acc);
    }
#pragma unroll
    for (int j = 0; j < 12; ++j) {
      double v = acc[j];
      v = v + __shfl_xor(v, 16);
      v = v + __shfl_xor(v, 32);
      acc[j] = r < 12 ? v : 0.0;
    }
  }
};

__device__ __forceinline__ void gauss_newton(const double (&Lr)[10], double rho_r, double (&betas)[4]) {
#pragma unroll 1
  for (int it = 0; it < 5; ++it) {
    const double* l = Lr;
    double a[4], x[4];
    a[0] = 2 * l[0] * betas[0] + l[1] * betas[1] + l[3] * betas[2] + l[6] * betas[3];
    a[1] = l[1] * betas[0] + 2 * l[2] * betas[1] + l[4] * betas[2] + l[7] * betas[3];
    a[2] = l[3] * betas[0] + l[4] * betas[1] + 2 * l[5] * betas[2] + l[8] * betas[3];
    a[3] = l[6] * betas[0] + l[7] * betas[1] + l[8] * betas[2] + 2 * l[9] * betas[3];
    const double b = rho_r - (l[0] * betas[0] * betas[0] + l[1] * betas[0] * betas[1] + l[2] * betas[1] * betas[1] +
                              l[3] * betas[0] * betas[2] + l[4] * betas[1] * betas[2] + l[5] * betas[2] * betas[2] +
                              l[6] * betas[0] * betas[3] + l[7] * betas[1] * betas[3] + l[8] * betas[2] * betas[3] +
                              l[9] * betas[3] * betas[3]);
    lsq_rows<4>(a, b, x);
#pragma unroll
    for (int k = 0; k < 4; ++k) betas[k] += x[k];
  }
}

// Procrustes on the 3x3 correlation H = sum (pc - cc)(pw - cw)^T as OpenCV's epnp.cpp
// estimate_R_and_t does it: R = U V^T of H's SVD, and when det(R) < 0 its third row negated. For a
// rank-3 H, U V^T is the polar factor (det = sign det H), which is the Kabsch rotation
// U diag(1,1,1) V^T when det H > 0 and U diag(1,1,-1) V^T otherwise (u2 = u0 x u1, v2 = v0 x v1 below).
// A rank-deficient H (coplanar points) leaves cv2's result to its SVD's sign choices; it is kept
// proper (Kabsch) here. oracle/pnp_ref.c restates it (kabsch).
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
  const double detH = H[0] * (H[4] * H[8] - H[5] * H[7]) - H[1] * (H[3] * H[8] - H[5] * H[6]) +
                      H[2] * (H[3] * H[7] - H[4] * H[6]);
  const bool refl = detH < 0.0 && w[2] > 1e-24 * w[0];
  const double s2 = refl ? -1.0 : 1.0;
#pragma unroll
  for (int r = 0; r < 3; ++r)
#pragma unroll
    for (int c = 0; c < 3; ++c) R[r * 3 + c] = U[r] * V[c] + U[3 + r] * V[3 + c] + (s2 * U[6 + r]) * v2[c];
  if (refl) {
    R[6] = -R[6]; R[7] = -R[7]; R[8] = -R[8];
  }
}

// R, t from betas (lane r holds component r of the 4 null-space vectors: vq); returns the mean
// reprojection error. Forced inline like epnp below: as real calls (the compiler's choice for
// functions this size) their struct / array arguments went through the stack, 216 B of scratch
// per lane of the hypothesis kernel, written once per hypothesis.
template <class SUM>
__device__ __forceinline__ double r_and_t(const SUM& sum, const double (&vq)[4], const double (&betas)[4], const double cws[4][3],
                          const double* ci, const double* cw, const Cam& cam, double (&R)[9], double (&t)[3]) {
  const int base = (threadIdx.x & 63) & ~15;
  double cr = 0.0;
#pragma unroll
  for (int i = 0; i < 4; ++i) cr += betas[i] * vq[i];
  double ccs[4][3];
#pragma unroll
  for (int j = 0; j < 4; ++j)
#pragma unroll
    for (int k = 0; k < 3; ++k) ccs[j][k] = shfl_f64(cr, base + 3 * j + k);
  // solve_for_sign: the first point must lie in front of the camera
  double p0[3], q0[2], a0[4];
  sum.pt(0, p0, q0);
  alphas_of(p0, cws, ci, a0);
  const double z0 = a0[0] * ccs[0][2] + a0[1] * ccs[1][2] + a0[2] * ccs[2][2] + a0[3] * ccs[3][2];
  const double sg = z0 < 0.0 ? -1.0 : 1.0;
  const int n = sum.count();
  double cc[3];
  sum([&](const double* X, const double*, double (&acc)[3]) {
        double a[4];
        alphas_of(X, cws, ci, a);
#pragma unroll
        for (int k = 0; k < 3; ++k) acc[k] += sg * (a[0] * ccs[0][k] + a[1] * ccs[1][k] + a[2] * ccs[2][k] + a[3] * ccs[3][k]);
      }, cc);
#pragma unroll
  for (int k = 0; k < 3; ++k) cc[k] /= n;
  double H[9];
  sum([&](const double* X, const double*, double (&acc)[9]) {
        double a[4], pc[3];
        alphas_of(X, cws, ci, a);
#pragma unroll
        for (int k = 0; k < 3; ++k) pc[k] = sg * (a[0] * ccs[0][k] + a[1] * ccs[1][k] + a[2] * ccs[2][k] + a[3] * ccs[3][k]);
#pragma unroll
        for (int r = 0; r < 3; ++r)
#pragma unroll
          for (int c = 0; c < 3; ++c) acc[r * 3 + c] += (pc[r] - cc[r]) * (X[c] - cw[c]);
      }, H);
  kabsch(H, R);
#pragma unroll
  for (int r = 0; r < 3; ++r) t[r] = cc[r] - (R[r * 3 + 0] * cw[0] + R[r * 3 + 1] * cw[1] + R[r * 3 + 2] * cw[2]);
  double err[1];
  sum([&](const double* X, const double* q, double (&acc)[1]) {
        const double Xc = dot3(R, X) + t[0], Yc = dot3(R + 3, X) + t[1], Zc = dot3(R + 6, X) + t[2];
        const double iz = 1.0 / Zc;
        const double du = q[0] - (cam.uc + cam.fu * Xc * iz), dv = q[1] - (cam.vc + cam.fv * Yc * iz);
        acc[0] += sqrt(du * du + dv * dv);
      }, err);
  return err[0] / n;
}

// EPnP (Lepetit et al. 2009) over the points of `sum`, spread over an aligned 16-lane group: the
// point sums and the small dense algebra replicated in every lane, the rows of M^T M, of the 6 x 10
// L matrix and of every 6 x N least-squares system one per lane, the 12 x 12 eigen-solve shared
// (eig12_rows). Result R (row-major), t as f32 (the precision both callers keep), identical in every
// lane of the group. The control points and their inverse (cws, ci; 21 values, the same in every lane)
// live in the group's LDS slot `ctl` after the setup: in registers they were 42 more VGPRs through
// the whole solve.
template <class SUM>
__device__ __forceinline__ void epnp(const SUM& sum, const Cam& cam, double* ctl, float (&Rout)[9], float (&tout)[3]) {
#pragma clang fp contract(off)
  const int lane = threadIdx.x & 63, r = lane & 15, base = lane & ~15;
  const int n = sum.count();
  {
    double cws[4][3], ci[9], cw[3];
    sum([&](const double* X, const double*, double (&acc)[3]) {
          acc[0] += X[0]; acc[1] += X[1]; acc[2] += X[2];
        }, cw);
#pragma unroll
    for (int j = 0; j < 3; ++j) cw[j] /= n;
    double C6[6];
    sum([&](const double* X, const double*, double (&acc)[6]) {
          const double d0 = X[0] - cw[0], d1 = X[1] - cw[1], d2 = X[2] - cw[2];
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
#pragma unroll
    for (int j = 0; j < 12; ++j) ctl[j] = cws[j / 3][j % 3];
#pragma unroll
    for (int i = 0; i < 9; ++i) ctl[12 + i] = ci[i];
  }
  asm volatile("" ::: "memory");  // read back from LDS below, not forwarded in registers
  const double(*cws)[3] = reinterpret_cast<const double(*)[3]>(ctl);
  const double* ci = ctl + 12;
  const double* cw = ctl;  // cws[0] is the centroid
  double vq[4];
  {
    double mrow[12];
    sum.rows(cws, ci, cam, mrow);
    eig12_rows(mrow, vq, ctl + 32);
  }
  // lane i < 6: row i of L (6 x 10) and rho[i]; pair (a, b) of control points per row
  const int li = r < 6 ? r : 5;
  const int pa = li < 3 ? 0 : (li < 5 ? 1 : 2);
  const int pb = li < 3 ? li + 1 : (li < 5 ? li - 1 : 3);
  double Lr[10], rho_r;
  {
    double dv[4][3];
#pragma unroll
    for (int q = 0; q < 4; ++q)
#pragma unroll
      for (int k = 0; k < 3; ++k) dv[q][k] = shfl_f64(vq[q], base + 3 * pa + k) - shfl_f64(vq[q], base + 3 * pb + k);
    Lr[0] = dot3(dv[0], dv[0]);
    Lr[1] = 2.0 * dot3(dv[0], dv[1]);
    Lr[2] = dot3(dv[1], dv[1]);
    Lr[3] = 2.0 * dot3(dv[0], dv[2]);
    Lr[4] = 2.0 * dot3(dv[1], dv[2]);
    Lr[5] = dot3(dv[2], dv[2]);
    Lr[6] = 2.0 * dot3(dv[0], dv[3]);
    Lr[7] = 2.0 * dot3(dv[1], dv[3]);
    Lr[8] = 2.0 * dot3(dv[2], dv[3]);
    Lr[9] = dot3(dv[3], dv[3]);
    double rho6[6];
    int a = 0, b = 1;
#pragma unroll
    for (int j = 0; j < 6; ++j) {
      const double d0 = cws[a][0] - cws[b][0], d1 = cws[a][1] - cws[b][1], d2 = cws[a][2] - cws[b][2];
      rho6[j] = d0 * d0 + d1 * d1 + d2 * d2;
      if (++b > 3) { ++a; b = a + 1; }
    }
    rho_r = pick(rho6, li);
  }
  double best_err = 1e300;
#pragma unroll 1
  for (int approx = 1; approx <= 3; ++approx) {
    asm volatile("" ::: "memory");  // keeps the LDS reads of cws / ci in the loop body
    double betas[4] = {0, 0, 0, 0};
    if (approx == 1) {
      const double arow[4] = {Lr[0], Lr[1], Lr[3], Lr[6]};
      double x[4];
      lsq_rows<4>(arow, rho_r, x);
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
      const double arow[3] = {Lr[0], Lr[1], Lr[2]};
      double x[3];
      lsq_rows<3>(arow, rho_r, x);
      if (x[0] < 0) {
        betas[0] = sqrt(-x[0]);
        betas[1] = (x[2] < 0) ? sqrt(-x[2]) : 0.0;
      } else {
        betas[0] = sqrt(x[0]);
        betas[1] = (x[2] > 0) ? sqrt(x[2]) : 0.0;
      }
      if (x[1] < 0) betas[0] = -betas[0];
    } else {
      const double arow[5] = {Lr[0], Lr[1], Lr[2], Lr[3], Lr[4]};
      double x[5];
      lsq_rows<5>(arow, rho_r, x);
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
    gauss_newton(Lr, rho_r, betas);
    double R[9], t[3];
    const double err = r_and_t(sum, vq, betas, cws, ci, cw, cam, R, t);
    if (approx == 1 || err < best_err) {
      best_err = err;
#pragma unroll
      for (int i = 0; i < 9; ++i) Rout[i] = (float)R[i];
#pragma unroll
      for (int i = 0; i < 3; ++i) tout[i] = (float)t[i];
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

// Phase 1: one RANSAC hypothesis per 16-lane group, kHypPerBlock per block, grid (B, ceil(H / kHypPerBlock)). Writes the
// f32 pose (R, t: the precision the inlier test uses) and the inlier count of every hypothesis. LDS:
// the P correspondences only (5 KB at P = 256), so the blocks co-reside with the fusion / TBase
// launches they run beside; no scratch memory (every register array has compile-time indices).
template <int kHypPerBlock>
__global__ __launch_bounds__(16 * kHypPerBlock, 2) void pnp_hyp_kernel(
    const float* __restrict__ xyz, int HW, const long long* __restrict__ choose, int N, const int* __restrict__ sel,
    int P, const float* __restrict__ xmap, const float* __restrict__ ymap, const float* __restrict__ K4,
    const double* __restrict__ extent, const double* __restrict__ lfb, const int* __restrict__ subsets, int H,
    float thr, float* __restrict__ hyp_pose, int* __restrict__ hyp_cnt) {
  extern __shared__ float pnp_corr[];
  __shared__ __attribute__((aligned(16))) double sctl[kHypPerBlock][32 + kPnpXs];
  float* sobj = pnp_corr;
  float* simg = sobj + 3 * P;
  const int b = blockIdx.x;
  const Cam cam = {K4[4 * b + 0], K4[4 * b + 1], K4[4 * b + 2], K4[4 * b + 3]};
  load_corr(b, xyz, HW, choose, N, sel, P, xmap, ymap, extent, lfb, sobj, simg);
  __syncthreads();
  const int r = threadIdx.x & 15;
  const int h = blockIdx.y * kHypPerBlock + (threadIdx.x >> 4);
  const int hs = h < H ? h : H - 1;  // a tail group solves a duplicate (whole groups stay active) and writes nothing
  HypSum sub;
  sub.obj = sobj;
  sub.img = simg;
#pragma unroll
  for (int i = 0; i < 5; ++i) sub.ids[i] = subsets[((long long)b * H + hs) * 5 + i];
  float Rf[9], tf[3];
  epnp(sub, cam, sctl[threadIdx.x >> 4], Rf, tf);
  const float thr2 = thr * thr;
  int cnt = 0;
  for (int p = r; p < P; p += 16) cnt += is_inlier(Rf, tf, sobj + 3 * p, simg + 2 * p, cam, thr2) ? 1 : 0;
#pragma unroll
  for (int off = 8; off > 0; off >>= 1) cnt += __shfl_xor(cnt, off);
  if (h >= H || r != 0) return;
  float* o = hyp_pose + ((long long)b * H + h) * 12;
#pragma unroll
  for (int i = 0; i < 9; ++i) o[i] = Rf[i];
#pragma unroll
  for (int i = 0; i < 3; ++i) o[9 + i] = tf[i];
  hyp_cnt[(long long)b * H + h] = cnt;
}

// cv::RANSACUpdateNumIters (ptsetreg.cpp): iterations needed for `conf` given outlier ratio ep
__device__ __forceinline__ int ransac_update_niters(double conf, double ep, int model_points, int max_iters) {
  conf = fmin(fmax(conf, 0.0), 1.0);
  ep = fmin(fmax(ep, 0.0), 1.0);
  double num = fmax(1.0 - conf, 2.2250738585072014e-308);
  double denom = 1.0 - pow(1.0 - ep, (double)model_points);
  if (denom < 2.2250738585072014e-308) return 0;
  num = log(num);
  denom = log(denom);
  return (denom >= 0 || -num >= max_iters * (-denom)) ? max_iters : (int)rint(num / denom);
}

// Phase 2: one wave per crop. The RANSAC loop of ptsetreg.cpp over the scored hypotheses in
// order: hypothesis h is considered while h < niters; a strictly better count (and >= 5 inliers:
// goodCount > max(maxGoodCount, modelPoints - 1)) becomes the best and lowers niters to
// RANSACUpdateNumIters(confidence, outlier ratio, 5, niters). Then the best hypothesis' ordered
// inlier set and EPnP on all inliers (WaveSum: the point sums spread over the 64 lanes, each of the 4
// lane groups solving the same replicated system).
__global__ __launch_bounds__(64) void pnp_refine_kernel(
    const float* __restrict__ xyz, int HW, const long long* __restrict__ choose, int N, const int* __restrict__ sel,
    int P, const float* __restrict__ xmap, const float* __restrict__ ymap, const float* __restrict__ K4,
    const double* __restrict__ extent, const double* __restrict__ lfb, int H, float thr, double conf,
    const float* __restrict__ hyp_pose, const int* __restrict__ hyp_cnt, float* __restrict__ Rout,
    float* __restrict__ tout, int* __restrict__ inl_out, unsigned char* __restrict__ mask_out) {
  __shared__ float sobj[kPnpMaxP * 3];
  __shared__ float simg[kPnpMaxP * 2];
  __shared__ int slist[kPnpMaxP];
  __shared__ __attribute__((aligned(16))) double sctl[4][32 + kPnpXs];
  const int b = blockIdx.x;
  const int lane = threadIdx.x;
  const Cam cam = {K4[4 * b + 0], K4[4 * b + 1], K4[4 * b + 2], K4[4 * b + 3]};
  load_corr(b, xyz, HW, choose, N, sel, P, xmap, ymap, extent, lfb, sobj, simg);
  __syncthreads();
  // the sequential scan (every lane, identical): counts come 64 at a time through one load each
  int best_h = -1, best_cnt = 0, niters = H;
  for (int h0 = 0; h0 < niters; h0 += 64) {
    const int mine = h0 + lane < H ? hyp_cnt[(long long)b * H + h0 + lane] : 0;
    for (int i = 0; i < 64 && h0 + i < niters; ++i) {
      const int cnt = __shfl(mine, i);
      if (cnt > (best_cnt > 4 ? best_cnt : 4)) {
        best_cnt = cnt;
        best_h = h0 + i;
        niters = ransac_update_niters(conf, (double)(P - cnt) / P, 5, niters);
      }
    }
  }
  const bool ok = best_h >= 0;
  float Rf[9], tf[3];
  {
    const float* hp = hyp_pose + ((long long)b * H + (ok ? best_h : 0)) * 12;
#pragma unroll
    for (int i = 0; i < 9; ++i) Rf[i] = ok ? hp[i] : 0.f;
#pragma unroll
    for (int i = 0; i < 3; ++i) tf[i] = ok ? hp[9 + i] : 0.f;
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
    const WaveSum inl{sobj, simg, slist, n};
    float R[9], t[3];
    epnp(inl, cam, sctl[lane >> 4], R, t);
    if (lane == 0) {
#pragma unroll
      for (int i = 0; i < 9; ++i) Rout[9 * b + i] = R[i];
#pragma unroll
      for (int i = 0; i < 3; ++i) tout[3 * b + i] = t[i];
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
                                 const double* lfborder, const int* subsets, int H, float thr, double conf,
                                 float* workspace, float* R, float* t, int* inliers, unsigned char* inlier_mask, int B,
                                 void* stream) {
  if (!xyz || !choose || !sel || !xmap || !ymap || !K4 || !extent || !lfborder || !subsets || !workspace || !R ||
      !t || !inliers)
    return KRRN_EARG;
  if (B < 1 || P < 5 || P > kPnpMaxP || H < 1 || H > 4095 || N < 1 || HW < 1 || !(conf >= 0.0 && conf <= 1.0))
    return KRRN_ESHAPE;
  hipStream_t s = (hipStream_t)stream;
  float* hyp_pose = workspace;
  int* hyp_cnt = reinterpret_cast<int*>(workspace + (size_t)B * H * 12);
  // hypotheses per block: 4 (one wave) leaves no idle tail groups at H = 100 and schedules at wave
  // granularity (occupancy is one wave per SIMD either way; the round-2 4-wave blocks of 16 were slower)
  hipLaunchKernelGGL(pnp_hyp_kernel<4>, dim3(B, krrn_cdiv(H, 4)), dim3(64), sizeof(float) * 5 * (size_t)P, s,
                     xyz, HW, choose, N, sel, P, xmap, ymap, K4, extent, lfborder, subsets, H, thr, hyp_pose, hyp_cnt);
  hipLaunchKernelGGL(pnp_refine_kernel, dim3(B), dim3(64), 0, s, xyz, HW, choose, N, sel, P, xmap, ymap, K4, extent,
                     lfborder, H, thr, conf, hyp_pose, hyp_cnt, R, t, inliers, inlier_mask);
  return krrn_launch_status();
}
