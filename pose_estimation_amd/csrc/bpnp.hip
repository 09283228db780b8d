// Back-propagatable PnP (lib/network/dnn/BPnP.py).
//
//   forward  (BPnP.py:24-51): the pose y = (angle-axis w, t) minimising the summed squared
//            reprojection error from an initial pose — cv2.solvePnP(SOLVEPNP_ITERATIVE,
//            useExtrinsicGuess=True) restated as Levenberg-Marquardt (krrn_bpnp_solve_f32).
//   backward (BPnP.py:53-117): implicit-function gradients. Per crop and pose parameter j
//            f_j = sum_i sum_k c_ikj r_ik,  r_i = x_i s_i - q_i[0:2],  q_i = K (R(w) z_i + t),
//            s_i = q_i[2],  c_ikj = -2 d(q_ik / s_i) / d y_j  (differentiated too: create_graph),
//            J_f* = d f / d(y, x, z, K);  grad_* = -g J_fy^-1 J_f*  (krrn_bpnp_backward_f32).
//
// R(w) is kornia's angle_axis_to_rotation_matrix (Rodrigues with w / (theta + 1e-6); first
// order I + [w]x where theta^2 <= 1e-6), evaluated once per crop with its first and second
// derivatives in a value / gradient / Hessian number (D2). Everything per point is analytic:
// with Q_j = d q / d y_j and g_kj = (Q_jk s - q_k Q_j2) / s^2 (c = -2 g), a perturbation
// (dq, dQ) of any input gives dg_kj = (dQ_jk s + Q_jk ds - dq_k Q_j2 - q_k dQ_j2) / s^2
// - 2 g_kj ds / s and dr_k = x_k ds - dq_k, so each column of J_fy / J_fz / J_fK is one
// directional derivative. All arithmetic is f64 (the reference runs autograd in f32).
//
// One 64-lane wave per crop, points strided over lanes; per-lane sums are combined by a fixed
// butterfly (deterministic); the 6x6 systems are solved redundantly by every lane (partial
// pivoting). The batch sums of grad_z / grad_K (BPnP.py:114-115) are a second launch that adds
// the per-crop partials in crop order.
#include <math.h>

#include "krrn_common.h"

namespace {

constexpr double kKorniaEps = 1e-6;

// value, gradient and Hessian w.r.t. the three angle-axis components
struct D2 {
  double v, g[3], h[3][3];
};

__device__ inline D2 d2_const(double c) {
  D2 r;
  r.v = c;
#pragma unroll
  for (int i = 0; i < 3; ++i) {
    r.g[i] = 0.0;
#pragma unroll
    for (int j = 0; j < 3; ++j) r.h[i][j] = 0.0;
  }
  return r;
}
__device__ inline D2 d2_var(double c, int i) {
  D2 r = d2_const(c);
  r.g[i] = 1.0;
  return r;
}
__device__ inline D2 operator+(const D2& a, const D2& b) {
  D2 r;
  r.v = a.v + b.v;
#pragma unroll
  for (int i = 0; i < 3; ++i) {
    r.g[i] = a.g[i] + b.g[i];
#pragma unroll
    for (int j = 0; j < 3; ++j) r.h[i][j] = a.h[i][j] + b.h[i][j];
  }
  return r;
}
__device__ inline D2 operator-(const D2& a, const D2& b) {
  D2 r;
  r.v = a.v - b.v;
#pragma unroll
  for (int i = 0; i < 3; ++i) {
    r.g[i] = a.g[i] - b.g[i];
#pragma unroll
    for (int j = 0; j < 3; ++j) r.h[i][j] = a.h[i][j] - b.h[i][j];
  }
  return r;
}
__device__ inline D2 operator-(const D2& a) { return d2_const(0.0) - a; }
__device__ inline D2 operator*(const D2& a, const D2& b) {
  D2 r;
  r.v = a.v * b.v;
#pragma unroll
  for (int i = 0; i < 3; ++i) {
    r.g[i] = a.g[i] * b.v + a.v * b.g[i];
#pragma unroll
    for (int j = 0; j < 3; ++j) r.h[i][j] = a.h[i][j] * b.v + a.g[i] * b.g[j] + a.g[j] * b.g[i] + a.v * b.h[i][j];
  }
  return r;
}
// f(a) from f(a.v), f'(a.v), f''(a.v)
__device__ inline D2 d2_apply(const D2& a, double f, double f1, double f2) {
  D2 r;
  r.v = f;
#pragma unroll
  for (int i = 0; i < 3; ++i) {
    r.g[i] = f1 * a.g[i];
#pragma unroll
    for (int j = 0; j < 3; ++j) r.h[i][j] = f2 * a.g[i] * a.g[j] + f1 * a.h[i][j];
  }
  return r;
}
__device__ inline D2 d2_sqrt(const D2& a) {
  const double s = sqrt(a.v);
  return d2_apply(a, s, 0.5 / s, -0.25 / (s * a.v));
}
__device__ inline D2 d2_inv(const D2& a) { return d2_apply(a, 1.0 / a.v, -1.0 / (a.v * a.v), 2.0 / (a.v * a.v * a.v)); }
__device__ inline D2 d2_sin(const D2& a) { return d2_apply(a, sin(a.v), cos(a.v), -sin(a.v)); }
__device__ inline D2 d2_cos(const D2& a) { return d2_apply(a, cos(a.v), -sin(a.v), -cos(a.v)); }

// R[a][b] with dR/dw_j and d2R/dw_j dw_l (kornia's formula, see the header)
struct Rot {
  double R[3][3];
  double dR[3][3][3];      // [j][a][b]
  double d2R[3][3][3][3];  // [j][l][a][b]
};

__device__ inline void rodrigues(const double w0, const double w1, const double w2, Rot& o) {
  const D2 w[3] = {d2_var(w0, 0), d2_var(w1, 1), d2_var(w2, 2)};
  D2 M[3][3];
  const double th2v = w0 * w0 + w1 * w1 + w2 * w2;
  if (th2v > kKorniaEps) {
    const D2 th2 = w[0] * w[0] + w[1] * w[1] + w[2] * w[2];
    const D2 th = d2_sqrt(th2);
    const D2 inv = d2_inv(th + d2_const(kKorniaEps));
    const D2 x = w[0] * inv, y = w[1] * inv, z = w[2] * inv;
    const D2 c = d2_cos(th), s = d2_sin(th);
    const D2 oc = d2_const(1.0) - c;
    M[0][0] = c + x * x * oc;
    M[0][1] = x * y * oc - z * s;
    M[0][2] = y * s + x * z * oc;
    M[1][0] = z * s + x * y * oc;
    M[1][1] = c + y * y * oc;
    M[1][2] = -(x * s) + y * z * oc;
    M[2][0] = -(y * s) + x * z * oc;
    M[2][1] = x * s + y * z * oc;
    M[2][2] = c + z * z * oc;
  } else {
    const D2 one = d2_const(1.0);
    M[0][0] = one;   M[0][1] = -w[2]; M[0][2] = w[1];
    M[1][0] = w[2];  M[1][1] = one;   M[1][2] = -w[0];
    M[2][0] = -w[1]; M[2][1] = w[0];  M[2][2] = one;
  }
#pragma unroll
  for (int a = 0; a < 3; ++a)
#pragma unroll
    for (int b = 0; b < 3; ++b) {
      o.R[a][b] = M[a][b].v;
#pragma unroll
      for (int j = 0; j < 3; ++j) {
        o.dR[j][a][b] = M[a][b].g[j];
#pragma unroll
        for (int l = 0; l < 3; ++l) o.d2R[j][l][a][b] = M[a][b].h[j][l];
      }
    }
}

// Element e = 3a + b of the same R, dR, d2R (the same D2 operations as rodrigues, one entry):
// nine lanes build a crop's rotation side by side instead of lane 0 holding all nine D2 entries
// (117 doubles, which went to scratch in the backward kernel).
__device__ inline void rodrigues_elem(const double w0, const double w1, const double w2, int e, Rot& o) {
  const D2 w[3] = {d2_var(w0, 0), d2_var(w1, 1), d2_var(w2, 2)};
  const int a = e / 3, b = e % 3;
  D2 m;
  const double th2v = w0 * w0 + w1 * w1 + w2 * w2;
  if (th2v > kKorniaEps) {
    const D2 th2 = w[0] * w[0] + w[1] * w[1] + w[2] * w[2];
    const D2 th = d2_sqrt(th2);
    const D2 inv = d2_inv(th + d2_const(kKorniaEps));
    const D2 x = w[0] * inv, y = w[1] * inv, z = w[2] * inv;
    const D2 c = d2_cos(th), s = d2_sin(th);
    const D2 oc = d2_const(1.0) - c;
    switch (e) {
      case 0: m = c + x * x * oc; break;
      case 1: m = x * y * oc - z * s; break;
      case 2: m = y * s + x * z * oc; break;
      case 3: m = z * s + x * y * oc; break;
      case 4: m = c + y * y * oc; break;
      case 5: m = -(x * s) + y * z * oc; break;
      case 6: m = -(y * s) + x * z * oc; break;
      case 7: m = x * s + y * z * oc; break;
      default: m = c + z * z * oc; break;
    }
  } else {
    switch (e) {
      case 1: m = -w[2]; break;
      case 2: m = w[1]; break;
      case 3: m = w[2]; break;
      case 5: m = -w[0]; break;
      case 6: m = -w[1]; break;
      case 7: m = w[0]; break;
      default: m = d2_const(1.0); break;
    }
  }
  o.R[a][b] = m.v;
#pragma unroll
  for (int j = 0; j < 3; ++j) {
    o.dR[j][a][b] = m.g[j];
#pragma unroll
    for (int l = 0; l < 3; ++l) o.d2R[j][l][a][b] = m.h[j][l];
  }
}

__device__ inline void matvec(const double (&A)[3][3], const double (&v)[3], double (&o)[3]) {
#pragma unroll
  for (int a = 0; a < 3; ++a) o[a] = A[a][0] * v[0] + A[a][1] * v[1] + A[a][2] * v[2];
}

__device__ inline double wave_sum(double v) {
#pragma unroll
  for (int o = 32; o >= 1; o >>= 1) v += __shfl_xor(v, o, 64);
  return v;
}

// Solve A x = b (6x6, partial pivoting); A, b overwritten. Returns false if singular.
__device__ inline bool solve6(double (&A)[6][6], double (&b)[6], double (&x)[6]) {
#pragma unroll
  for (int c = 0; c < 6; ++c) {
    int p = c;
    double best = fabs(A[c][c]);
#pragma unroll
    for (int r = c + 1; r < 6; ++r)
      if (fabs(A[r][c]) > best) { best = fabs(A[r][c]); p = r; }
    if (!(best > 0.0)) return false;
    // row swap c <-> p as selects over the candidate rows (a branch on the pivot row let the
    // compiler index A dynamically and put it in scratch)
#pragma unroll
    for (int r = c + 1; r < 6; ++r) {
      const bool sw = r == p;
#pragma unroll
      for (int k = 0; k < 6; ++k) {
        const double t = A[r][k];
        A[r][k] = sw ? A[c][k] : t;
        A[c][k] = sw ? t : A[c][k];
      }
      const double t = b[r];
      b[r] = sw ? b[c] : t;
      b[c] = sw ? t : b[c];
    }
#pragma unroll
    for (int r = c + 1; r < 6; ++r) {
      const double f = A[r][c] / A[c][c];
#pragma unroll
      for (int k = c; k < 6; ++k) A[r][k] -= f * A[c][k];
      b[r] -= f * b[c];
    }
  }
#pragma unroll
  for (int r = 5; r >= 0; --r) {
    double s = b[r];
#pragma unroll
    for (int k = r + 1; k < 6; ++k) s -= A[r][k] * x[k];
    x[r] = s / A[r][r];
  }
  return true;
}

// Per-point geometry shared by forward and backward.
struct PointGeo {
  double p[3], q[3], s;  // camera point, K p, depth row
  double Dz[3][3];       // dR_j z  (j < 3)
  double Q[6][3];        // dq / dy_j
  double g[2][6];        // d pi_k / d y_j
};

__device__ inline void point_geo(const Rot& r, const double (&K)[3][3], const double (&t)[3], const double (&z)[3],
                                 PointGeo& o) {
  double Rz[3];
  matvec(r.R, z, Rz);
#pragma unroll
  for (int a = 0; a < 3; ++a) o.p[a] = Rz[a] + t[a];
  matvec(K, o.p, o.q);
  o.s = o.q[2];
#pragma unroll
  for (int j = 0; j < 3; ++j) {
    matvec(r.dR[j], z, o.Dz[j]);
    matvec(K, o.Dz[j], o.Q[j]);
  }
#pragma unroll
  for (int j = 3; j < 6; ++j)
#pragma unroll
    for (int a = 0; a < 3; ++a) o.Q[j][a] = K[a][j - 3];
  const double is2 = 1.0 / (o.s * o.s);
#pragma unroll
  for (int k = 0; k < 2; ++k)
#pragma unroll
    for (int j = 0; j < 6; ++j) o.g[k][j] = (o.Q[j][k] * o.s - o.q[k] * o.Q[j][2]) * is2;
}

// d f_j along one input direction given (dq, dQ_j): sum_k dc_kj r_k + c_kj dr_k
__device__ inline void dir_deriv(const PointGeo& G, const double (&x)[2], const double (&r)[2], const double (&dq)[3],
                                 const double (&dQ)[6][3], double (&df)[6]) {
  const double ds = dq[2], is2 = 1.0 / (G.s * G.s);
  double dr[2];
#pragma unroll
  for (int k = 0; k < 2; ++k) dr[k] = x[k] * ds - dq[k];
#pragma unroll
  for (int j = 0; j < 6; ++j) {
    double acc = 0.0;
#pragma unroll
    for (int k = 0; k < 2; ++k) {
      const double dg = (dQ[j][k] * G.s + G.Q[j][k] * ds - dq[k] * G.Q[j][2] - G.q[k] * dQ[j][2]) * is2 -
                        2.0 * G.g[k][j] * ds / G.s;
      acc += -2.0 * dg * r[k] + -2.0 * G.g[k][j] * dr[k];
    }
    df[j] = acc;
  }
}

// d f / d z_m for m = 0..2 -> Jz[j][m]
__device__ inline void dz_cols(const Rot& R, const double (&K)[3][3], const PointGeo& G, const double (&x)[2],
                               const double (&r)[2], double (&Jz)[6][3]) {
#pragma unroll
  for (int m = 0; m < 3; ++m) {
    double col[3], dq[3], dQ[6][3];
#pragma unroll
    for (int a = 0; a < 3; ++a) col[a] = R.R[a][m];
    matvec(K, col, dq);
#pragma unroll
    for (int j = 0; j < 3; ++j) {
#pragma unroll
      for (int a = 0; a < 3; ++a) col[a] = R.dR[j][a][m];
      matvec(K, col, dQ[j]);
    }
#pragma unroll
    for (int j = 3; j < 6; ++j) dQ[j][0] = dQ[j][1] = dQ[j][2] = 0.0;
    double df[6];
    dir_deriv(G, x, r, dq, dQ, df);
#pragma unroll
    for (int j = 0; j < 6; ++j) Jz[j][m] = df[j];
  }
}

struct CropIn {
  Rot R;
  double K[3][3], t[3], w[3];
};

// the crop's pose, K and rotation derivatives, built into LDS (uniform over the wave): lane 0 the
// pose and K, lanes 0-8 one rotation entry each
__device__ inline void load_crop(const float* P6, const float* Kp, int b, CropIn& c) {
  if (threadIdx.x == 0) {
#pragma unroll
    for (int a = 0; a < 3; ++a) {
      c.w[a] = (double)P6[b * 6 + a];
      c.t[a] = (double)P6[b * 6 + 3 + a];
#pragma unroll
      for (int e = 0; e < 3; ++e) c.K[a][e] = (double)Kp[3 * a + e];
    }
  }
  if (threadIdx.x < 9)
    rodrigues_elem((double)P6[b * 6], (double)P6[b * 6 + 1], (double)P6[b * 6 + 2], threadIdx.x, c.R);
  __syncthreads();
}

__global__ __launch_bounds__(64) void bpnp_backward_kernel(const float* __restrict__ x2, const float* __restrict__ P6,
                                                           const float* __restrict__ z3, long long z_bs,
                                                           const float* __restrict__ Kp, const float* __restrict__ gout,
                                                           int n, float* __restrict__ grad_x, double* __restrict__ gz_part,
                                                           double* __restrict__ gK_part) {
  const int b = blockIdx.x, lane = threadIdx.x;
  __shared__ CropIn C;
  load_crop(P6, Kp, b, C);
  const float* Z = z3 + (size_t)b * z_bs;
  const float* X = x2 + (size_t)b * n * 2;
  // pass 1: J_fy (6x6) and J_fK (6x9) summed over points. Every lane's 90 running sums live in
  // LDS (column = lane, conflict-free 8-byte rows) instead of registers: held in VGPRs beside the
  // point geometry they spilled 1860 B per lane to scratch. The summation order is unchanged (each
  // lane in point order, then the wave's butterfly), so the results are bit-identical.
  constexpr int kJ = 36 + 54;
  __shared__ double acc[kJ][64];
  __shared__ double red[kJ];
#pragma unroll 1
  for (int e = 0; e < kJ; ++e) acc[e][lane] = 0.0;
  for (int i = lane; i < n; i += 64) {
    const double z[3] = {(double)Z[3 * i], (double)Z[3 * i + 1], (double)Z[3 * i + 2]};
    const double x[2] = {(double)X[2 * i], (double)X[2 * i + 1]};
    PointGeo G;
    point_geo(C.R, C.K, C.t, z, G);
    const double r[2] = {x[0] * G.s - G.q[0], x[1] * G.s - G.q[1]};
    // columns y_l (not unrolled: the fifteen columns' operands at once did not fit the register
    // file; dq = Q_l is rebuilt from the LDS copy of R' / K, the same products as point_geo's)
#pragma unroll 1
    for (int l = 0; l < 6; ++l) {
      double dQ[6][3], df[6], ql[3];
      if (l < 3) {
        double v[3];
        matvec(C.R.dR[l], z, v);
        matvec(C.K, v, ql);
      } else {
#pragma unroll
        for (int e = 0; e < 3; ++e) ql[e] = C.K[e][l - 3];
      }
#pragma unroll
      for (int j = 0; j < 6; ++j) {
        if (j < 3 && l < 3) {
          double v[3];
          matvec(C.R.d2R[j][l], z, v);
          matvec(C.K, v, dQ[j]);
        } else {
          dQ[j][0] = dQ[j][1] = dQ[j][2] = 0.0;
        }
      }
      dir_deriv(G, x, r, ql, dQ, df);
#pragma unroll
      for (int j = 0; j < 6; ++j) acc[j * 6 + l][lane] += df[j];
    }
    // columns K[a][e2]: dq = e_a p_e2, dQ_j = e_a (dR_j z)_e2 (j < 3) or e_a delta(e2, j-3)
#pragma unroll
    for (int a = 0; a < 3; ++a)
#pragma unroll
      for (int e2 = 0; e2 < 3; ++e2) {
        double dq[3] = {0.0, 0.0, 0.0}, dQ[6][3], df[6];
        dq[a] = G.p[e2];
#pragma unroll
        for (int j = 0; j < 6; ++j) {
          dQ[j][0] = dQ[j][1] = dQ[j][2] = 0.0;
          dQ[j][a] = j < 3 ? G.Dz[j][e2] : (e2 == j - 3 ? 1.0 : 0.0);
        }
        dir_deriv(G, x, r, dq, dQ, df);
#pragma unroll
        for (int j = 0; j < 6; ++j) acc[36 + j * 9 + 3 * a + e2][lane] += df[j];
      }
  }
#pragma unroll 1
  for (int e = 0; e < kJ; ++e) {
    const double t = wave_sum(acc[e][lane]);
    if (lane == 0) red[e] = t;
  }
  __syncthreads();
  // v = -g J_fy^-1  <=>  J_fy^T v = -g
  double A[6][6], rhs[6], v[6];
#pragma unroll
  for (int j = 0; j < 6; ++j) {
    rhs[j] = -(double)gout[b * 6 + j];
#pragma unroll
    for (int l = 0; l < 6; ++l) A[j][l] = red[l * 6 + j];
  }
  if (!solve6(A, rhs, v)) {
#pragma unroll
    for (int j = 0; j < 6; ++j) v[j] = NAN;  // torch.inverse of a singular J_fy raises; NaN marks it
  }
  if (lane < 9) {
    double s = 0.0;
#pragma unroll
    for (int j = 0; j < 6; ++j) s += v[j] * red[36 + j * 9 + lane];
    gK_part[b * 9 + lane] = s;
  }
  // pass 2: grad_x (J_fx = c s) and the per-crop grad_z
  for (int i = lane; i < n; i += 64) {
    const double z[3] = {(double)Z[3 * i], (double)Z[3 * i + 1], (double)Z[3 * i + 2]};
    const double x[2] = {(double)X[2 * i], (double)X[2 * i + 1]};
    PointGeo G;
    point_geo(C.R, C.K, C.t, z, G);
    const double r[2] = {x[0] * G.s - G.q[0], x[1] * G.s - G.q[1]};
#pragma unroll
    for (int k = 0; k < 2; ++k) {
      double s = 0.0;
#pragma unroll
      for (int j = 0; j < 6; ++j) s += v[j] * (-2.0 * G.g[k][j] * G.s);
      grad_x[((size_t)b * n + i) * 2 + k] = (float)s;
    }
    double Jz[6][3];
    dz_cols(C.R, C.K, G, x, r, Jz);
#pragma unroll
    for (int m = 0; m < 3; ++m) {
      double s = 0.0;
#pragma unroll
      for (int j = 0; j < 6; ++j) s += v[j] * Jz[j][m];
      gz_part[((size_t)b * n + i) * 3 + m] = s;
    }
  }
}

// grad_z / grad_K: crop-ordered sums of the partials (shared points), or a cast (per-crop).
__global__ void bpnp_reduce_kernel(const double* __restrict__ gz_part, const double* __restrict__ gK_part, int B,
                                   int n, int per_crop, float* __restrict__ grad_z, float* __restrict__ grad_K) {
  const long long e = (long long)blockIdx.x * blockDim.x + threadIdx.x;
  const long long nz = per_crop ? (long long)B * n * 3 : (long long)n * 3;
  if (e < nz) {
    if (per_crop) {
      grad_z[e] = (float)gz_part[e];
    } else {
      double s = 0.0;
      for (int b = 0; b < B; ++b) s += gz_part[(size_t)b * n * 3 + e];
      grad_z[e] = (float)s;
    }
  } else if (e < nz + 9) {
    const int k = (int)(e - nz);
    double s = 0.0;
    for (int b = 0; b < B; ++b) s += gK_part[b * 9 + k];
    grad_K[k] = (float)s;
  }
}

// angle-axis of a rotation matrix (log map; theta near pi from the dominant column of R + I)
__device__ inline void rot_log(const float* Rf, double (&w)[3]) {
  double R[3][3];
#pragma unroll
  for (int a = 0; a < 3; ++a)
#pragma unroll
    for (int b = 0; b < 3; ++b) R[a][b] = (double)Rf[3 * a + b];
  const double c = fmin(1.0, fmax(-1.0, (R[0][0] + R[1][1] + R[2][2] - 1.0) * 0.5));
  const double th = acos(c), s = sin(th);
  const double v[3] = {R[2][1] - R[1][2], R[0][2] - R[2][0], R[1][0] - R[0][1]};
  if (s > 1e-6) {
    const double f = th / (2.0 * s);
#pragma unroll
    for (int a = 0; a < 3; ++a) w[a] = f * v[a];
  } else if (c > 0.0) {
#pragma unroll
    for (int a = 0; a < 3; ++a) w[a] = 0.5 * v[a];
  } else {
    int k = 0;
#pragma unroll
    for (int a = 1; a < 3; ++a)
      if (R[a][a] > R[k][k]) k = a;
    double nv[3];
    const double nk = sqrt(fmax(0.0, (R[k][k] + 1.0) * 0.5));
#pragma unroll
    for (int a = 0; a < 3; ++a) nv[a] = a == k ? nk : (R[a][k] + R[k][a]) / (4.0 * nk);
    const double sg = (nv[0] * v[0] + nv[1] * v[1] + nv[2] * v[2]) < 0.0 ? -1.0 : 1.0;
#pragma unroll
    for (int a = 0; a < 3; ++a) w[a] = sg * th * nv[a];
  }
}

// Levenberg-Marquardt on sum_i ||pi(z_i; y) - x_i||^2, one wave per crop.
__global__ __launch_bounds__(64) void bpnp_solve_kernel(const float* __restrict__ x2, const float* __restrict__ z3,
                                                        long long z_bs, const float* __restrict__ Kp,
                                                        const float* __restrict__ y0, const float* __restrict__ R0,
                                                        int n, int iters, float* __restrict__ y_out,
                                                        float* __restrict__ cost_out) {
  const int b = blockIdx.x, lane = threadIdx.x;
  const float* Z = z3 + (size_t)b * z_bs;
  const float* X = x2 + (size_t)b * n * 2;
  double K[3][3], y[6];
#pragma unroll
  for (int a = 0; a < 3; ++a)
#pragma unroll
    for (int e = 0; e < 3; ++e) K[a][e] = (double)Kp[3 * a + e];
#pragma unroll
  for (int j = 0; j < 6; ++j) y[j] = (double)y0[b * 6 + j];
  if (R0) {
    double w[3];
    rot_log(R0 + b * 9, w);
#pragma unroll
    for (int a = 0; a < 3; ++a) y[a] = w[a];
  }

  // cost (and optionally the normal equations) at pose yy
  auto evaluate = [&](const double (&yy)[6], bool normal, double (&H)[6][6], double (&gv)[6]) -> double {
    Rot R;
    rodrigues(yy[0], yy[1], yy[2], R);
    const double t[3] = {yy[3], yy[4], yy[5]};
    double cost = 0.0;
#pragma unroll
    for (int j = 0; j < 6; ++j) {
      gv[j] = 0.0;
#pragma unroll
      for (int l = 0; l < 6; ++l) H[j][l] = 0.0;
    }
    for (int i = lane; i < n; i += 64) {
      const double z[3] = {(double)Z[3 * i], (double)Z[3 * i + 1], (double)Z[3 * i + 2]};
      PointGeo G;
      point_geo(R, K, t, z, G);
#pragma unroll
      for (int k = 0; k < 2; ++k) {
        const double e = G.q[k] / G.s - (double)X[2 * i + k];
        cost += e * e;
        if (normal) {
#pragma unroll
          for (int j = 0; j < 6; ++j) {
            gv[j] += G.g[k][j] * e;
#pragma unroll
            for (int l = 0; l < 6; ++l) H[j][l] += G.g[k][j] * G.g[k][l];
          }
        }
      }
    }
    if (normal) {
#pragma unroll
      for (int j = 0; j < 6; ++j) {
        gv[j] = wave_sum(gv[j]);
#pragma unroll
        for (int l = 0; l < 6; ++l) H[j][l] = wave_sum(H[j][l]);
      }
    }
    return wave_sum(cost);
  };

  double H[6][6], gv[6], Ht[6][6], gt[6];
  double cost = evaluate(y, true, H, gv);
  double lam = 1e-3;
  for (int it = 0; it < iters; ++it) {
    bool improved = false;
    double step_max = 0.0;
    for (int tries = 0; tries < 30; ++tries) {
      double A[6][6], rhs[6], d[6];
#pragma unroll
      for (int j = 0; j < 6; ++j) {
        rhs[j] = -gv[j];
#pragma unroll
        for (int l = 0; l < 6; ++l) A[j][l] = H[j][l] + (j == l ? lam * H[j][j] : 0.0);
      }
      if (!solve6(A, rhs, d)) { lam *= 10.0; continue; }
      double yn[6];
      step_max = 0.0;
#pragma unroll
      for (int j = 0; j < 6; ++j) {
        yn[j] = y[j] + d[j];
        step_max = fmax(step_max, fabs(d[j]));
      }
      const double cn = evaluate(yn, false, Ht, gt);
      if (cn <= cost) {
#pragma unroll
        for (int j = 0; j < 6; ++j) y[j] = yn[j];
        cost = evaluate(y, true, H, gv);
        lam = fmax(lam * 0.1, 1e-12);
        improved = true;
        break;
      }
      lam *= 10.0;
    }
    double ymax = 1.0;
#pragma unroll
    for (int j = 0; j < 6; ++j) ymax = fmax(ymax, fabs(y[j]));
    if (!improved || step_max < 1e-13 * ymax) break;
  }
  if (lane < 6) y_out[b * 6 + lane] = (float)y[lane];
  if (cost_out && lane == 0) cost_out[b] = (float)cost;
}

}  // namespace

KRRN_API int krrn_bpnp_solve_f32(const float* pts2d, const float* pts3d, int z_per_crop, const float* K,
                                 const float* y_init, const float* R_init, int B, int n, int iters, float* y_out,
                                 float* cost_out, void* stream) {
  if (!pts2d || !pts3d || !K || !y_init || !y_out) return KRRN_EARG;
  if (B < 1 || n < 3 || iters < 0 || iters > 1000) return KRRN_ESHAPE;
  hipLaunchKernelGGL(bpnp_solve_kernel, dim3(B), dim3(64), 0, (hipStream_t)stream, pts2d, pts3d,
                     z_per_crop ? (long long)n * 3 : 0LL, K, y_init, R_init, n, iters, y_out, cost_out);
  return krrn_launch_status();
}

KRRN_API int krrn_bpnp_backward_f32(const float* pts2d, const float* P6, const float* pts3d, int z_per_crop,
                                    const float* K, const float* grad_out, int B, int n, float* grad_x,
                                    float* grad_z, float* grad_K, double* workspace, void* stream) {
  if (!pts2d || !P6 || !pts3d || !K || !grad_out || !grad_x || !grad_z || !grad_K || !workspace) return KRRN_EARG;
  if (B < 1 || n < 1) return KRRN_ESHAPE;
  hipStream_t s = (hipStream_t)stream;
  double* gz_part = workspace;
  double* gK_part = workspace + (size_t)B * n * 3;
  hipLaunchKernelGGL(bpnp_backward_kernel, dim3(B), dim3(64), 0, s, pts2d, P6, pts3d,
                     z_per_crop ? (long long)n * 3 : 0LL, K, grad_out, n, grad_x, gz_part, gK_part);
  const long long total = (z_per_crop ? (long long)B * n * 3 : (long long)n * 3) + 9;
  hipLaunchKernelGGL(bpnp_reduce_kernel, dim3((unsigned)((total + 255) / 256)), dim3(256), 0, s, gz_part, gK_part, B, n,
                     z_per_crop, grad_z, grad_K);
  return krrn_launch_status();
}
