/*
 * ORACLE — test infrastructure only (tests/, __graft_entry__.smoke(), bench.py cpu_baseline).
 * Never linked into or called by the product path.
 *
 * CPU restatement of the pose step of Trainer.get_pose (tools/trainer.py:383-438):
 *   cv2.solvePnPRansac(obj, img, K, None, flags=SOLVEPNP_EPNP, confidence=0.9999,
 *                      reprojectionError=1)
 * OpenCV is a third-party dependency absent from /root/reference (opencv-python,
 * version unpinned: the reference ships no requirements file). Its published algorithm is
 * restated here:
 *   - EPnP (Lepetit, Moreno-Noguer, Fua, IJCV 2009) as structured in OpenCV's epnp.cpp:
 *     PCA control points, barycentric alphas, M (2n x 12), null space of M^T M (4 smallest
 *     eigenvectors), L_6x10 / rho, beta approximations 1/2/3 each refined by 5 Gauss-Newton
 *     steps, R,t by Procrustes, the solution with the smallest mean reprojection error wins;
 *   - RANSAC as ptsetreg.cpp runs it: 5-point EPnP hypotheses in order while h < niters,
 *     inlier test ||proj - img||^2 <= thr^2, a count above max(best, modelPoints - 1) becomes
 *     the best and sets niters = RANSACUpdateNumIters(confidence, outlier ratio, 5, niters)
 *     (iterationsCount = H), then EPnP on all inliers of the best hypothesis.
 * Deliberate, documented differences (DESIGN.md "PnP"): the H hypothesis subsets are given
 * by the caller (so GPU and oracle score identical subsets) instead of cv::RNG; the 12x12
 * solve is the GPU kernel's parallel-ordered Jacobi (jacobi12_par); Procrustes uses the Kabsch
 * det-correction R = U diag(1,1,d) V^T.
 * PARITY UNPINNED against cv2 itself (not installable here); pinned by known-answer tests
 * (exact recovery of a known (R, t) on noiseless correspondences, tests/test_oracle_pnp.py).
 */
#include <math.h>
#include <string.h>

#define MAXP 4096

/* ---------------- small dense linear algebra (double) ---------------- */

/* cyclic Jacobi eigen-decomposition of symmetric n x n A (row-major, destroyed);
 * eigenvalues -> w, eigenvectors -> rows of V (V[i*n + :] is the i-th eigenvector),
 * sorted by descending eigenvalue. */
static void jacobi_eig(double* A, int n, double* w, double* V) {
  for (int i = 0; i < n; ++i)
    for (int j = 0; j < n; ++j) V[i * n + j] = (i == j) ? 1.0 : 0.0; /* columns = eigvecs during sweep */
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
  /* sort descending, transpose to row eigenvectors */
  int order[16];
  for (int i = 0; i < n; ++i) { order[i] = i; w[i] = A[i * n + i]; }
  for (int i = 0; i < n; ++i)
    for (int j = i + 1; j < n; ++j)
      if (w[order[j]] > w[order[i]]) { int tmp = order[i]; order[i] = order[j]; order[j] = tmp; }
  double Vt[144], ws[16];
  for (int i = 0; i < n; ++i) {
    ws[i] = w[order[i]];
    for (int k = 0; k < n; ++k) Vt[i * n + k] = V[k * n + order[i]];
  }
  memcpy(w, ws, sizeof(double) * n);
  memcpy(V, Vt, sizeof(double) * n * n);
}

/* The 12x12 solve of EPnP (M^T M) exactly as csrc/pnp.hip's eig12_group evaluates it:
 * parallel-ordered (round-robin) Jacobi, 11 steps of 6 disjoint rotations per sweep; per step every
 * pair's (c, s) from the pre-step matrix, then A <- A J, A <- J^T A, U <- U J. Convergence
 * off <= 1e-30 tot with per-row sums reduced by the kernel's 16-lane butterfly. Returns the
 * eigenvectors of the 4 smallest eigenvalues, ascending (ties: lower column first): v4[q][k]. */
static double bfly16(const double* x) {
  double v[16], t[16];
  for (int i = 0; i < 16; ++i) v[i] = x[i];
  for (int off = 8; off > 0; off >>= 1) {
    for (int i = 0; i < 16; ++i) t[i] = v[i] + v[i ^ off];
    for (int i = 0; i < 16; ++i) v[i] = t[i];
  }
  return v[0];
}

static int rr_partner(int k, int r) { return r == 11 ? k : (r == k ? 11 : (2 * k - r + 11) % 11); }

static void jacobi12_par(double* A, double v4[4][12]) {
  double U[144], A0[144];
  for (int i = 0; i < 144; ++i) U[i] = (i % 13 == 0) ? 1.0 : 0.0;
  for (int sweep = 0; sweep < 40; ++sweep) {
    double tr[16] = {0}, orr[16] = {0};
    for (int r = 0; r < 12; ++r)
      for (int j = 0; j < 12; ++j) {
        const double x2 = A[r * 12 + j] * A[r * 12 + j];
        tr[r] += x2;
        if (j != r) orr[r] += x2;
      }
    const double tot = bfly16(tr), off = bfly16(orr);
    if (off <= 1e-30 * tot || off < 1e-300) break;
    for (int k = 0; k < 11; ++k) {
      double c[12], sn[12];
      for (int r = 0; r < 12; ++r) {
        const int pr = rr_partner(k, r), lo = r < pr ? r : pr, hi = r < pr ? pr : r;
        const double apq = A[lo * 12 + hi], app = A[lo * 13], aqq = A[hi * 13];
        c[r] = 1.0;
        sn[r] = 0.0;
        if (!(fabs(apq) < 1e-300 || fabs(apq) < 1e-18 * sqrt(fabs(app * aqq)))) {
          const double theta = (aqq - app) / (2.0 * apq);
          const double tt = (theta >= 0 ? 1.0 : -1.0) / (fabs(theta) + sqrt(theta * theta + 1.0));
          c[r] = 1.0 / sqrt(tt * tt + 1.0);
          sn[r] = tt * c[r];
        }
      }
      int pp[6], qq[6];
      for (int i = 0; i < 6; ++i) {
        const int x = i == 0 ? k : (k + i) % 11, y = i == 0 ? 11 : (k - i + 11) % 11;
        pp[i] = x < y ? x : y;
        qq[i] = x < y ? y : x;
      }
      for (int r = 0; r < 12; ++r)
        for (int i = 0; i < 6; ++i) {
          const double cs = c[pp[i]], ss = sn[pp[i]];
          const double xp = A[r * 12 + pp[i]], xq = A[r * 12 + qq[i]];
          A[r * 12 + pp[i]] = cs * xp - ss * xq;
          A[r * 12 + qq[i]] = ss * xp + cs * xq;
        }
      memcpy(A0, A, sizeof A0);
      for (int r = 0; r < 12; ++r) {
        const int pr = rr_partner(k, r);
        for (int j = 0; j < 12; ++j) {
          const double y = A0[pr * 12 + j], x = A0[r * 12 + j];
          A[r * 12 + j] = r < pr ? c[r] * x - sn[r] * y : sn[r] * y + c[r] * x;
        }
      }
      for (int r = 0; r < 12; ++r)
        for (int i = 0; i < 6; ++i) {
          const double cs = c[pp[i]], ss = sn[pp[i]];
          const double xp = U[r * 12 + pp[i]], xq = U[r * 12 + qq[i]];
          U[r * 12 + pp[i]] = cs * xp - ss * xq;
          U[r * 12 + qq[i]] = ss * xp + cs * xq;
        }
    }
  }
  unsigned used = 0;
  for (int q = 0; q < 4; ++q) {
    int m = -1;
    double wm = 0.0;
    for (int j = 0; j < 12; ++j) {
      if (used & (1u << j)) continue;
      if (m < 0 || A[j * 13] < wm) { m = j; wm = A[j * 13]; }
    }
    used |= 1u << m;
    for (int k = 0; k < 12; ++k) v4[q][k] = U[k * 12 + m];
  }
}

/* cv::RANSACUpdateNumIters (ptsetreg.cpp) */
static int ransac_update_niters(double conf, double ep, int model_points, int max_iters) {
  conf = fmin(fmax(conf, 0.0), 1.0);
  ep = fmin(fmax(ep, 0.0), 1.0);
  double num = fmax(1.0 - conf, 2.2250738585072014e-308);
  double denom = 1.0 - pow(1.0 - ep, (double)model_points);
  if (denom < 2.2250738585072014e-308) return 0;
  num = log(num);
  denom = log(denom);
  return (denom >= 0 || -num >= max_iters * (-denom)) ? max_iters : (int)rint(num / denom);
}

/* least squares min ||A x - b|| for A m x n (m <= 6, n <= 5), as csrc/pnp.hip (lsq_rows) evaluates
 * it: the normal equations summed row by row in order, Cholesky when A has full column rank (the
 * usual case), else the pseudo-inverse from the eigen-decomposition of A^T A (OpenCV solves these
 * with CV_SVD; the two agree to rounding on full-rank systems). */
static void lsq_solve(const double* A, int m, int n, const double* b, double* x) {
  double AtA[25], w[5], V[25], Atb[5], C[25];
  for (int i = 0; i < n * n; ++i) AtA[i] = 0.0;
  for (int i = 0; i < n; ++i) Atb[i] = 0.0;
  for (int k = 0; k < m; ++k)
    for (int i = 0; i < n; ++i) {
      for (int j = 0; j < n; ++j) AtA[i * n + j] += A[k * n + i] * A[k * n + j];
      Atb[i] += A[k * n + i] * b[k];
    }
  double dmax = 0.0;
  for (int i = 0; i < n; ++i) dmax = fmax(dmax, AtA[i * n + i]);
  int spd = dmax > 0.0;
  for (int j = 0; j < n; ++j) {
    double d = AtA[j * n + j];
    for (int k = 0; k < j; ++k) d -= C[j * n + k] * C[j * n + k];
    spd = spd && d > 1e-14 * dmax;
    const double cjj = sqrt(fmax(d, 1e-300));
    C[j * n + j] = cjj;
    for (int i = j + 1; i < n; ++i) {
      double s = AtA[i * n + j];
      for (int k = 0; k < j; ++k) s -= C[i * n + k] * C[j * n + k];
      C[i * n + j] = s / cjj;
    }
  }
  if (spd) {
    double y[5];
    for (int i = 0; i < n; ++i) {
      double s = Atb[i];
      for (int k = 0; k < i; ++k) s -= C[i * n + k] * y[k];
      y[i] = s / C[i * n + i];
    }
    for (int i = n - 1; i >= 0; --i) {
      double s = y[i];
      for (int k = i + 1; k < n; ++k) s -= C[k * n + i] * x[k];
      x[i] = s / C[i * n + i];
    }
    return;
  }
  jacobi_eig(AtA, n, w, V);
  const double tol = (w[0] > 0 ? w[0] : 0.0) * 1e-24;
  for (int j = 0; j < n; ++j) x[j] = 0.0;
  for (int i = 0; i < n; ++i) {
    double proj = 0.0;
    for (int k = 0; k < n; ++k) proj += V[i * n + k] * Atb[k];
    proj = (w[i] > tol) ? proj / w[i] : 0.0;
    for (int k = 0; k < n; ++k) x[k] += proj * V[i * n + k];
  }
}

/* 3x3 pseudo-inverse (OpenCV inverts CC with CV_SVD): for planar point sets the third PCA
 * axis has zero length, CC is singular and the pseudo-inverse gives the 4th control point a
 * zero barycentric weight, which is how EPnP handles the planar case.
 * a^+ = sum_{w_i > tol} (1 / w_i) v_i v_i^T a^T with (w, v) = eig(a^T a). */
static void pinv3(const double* a, double* r) {
  double AtA[9], w[3], V[9];
  for (int i = 0; i < 3; ++i)
    for (int j = 0; j < 3; ++j) AtA[i * 3 + j] = a[0 * 3 + i] * a[0 * 3 + j] + a[1 * 3 + i] * a[1 * 3 + j] + a[2 * 3 + i] * a[2 * 3 + j];
  jacobi_eig(AtA, 3, w, V);
  const double tol = (w[0] > 0 ? w[0] : 0.0) * 1e-20;
  double P[9] = {0};
  for (int k = 0; k < 3; ++k) {
    const double iw = (w[k] > tol) ? 1.0 / w[k] : 0.0;
    for (int i = 0; i < 3; ++i)
      for (int j = 0; j < 3; ++j) P[i * 3 + j] += V[k * 3 + i] * V[k * 3 + j] * iw;
  }
  for (int i = 0; i < 3; ++i)
    for (int j = 0; j < 3; ++j) r[i * 3 + j] = P[i * 3 + 0] * a[j * 3 + 0] + P[i * 3 + 1] * a[j * 3 + 1] + P[i * 3 + 2] * a[j * 3 + 2];
}

/* ---------------- the kernel's summation orders ---------------- */

/* csrc/pnp.hip sums over points in one of two orders: SUM_SEQ, the points in order (a RANSAC
 * hypothesis' 5 points, replicated in its 16-lane group: HypSum), or SUM_WAVE, the refinement on
 * all inliers by one 64-lane wave (WaveSum): lane l sums points l, l + 64, ... in order, then the
 * lanes combine by the butterfly v += shfl_xor(v, off), off = 32, 16, ..., 1 (lane 0's value).
 * The rows of M^T M in SUM_WAVE: group g = lane / 16 sums points g, g + 4, ... in order, then
 * (G0 + G1) + (G2 + G3). */
enum { SUM_SEQ = 0, SUM_WAVE = 1 };
/* diagnostics of the last EPnP call (oracle_pnp_hypotheses_diag): the winning approximation
 * (1..3) and whether its Procrustes hit det(U V^T) < 0 (Kabsch: diag(1,1,-1); OpenCV: third row
 * negated) */
static int g_diag_approx, g_diag_detneg[4];
/* diagnostics only (tests/pnp_divergence.py), 0 everywhere else: swaps single ingredients of the
 * OpenCV-semantics EPnP for the kernel's -- bit 0: the 12 x 12 null-space basis from the kernel's
 * parallel-ordered Jacobi; bit 1: the kernel's Procrustes (U from the cross-product frame) instead of
 * the SVD one; bit 2: the beta and Gauss-Newton solves by the kernel's Cholesky normal equations;
 * bit 3: the kernel's Procrustes without the det rule (plain Kabsch, the kernel before round 5) */
static int g_cv_variant;
void oracle_set_cv_variant(int v) { g_cv_variant = v; }
static double contrib_buf[MAXP * 12];

/* out[k] = sum over points of contrib[p * nv + k], in the kernel's order */
static void reduce_points(int mode, int n, int nv, const double* contrib, double* out) {
  for (int k = 0; k < nv; ++k) {
    if (mode == SUM_SEQ) {
      double v = 0.0;
      for (int p = 0; p < n; ++p) v += contrib[p * nv + k];
      out[k] = v;
      continue;
    }
    double v[64], t[64];
    for (int l = 0; l < 64; ++l) v[l] = 0.0;
    for (int p = 0; p < n; ++p) v[p % 64] += contrib[p * nv + k];
    for (int off = 32; off > 0; off >>= 1) {
      for (int l = 0; l < 64; ++l) t[l] = v[l] + v[l ^ off];
      for (int l = 0; l < 64; ++l) v[l] = t[l];
    }
    out[k] = v[0];
  }
}

/* Procrustes on the 3x3 correlation H as csrc/pnp.hip kabsch evaluates it, with OpenCV's epnp.cpp
 * rule: R = U V^T, third row negated when det < 0 (for a rank-3 H: Kabsch's U diag(1,1,-1) V^T with
 * the third row negated); a rank-deficient H (coplanar points) keeps the proper Kabsch rotation. */
static void kabsch(const double* H, double* R) {
  /* SVD H = U S V^T through eig(H^T H) = V S^2 V^T, U = H V / S */
  double HtH[9], w[3], V[9];
  for (int i = 0; i < 3; ++i)
    for (int j = 0; j < 3; ++j) {
      double s = 0;
      for (int k = 0; k < 3; ++k) s += H[k * 3 + i] * H[k * 3 + j];
      HtH[i * 3 + j] = s;
    }
  jacobi_eig(HtH, 3, w, V); /* rows of V = right singular vectors */
  double U[9];
  for (int i = 0; i < 2; ++i) {
    double u[3];
    for (int r = 0; r < 3; ++r) u[r] = H[r * 3 + 0] * V[i * 3 + 0] + H[r * 3 + 1] * V[i * 3 + 1] + H[r * 3 + 2] * V[i * 3 + 2];
    double nr = sqrt(u[0] * u[0] + u[1] * u[1] + u[2] * u[2]);
    if (nr < 1e-300) nr = 1e-300;
    for (int r = 0; r < 3; ++r) U[i * 3 + r] = u[r] / nr; /* U stored by rows = left vectors */
  }
  /* re-orthogonalise u1 against u0 */
  {
    double d = U[0] * U[3] + U[1] * U[4] + U[2] * U[5];
    for (int r = 0; r < 3; ++r) U[3 + r] -= d * U[r];
    double nr = sqrt(U[3] * U[3] + U[4] * U[4] + U[5] * U[5]);
    if (nr < 1e-300) nr = 1e-300;
    for (int r = 0; r < 3; ++r) U[3 + r] /= nr;
  }
  U[6] = U[1] * U[5] - U[2] * U[4];
  U[7] = U[2] * U[3] - U[0] * U[5];
  U[8] = U[0] * U[4] - U[1] * U[3];
  /* third right vector consistent with det(V) = +1 */
  double v2[3] = {V[1] * V[5] - V[2] * V[4], V[2] * V[3] - V[0] * V[5], V[0] * V[4] - V[1] * V[3]};
  const double detH = H[0] * (H[4] * H[8] - H[5] * H[7]) - H[1] * (H[3] * H[8] - H[5] * H[6]) +
                      H[2] * (H[3] * H[7] - H[4] * H[6]);
  const int refl = (g_cv_variant & 8) ? 0 : (detH < 0.0 && w[2] > 1e-24 * w[0]);
  const double s2 = refl ? -1.0 : 1.0;
  /* R = sum_i u_i v_i^T (u2 = u0 x u1, v2 = v0 x v1: det(R) = +1, Kabsch), u2 negated for a reflection */
  for (int r = 0; r < 3; ++r)
    for (int c = 0; c < 3; ++c)
      R[r * 3 + c] = U[0 * 3 + r] * V[0 * 3 + c] + U[1 * 3 + r] * V[1 * 3 + c] + (s2 * U[2 * 3 + r]) * v2[c];
  if (refl) {
    R[6] = -R[6]; R[7] = -R[7]; R[8] = -R[8];
  }
}

/* ---------------- EPnP ---------------- */

typedef struct {
  double fu, fv, uc, vc;
} Cam;

/* control points (PCA of the world points) and the inverse of their frame; cw = the centroid */
static void ctrl_points(int mode, const double* pw, int n, double cws[4][3], double ccinv[9], double cw[3]) {
  for (int p = 0; p < n; ++p)
    for (int j = 0; j < 3; ++j) contrib_buf[3 * p + j] = pw[3 * p + j];
  reduce_points(mode, n, 3, contrib_buf, cw);
  for (int j = 0; j < 3; ++j) cw[j] /= n;
  double C6[6];
  for (int p = 0; p < n; ++p) {
    const double d0 = pw[3 * p] - cw[0], d1 = pw[3 * p + 1] - cw[1], d2 = pw[3 * p + 2] - cw[2];
    double* c = contrib_buf + 6 * p;
    c[0] = d0 * d0; c[1] = d0 * d1; c[2] = d0 * d2; c[3] = d1 * d1; c[4] = d1 * d2; c[5] = d2 * d2;
  }
  reduce_points(mode, n, 6, contrib_buf, C6);
  double C[9] = {C6[0], C6[1], C6[2], C6[1], C6[3], C6[4], C6[2], C6[4], C6[5]};
  double w[3], V[9];
  jacobi_eig(C, 3, w, V);
  for (int j = 0; j < 3; ++j) cws[0][j] = cw[j];
  for (int i = 0; i < 3; ++i) {
    const double k = sqrt((w[i] > 0 ? w[i] : 0.0) / n);
    for (int j = 0; j < 3; ++j) cws[i + 1][j] = cw[j] + k * V[i * 3 + j];
  }
  double CC[9];
  for (int i = 0; i < 3; ++i)
    for (int j = 1; j < 4; ++j) CC[i * 3 + j - 1] = cws[j][i] - cws[0][i];
  pinv3(CC, ccinv);
}

static void alphas_of(const double* p, double cws[4][3], const double* ci, double a[4]) {
  const double d0 = p[0] - cws[0][0], d1 = p[1] - cws[0][1], d2 = p[2] - cws[0][2];
  a[1] = ci[0] * d0 + ci[1] * d1 + ci[2] * d2;
  a[2] = ci[3] * d0 + ci[4] * d1 + ci[5] * d2;
  a[3] = ci[6] * d0 + ci[7] * d1 + ci[8] * d2;
  a[0] = 1.0 - a[1] - a[2] - a[3];
}

static double dot3(const double* a, const double* b) { return a[0] * b[0] + a[1] * b[1] + a[2] * b[2]; }

static void gauss_newton(const double* L, const double* rho, double betas[4]) {
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

/* R,t from betas (Procrustes on the camera-frame points, Kabsch); returns mean reprojection error */
static double r_and_t(int mode, const double* ut, const double betas[4], const double* pw, const double* uv, int n,
                      double cws[4][3], const double* ci, const double* cw, Cam cam, double* R, double* t) {
  double ccs[4][3] = {{0}};
  for (int i = 0; i < 4; ++i) {
    const double* v = ut + 12 * (11 - i);
    for (int j = 0; j < 4; ++j)
      for (int k = 0; k < 3; ++k) ccs[j][k] += betas[i] * v[3 * j + k];
  }
  /* solve_for_sign: the first point must lie in front of the camera */
  double a0[4];
  alphas_of(pw, cws, ci, a0);
  const double z0 = a0[0] * ccs[0][2] + a0[1] * ccs[1][2] + a0[2] * ccs[2][2] + a0[3] * ccs[3][2];
  const double sg = z0 < 0.0 ? -1.0 : 1.0;
  double cc[3], H[9], err;
  for (int p = 0; p < n; ++p) {
    double a[4];
    alphas_of(pw + 3 * p, cws, ci, a);
    for (int k = 0; k < 3; ++k)
      contrib_buf[3 * p + k] = sg * (a[0] * ccs[0][k] + a[1] * ccs[1][k] + a[2] * ccs[2][k] + a[3] * ccs[3][k]);
  }
  reduce_points(mode, n, 3, contrib_buf, cc);
  for (int k = 0; k < 3; ++k) cc[k] /= n;
  /* H = sum (pc - cc)(pw - cw)^T   (ABt in EPnP) */
  for (int p = 0; p < n; ++p) {
    double a[4], pc[3];
    alphas_of(pw + 3 * p, cws, ci, a);
    for (int k = 0; k < 3; ++k) pc[k] = sg * (a[0] * ccs[0][k] + a[1] * ccs[1][k] + a[2] * ccs[2][k] + a[3] * ccs[3][k]);
    for (int r = 0; r < 3; ++r)
      for (int c = 0; c < 3; ++c) contrib_buf[9 * p + 3 * r + c] = (pc[r] - cc[r]) * (pw[3 * p + c] - cw[c]);
  }
  reduce_points(mode, n, 9, contrib_buf, H);
  g_diag_detneg[0] = (H[0] * (H[4] * H[8] - H[5] * H[7]) - H[1] * (H[3] * H[8] - H[5] * H[6]) +
                      H[2] * (H[3] * H[7] - H[4] * H[6])) < 0;
  kabsch(H, R);
  for (int r = 0; r < 3; ++r) t[r] = cc[r] - (R[r * 3 + 0] * cw[0] + R[r * 3 + 1] * cw[1] + R[r * 3 + 2] * cw[2]);
  for (int p = 0; p < n; ++p) {
    const double* X = pw + 3 * p;
    const double Xc = dot3(R, X) + t[0], Yc = dot3(R + 3, X) + t[1], Zc = dot3(R + 6, X) + t[2];
    const double iz = 1.0 / Zc;
    const double ue = cam.uc + cam.fu * Xc * iz, ve = cam.vc + cam.fv * Yc * iz;
    const double du = uv[2 * p] - ue, dv = uv[2 * p + 1] - ve;
    contrib_buf[p] = sqrt(du * du + dv * dv);
  }
  reduce_points(mode, n, 1, contrib_buf, &err);
  return err / n;
}

/* EPnP on n >= 4 correspondences (pw: n x 3 world, uv: n x 2 pixels), sums in the kernel's `mode`. */
static double epnp_mode(int mode, const double* pw, const double* uv, int n, Cam cam, double* R, double* t) {
  double cws[4][3], ci[9], cw[3];
  ctrl_points(mode, pw, n, cws, ci, cw);
  double MtM[144] = {0};
  double G[4][144];
  if (mode == SUM_WAVE) memset(G, 0, sizeof G);
  for (int p = 0; p < n; ++p) {
    double a[4];
    alphas_of(pw + 3 * p, cws, ci, a);
    double r1[12], r2[12];
    for (int j = 0; j < 4; ++j) {
      r1[3 * j] = a[j] * cam.fu;
      r1[3 * j + 1] = 0.0;
      r1[3 * j + 2] = a[j] * (cam.uc - uv[2 * p]);
      r2[3 * j] = 0.0;
      r2[3 * j + 1] = a[j] * cam.fv;
      r2[3 * j + 2] = a[j] * (cam.vc - uv[2 * p + 1]);
    }
    double* M = mode == SUM_WAVE ? G[p % 4] : MtM;
    for (int i = 0; i < 12; ++i)
      for (int j = 0; j < 12; ++j) M[i * 12 + j] += r1[i] * r1[j] + r2[i] * r2[j];
  }
  if (mode == SUM_WAVE)
    for (int e = 0; e < 144; ++e) MtM[e] = (G[0][e] + G[1][e]) + (G[2][e] + G[3][e]);
  double v4[4][12], ut[144];
  jacobi12_par(MtM, v4);
  for (int q = 0; q < 4; ++q)
    for (int k = 0; k < 12; ++k) ut[(11 - q) * 12 + k] = v4[q][k];  /* rows 11, 10, 9, 8: ascending */
  /* L_6x10 and rho */
  double L[60], rho[6];
  {
    const double* v[4] = {ut + 12 * 11, ut + 12 * 10, ut + 12 * 9, ut + 12 * 8};
    double dv[4][6][3];
    for (int i = 0; i < 4; ++i) {
      int a = 0, b = 1;
      for (int j = 0; j < 6; ++j) {
        for (int k = 0; k < 3; ++k) dv[i][j][k] = v[i][3 * a + k] - v[i][3 * b + k];
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
  double Rs[4][9], ts[4][3], errs[4], betas[4];
  /* approx 1: B11 B12 B13 B14 from columns 0 1 3 6 */
  {
    double A[24], x[4];
    const int cols[4] = {0, 1, 3, 6};
    for (int i = 0; i < 6; ++i)
      for (int j = 0; j < 4; ++j) A[4 * i + j] = L[10 * i + cols[j]];
    lsq_solve(A, 6, 4, rho, x);
    if (x[0] < 0) {
      betas[0] = sqrt(-x[0]);
      betas[1] = -x[1] / betas[0];
      betas[2] = -x[2] / betas[0];
      betas[3] = -x[3] / betas[0];
    } else {
      betas[0] = sqrt(x[0]);
      betas[1] = betas[0] > 0 ? x[1] / betas[0] : 0.0;
      betas[2] = betas[0] > 0 ? x[2] / betas[0] : 0.0;
      betas[3] = betas[0] > 0 ? x[3] / betas[0] : 0.0;
    }
    gauss_newton(L, rho, betas);
    errs[1] = r_and_t(mode, ut, betas, pw, uv, n, cws, ci, cw, cam, Rs[1], ts[1]);
    g_diag_detneg[1] = g_diag_detneg[0];
  }
  /* approx 2: B11 B12 B22 from columns 0 1 2 */
  {
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
    betas[2] = 0.0;
    betas[3] = 0.0;
    gauss_newton(L, rho, betas);
    errs[2] = r_and_t(mode, ut, betas, pw, uv, n, cws, ci, cw, cam, Rs[2], ts[2]);
    g_diag_detneg[2] = g_diag_detneg[0];
  }
  /* approx 3: B11 B12 B22 B13 B23 from columns 0..4 */
  {
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
    betas[3] = 0.0;
    gauss_newton(L, rho, betas);
    errs[3] = r_and_t(mode, ut, betas, pw, uv, n, cws, ci, cw, cam, Rs[3], ts[3]);
    g_diag_detneg[3] = g_diag_detneg[0];
  }
  int N = 1;
  if (errs[2] < errs[1]) N = 2;
  if (errs[3] < errs[N]) N = 3;
  g_diag_approx = N;
  memcpy(R, Rs[N], sizeof(double) * 9);
  memcpy(t, ts[N], sizeof(double) * 3);
  return errs[N];
}

static double epnp(const double* pw, const double* uv, int n, Cam cam, double* R, double* t) {
  return epnp_mode(SUM_SEQ, pw, uv, n, cam, R, t);
}

/* ---------------- public oracle entry points ---------------- */

/* EPnP on the given points (double). Returns mean reprojection error. */
double oracle_epnp(const double* pw, const double* uv, int n, const double* K4, double* R, double* t) {
  Cam cam = {K4[0], K4[1], K4[2], K4[3]};
  return epnp(pw, uv, n, cam, R, t);
}

/* Every hypothesis of oracle_pnp_ransac (diagnostics): f32-cast pose and inlier count. */
void oracle_pnp_hypotheses(const float* obj, const float* img, int P, const float* K4, const int* subsets, int H,
                           float thr, float* R_out, float* t_out, int* cnt_out) {
  Cam cam = {K4[0], K4[1], K4[2], K4[3]};
  const float thr2 = thr * thr;
  for (int h = 0; h < H; ++h) {
    double spw[15], suv[10], R[9], t[3];
    for (int i = 0; i < 5; ++i) {
      const int id = subsets[5 * h + i];
      for (int k = 0; k < 3; ++k) spw[3 * i + k] = obj[3 * id + k];
      for (int k = 0; k < 2; ++k) suv[2 * i + k] = img[2 * id + k];
    }
    epnp(spw, suv, 5, cam, R, t);
    int cnt = 0;
    for (int p = 0; p < P; ++p) {
      const float X = obj[3 * p], Y = obj[3 * p + 1], Z = obj[3 * p + 2];
      const float xc = (float)R[0] * X + (float)R[1] * Y + (float)R[2] * Z + (float)t[0];
      const float yc = (float)R[3] * X + (float)R[4] * Y + (float)R[5] * Z + (float)t[1];
      const float zc = (float)R[6] * X + (float)R[7] * Y + (float)R[8] * Z + (float)t[2];
      const float iz = 1.0f / zc;
      const float du = img[2 * p] - ((float)cam.fu * xc * iz + (float)cam.uc);
      const float dv = img[2 * p + 1] - ((float)cam.fv * yc * iz + (float)cam.vc);
      if (du * du + dv * dv <= thr2) ++cnt;
    }
    for (int i = 0; i < 9; ++i) R_out[9 * h + i] = (float)R[i];
    for (int i = 0; i < 3; ++i) t_out[3 * h + i] = (float)t[i];
    cnt_out[h] = cnt;
  }
}

/*
 * RANSAC with caller-given hypothesis subsets.
 * obj: P x 3 (f32, metres, model frame), img: P x 2 (f32, pixels), K4 = fx, fy, cx, cy.
 * subsets: H x 5 indices into [0, P). thr: reprojection threshold in pixels.
 * Outputs R (9, f32 row-major), t (3), inlier mask (P bytes) of the final pose's source
 * hypothesis, and returns the inlier count of the best hypothesis (0 = RANSAC failed).
 */
int oracle_pnp_ransac(const float* obj, const float* img, int P, const float* K4, const int* subsets, int H,
                      float thr, double conf, float* R_out, float* t_out, unsigned char* inlier_mask, int* best_h) {
  static double pw[3 * MAXP], uv[2 * MAXP];
  Cam cam = {K4[0], K4[1], K4[2], K4[3]};
  if (P > MAXP) P = MAXP;
  int best = -1, best_cnt = 0;
  double bestR[9] = {1, 0, 0, 0, 1, 0, 0, 0, 1}, bestt[3] = {0, 0, 0};
  const float thr2 = thr * thr;
  int niters = H;
  for (int h = 0; h < niters; ++h) {
    double spw[15], suv[10], R[9], t[3];
    for (int i = 0; i < 5; ++i) {
      const int id = subsets[5 * h + i];
      for (int k = 0; k < 3; ++k) spw[3 * i + k] = obj[3 * id + k];
      for (int k = 0; k < 2; ++k) suv[2 * i + k] = img[2 * id + k];
    }
    epnp(spw, suv, 5, cam, R, t);
    int cnt = 0;
    for (int p = 0; p < P; ++p) {
      const float X = obj[3 * p], Y = obj[3 * p + 1], Z = obj[3 * p + 2];
      const float xc = (float)R[0] * X + (float)R[1] * Y + (float)R[2] * Z + (float)t[0];
      const float yc = (float)R[3] * X + (float)R[4] * Y + (float)R[5] * Z + (float)t[1];
      const float zc = (float)R[6] * X + (float)R[7] * Y + (float)R[8] * Z + (float)t[2];
      const float iz = 1.0f / zc;
      const float du = img[2 * p] - ((float)cam.fu * xc * iz + (float)cam.uc);
      const float dv = img[2 * p + 1] - ((float)cam.fv * yc * iz + (float)cam.vc);
      if (du * du + dv * dv <= thr2) ++cnt;
    }
    /* ptsetreg.cpp: goodCount > max(maxGoodCount, modelPoints - 1), then the adaptive count */
    if (cnt > (best_cnt > 4 ? best_cnt : 4)) {
      best_cnt = cnt;
      best = h;
      memcpy(bestR, R, sizeof bestR);
      memcpy(bestt, t, sizeof bestt);
      niters = ransac_update_niters(conf, (double)(P - cnt) / P, 5, niters);
    }
  }
  if (best_h) *best_h = best;
  double R[9], t[3];
  memcpy(R, bestR, sizeof R);
  memcpy(t, bestt, sizeof t);
  int n = 0;
  for (int p = 0; p < P; ++p) {
    int in = 0;
    if (best >= 0) {
      const float X = obj[3 * p], Y = obj[3 * p + 1], Z = obj[3 * p + 2];
      const float xc = (float)bestR[0] * X + (float)bestR[1] * Y + (float)bestR[2] * Z + (float)bestt[0];
      const float yc = (float)bestR[3] * X + (float)bestR[4] * Y + (float)bestR[5] * Z + (float)bestt[1];
      const float zc = (float)bestR[6] * X + (float)bestR[7] * Y + (float)bestR[8] * Z + (float)bestt[2];
      const float iz = 1.0f / zc;
      const float du = img[2 * p] - ((float)cam.fu * xc * iz + (float)cam.uc);
      const float dv = img[2 * p + 1] - ((float)cam.fv * yc * iz + (float)cam.vc);
      in = du * du + dv * dv <= thr2;
    }
    if (inlier_mask) inlier_mask[p] = (unsigned char)in;
    if (in) {
      for (int k = 0; k < 3; ++k) pw[3 * n + k] = obj[3 * p + k];
      for (int k = 0; k < 2; ++k) uv[2 * n + k] = img[2 * p + k];
      ++n;
    }
  }
  if (best >= 0 && n >= 5) epnp_mode(SUM_WAVE, pw, uv, n, cam, R, t);
  for (int i = 0; i < 9; ++i) R_out[i] = (float)R[i];
  for (int i = 0; i < 3; ++i) t_out[i] = (float)t[i];
  return best >= 0 ? best_cnt : 0;
}

/* ---------------- OpenCV-semantics EPnP (independent of the kernel's numerics) ----------------
 * The restatement above mirrors csrc/pnp.hip operation for operation (Cholesky normal equations,
 * the parallel-ordered 12x12 Jacobi, the kernel's summation orders), so it pins the kernel's
 * arithmetic, not cv2's. This second path follows OpenCV's epnp.cpp structure instead, with its
 * own numerics, and is compared with the kernel at loose tolerances (tests/test_gpu_pnp.py):
 *   - M^T M eigen-decomposition by cyclic Jacobi on the full 12 x 12 (cvSVD of MtM);
 *   - the beta approximations by the SVD pseudo-inverse (cvSolve(..., CV_SVD));
 *   - Gauss-Newton steps by Householder QR (epnp.cpp qr_solve);
 *   - R from the SVD of ABt as U V^T with OpenCV's det < 0 fix (negate the third row), not Kabsch;
 *   - every point sum sequential. */

/* min ||A x - b|| through the pseudo-inverse of A^T A's eigen-decomposition (singular values below
 * 1e-12 of the largest dropped, as an SVD solve does) */
static void lsq_svd(const double* A, int m, int n, const double* b, double* x) {
  double AtA[25], Atb[5], w[5], V[25];
  for (int i = 0; i < n; ++i) {
    Atb[i] = 0.0;
    for (int j = 0; j < n; ++j) AtA[i * n + j] = 0.0;
  }
  for (int k = 0; k < m; ++k)
    for (int i = 0; i < n; ++i) {
      for (int j = 0; j < n; ++j) AtA[i * n + j] += A[k * n + i] * A[k * n + j];
      Atb[i] += A[k * n + i] * b[k];
    }
  jacobi_eig(AtA, n, w, V);
  const double tol = (w[0] > 0 ? w[0] : 0.0) * 1e-24; /* (1e-12 sigma_max)^2 */
  for (int j = 0; j < n; ++j) x[j] = 0.0;
  for (int i = 0; i < n; ++i) {
    if (!(w[i] > tol)) continue;
    double proj = 0.0;
    for (int k = 0; k < n; ++k) proj += V[i * n + k] * Atb[k];
    proj /= w[i];
    for (int k = 0; k < n; ++k) x[k] += proj * V[i * n + k];
  }
}

/* Householder QR least squares of the 6 x 4 Gauss-Newton system (epnp.cpp qr_solve) */
static void qr_solve6x4(double* A, double* b, double* x) {
  const int nr = 6, nc = 4;
  double A1[4], A2[4];
  for (int k = 0; k < nc; ++k) {
    double eta = 0.0;
    for (int i = k; i < nr; ++i) eta = fmax(eta, fabs(A[i * nc + k]));
    if (eta == 0.0) { A1[k] = A2[k] = 0.0; continue; }
    double sum = 0.0;
    for (int i = k; i < nr; ++i) {
      A[i * nc + k] /= eta;
      sum += A[i * nc + k] * A[i * nc + k];
    }
    double sigma = sqrt(sum);
    if (A[k * nc + k] < 0) sigma = -sigma;
    A[k * nc + k] += sigma;
    A1[k] = sigma * A[k * nc + k];
    A2[k] = -eta * sigma;
    for (int j = k + 1; j < nc; ++j) {
      double s = 0.0;
      for (int i = k; i < nr; ++i) s += A[i * nc + k] * A[i * nc + j];
      const double tau = s / A1[k];
      for (int i = k; i < nr; ++i) A[i * nc + j] -= tau * A[i * nc + k];
    }
  }
  for (int j = 0; j < nc; ++j) {
    if (A1[j] == 0.0) continue;
    double tau = 0.0;
    for (int i = j; i < nr; ++i) tau += A[i * nc + j] * b[i];
    tau /= A1[j];
    for (int i = j; i < nr; ++i) b[i] -= tau * A[i * nc + j];
  }
  for (int i = nc - 1; i >= 0; --i) {
    double s = b[i];
    for (int j = i + 1; j < nc; ++j) s -= A[i * nc + j] * x[j];
    x[i] = A2[i] != 0.0 ? s / A2[i] : 0.0;
  }
}

static void gauss_newton_cv(const double* L, const double* rho, double betas[4]) {
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
    if (g_cv_variant & 4) lsq_solve(A, 6, 4, b, x);
    else qr_solve6x4(A, b, x);
    for (int k = 0; k < 4; ++k) betas[k] += x[k];
  }
}

/* epnp.cpp estimate_R_and_t: R = U V^T of ABt's SVD, third row negated when det(R) < 0 */
static double r_and_t_cv(const double* ut, const double betas[4], const double* pw, const double* uv, int n,
                         double cws[4][3], const double* ci, const double* cw, Cam cam, double* R, double* t) {
  double ccs[4][3] = {{0}};
  for (int i = 0; i < 4; ++i) {
    const double* v = ut + 12 * (11 - i);
    for (int j = 0; j < 4; ++j)
      for (int k = 0; k < 3; ++k) ccs[j][k] += betas[i] * v[3 * j + k];
  }
  double a0[4];
  alphas_of(pw, cws, ci, a0);
  const double z0 = a0[0] * ccs[0][2] + a0[1] * ccs[1][2] + a0[2] * ccs[2][2] + a0[3] * ccs[3][2];
  const double sg = z0 < 0.0 ? -1.0 : 1.0;
  double cc[3] = {0, 0, 0}, ABt[9] = {0};
  for (int p = 0; p < n; ++p) {
    double a[4];
    alphas_of(pw + 3 * p, cws, ci, a);
    for (int k = 0; k < 3; ++k) cc[k] += sg * (a[0] * ccs[0][k] + a[1] * ccs[1][k] + a[2] * ccs[2][k] + a[3] * ccs[3][k]);
  }
  for (int k = 0; k < 3; ++k) cc[k] /= n;
  for (int p = 0; p < n; ++p) {
    double a[4], pc[3];
    alphas_of(pw + 3 * p, cws, ci, a);
    for (int k = 0; k < 3; ++k) pc[k] = sg * (a[0] * ccs[0][k] + a[1] * ccs[1][k] + a[2] * ccs[2][k] + a[3] * ccs[3][k]);
    for (int r = 0; r < 3; ++r)
      for (int c = 0; c < 3; ++c) ABt[3 * r + c] += (pc[r] - cc[r]) * (pw[3 * p + c] - cw[c]);
  }
  /* SVD ABt = U S V^T: V from eig(ABt^T ABt), U = ABt V / S (the third left vector completes U) */
  double AtA[9], w[3], V[9], U[9];
  for (int i = 0; i < 3; ++i)
    for (int j = 0; j < 3; ++j) AtA[3 * i + j] = ABt[i] * ABt[j] + ABt[3 + i] * ABt[3 + j] + ABt[6 + i] * ABt[6 + j];
  jacobi_eig(AtA, 3, w, V);
  if (!(w[2] > 1e-24 * w[0]) || (g_cv_variant & 2)) {
    /* rank-deficient H (coplanar points): the third singular pair and so the sign of det(U V^T) are
     * the SVD's arbitrary choice; the proper rotation (Kabsch) is taken, as csrc/pnp.hip does */
    g_diag_detneg[0] = 0;
    kabsch(ABt, R);
  } else {
    for (int i = 0; i < 3; ++i) {
      double u[3];
      for (int r = 0; r < 3; ++r) u[r] = ABt[3 * r] * V[3 * i] + ABt[3 * r + 1] * V[3 * i + 1] + ABt[3 * r + 2] * V[3 * i + 2];
      double nr = sqrt(u[0] * u[0] + u[1] * u[1] + u[2] * u[2]);
      if (nr < 1e-300) nr = 1e-300;
      for (int r = 0; r < 3; ++r) U[3 * i + r] = u[r] / nr;
    }
    for (int r = 0; r < 3; ++r)
      for (int c = 0; c < 3; ++c) R[3 * r + c] = U[r] * V[c] + U[3 + r] * V[3 + c] + U[6 + r] * V[6 + c];
    const double det = R[0] * (R[4] * R[8] - R[5] * R[7]) - R[1] * (R[3] * R[8] - R[5] * R[6]) +
                       R[2] * (R[3] * R[7] - R[4] * R[6]);
    g_diag_detneg[0] = det < 0;
    if (det < 0) {
      R[6] = -R[6]; R[7] = -R[7]; R[8] = -R[8];
    }
  }
  for (int r = 0; r < 3; ++r) t[r] = cc[r] - (R[3 * r] * cw[0] + R[3 * r + 1] * cw[1] + R[3 * r + 2] * cw[2]);
  double err = 0.0;
  for (int p = 0; p < n; ++p) {
    const double* X = pw + 3 * p;
    const double Xc = dot3(R, X) + t[0], Yc = dot3(R + 3, X) + t[1], Zc = dot3(R + 6, X) + t[2];
    const double ue = cam.uc + cam.fu * Xc / Zc, ve = cam.vc + cam.fv * Yc / Zc;
    const double du = uv[2 * p] - ue, dv = uv[2 * p + 1] - ve;
    err += sqrt(du * du + dv * dv);
  }
  return err / n;
}

static double epnp_cv(const double* pw, const double* uv, int n, Cam cam, double* R, double* t) {
  double cws[4][3], ci[9], cw[3];
  ctrl_points(SUM_SEQ, pw, n, cws, ci, cw);
  double MtM[144] = {0};
  for (int p = 0; p < n; ++p) {
    double a[4], r1[12], r2[12];
    alphas_of(pw + 3 * p, cws, ci, a);
    for (int j = 0; j < 4; ++j) {
      r1[3 * j] = a[j] * cam.fu;
      r1[3 * j + 1] = 0.0;
      r1[3 * j + 2] = a[j] * (cam.uc - uv[2 * p]);
      r2[3 * j] = 0.0;
      r2[3 * j + 1] = a[j] * cam.fv;
      r2[3 * j + 2] = a[j] * (cam.vc - uv[2 * p + 1]);
    }
    for (int i = 0; i < 12; ++i)
      for (int j = 0; j < 12; ++j) MtM[i * 12 + j] += r1[i] * r1[j] + r2[i] * r2[j];
  }
  double w[12], ut[144];
  if (g_cv_variant & 1) {
    double v4[4][12];
    jacobi12_par(MtM, v4);
    for (int q = 0; q < 4; ++q)
      for (int k = 0; k < 12; ++k) ut[(11 - q) * 12 + k] = v4[q][k];
  } else {
    jacobi_eig(MtM, 12, w, ut); /* rows of ut: eigenvectors, descending: rows 11..8 = the 4 smallest */
  }
  double L[60], rho[6];
  {
    const double* v[4] = {ut + 12 * 11, ut + 12 * 10, ut + 12 * 9, ut + 12 * 8};
    double dv[4][6][3];
    for (int i = 0; i < 4; ++i) {
      int a = 0, b = 1;
      for (int j = 0; j < 6; ++j) {
        for (int k = 0; k < 3; ++k) dv[i][j][k] = v[i][3 * a + k] - v[i][3 * b + k];
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
  double Rs[4][9], ts[4][3], errs[4], betas[4];
  for (int approx = 1; approx <= 3; ++approx) {
    const int nb = approx == 1 ? 4 : (approx == 2 ? 3 : 5);
    static const int cols1[4] = {0, 1, 3, 6};
    double A[30], x[5];
    for (int i = 0; i < 6; ++i)
      for (int j = 0; j < nb; ++j) A[nb * i + j] = L[10 * i + (approx == 1 ? cols1[j] : j)];
    if (g_cv_variant & 4) lsq_solve(A, 6, nb, rho, x);
    else lsq_svd(A, 6, nb, rho, x);
    if (approx == 1) {
      if (x[0] < 0) {
        betas[0] = sqrt(-x[0]);
        for (int k = 1; k < 4; ++k) betas[k] = -x[k] / betas[0];
      } else {
        betas[0] = sqrt(x[0]);
        for (int k = 1; k < 4; ++k) betas[k] = betas[0] > 0 ? x[k] / betas[0] : 0.0;
      }
    } else {
      if (x[0] < 0) {
        betas[0] = sqrt(-x[0]);
        betas[1] = (x[2] < 0) ? sqrt(-x[2]) : 0.0;
      } else {
        betas[0] = sqrt(x[0]);
        betas[1] = (x[2] > 0) ? sqrt(x[2]) : 0.0;
      }
      if (x[1] < 0) betas[0] = -betas[0];
      betas[2] = approx == 3 && betas[0] != 0.0 ? x[3] / betas[0] : 0.0;
      betas[3] = 0.0;
    }
    gauss_newton_cv(L, rho, betas);
    errs[approx] = r_and_t_cv(ut, betas, pw, uv, n, cws, ci, cw, cam, Rs[approx], ts[approx]);
    g_diag_detneg[approx] = g_diag_detneg[0];
  }
  int N = 1;
  if (errs[2] < errs[1]) N = 2;
  if (errs[3] < errs[N]) N = 3;
  g_diag_approx = N;
  memcpy(R, Rs[N], sizeof(double) * 9);
  memcpy(t, ts[N], sizeof(double) * 3);
  return errs[N];
}

/* oracle_pnp_ransac with the OpenCV-semantics EPnP (same hypothesis subsets, inlier test and
 * RANSAC loop; the refinement is EPnP on the best hypothesis' inliers, as solvePnPRansac does). */
int oracle_pnp_ransac_cv(const float* obj, const float* img, int P, const float* K4, const int* subsets, int H,
                         float thr, double conf, float* R_out, float* t_out, int* best_h) {
  static double pw[3 * MAXP], uv[2 * MAXP];
  Cam cam = {K4[0], K4[1], K4[2], K4[3]};
  if (P > MAXP) P = MAXP;
  int best = -1, best_cnt = 0, niters = H;
  float bR[9] = {1, 0, 0, 0, 1, 0, 0, 0, 1}, bt[3] = {0, 0, 0};
  const float thr2 = thr * thr;
  for (int h = 0; h < niters; ++h) {
    double spw[15], suv[10], R[9], t[3];
    for (int i = 0; i < 5; ++i) {
      const int id = subsets[5 * h + i];
      for (int k = 0; k < 3; ++k) spw[3 * i + k] = obj[3 * id + k];
      for (int k = 0; k < 2; ++k) suv[2 * i + k] = img[2 * id + k];
    }
    epnp_cv(spw, suv, 5, cam, R, t);
    float Rf[9], tf[3];
    for (int i = 0; i < 9; ++i) Rf[i] = (float)R[i];
    for (int i = 0; i < 3; ++i) tf[i] = (float)t[i];
    int cnt = 0;
    for (int p = 0; p < P; ++p) {
      const float X = obj[3 * p], Y = obj[3 * p + 1], Z = obj[3 * p + 2];
      const float xc = Rf[0] * X + Rf[1] * Y + Rf[2] * Z + tf[0];
      const float yc = Rf[3] * X + Rf[4] * Y + Rf[5] * Z + tf[1];
      const float zc = Rf[6] * X + Rf[7] * Y + Rf[8] * Z + tf[2];
      const float du = img[2 * p] - ((float)cam.fu * xc / zc + (float)cam.uc);
      const float dv = img[2 * p + 1] - ((float)cam.fv * yc / zc + (float)cam.vc);
      if (du * du + dv * dv <= thr2) ++cnt;
    }
    if (cnt > (best_cnt > 4 ? best_cnt : 4)) {
      best_cnt = cnt;
      best = h;
      memcpy(bR, Rf, sizeof bR);
      memcpy(bt, tf, sizeof bt);
      niters = ransac_update_niters(conf, (double)(P - cnt) / P, 5, niters);
    }
  }
  if (best_h) *best_h = best;
  int n = 0;
  for (int p = 0; p < P && best >= 0; ++p) {
    const float X = obj[3 * p], Y = obj[3 * p + 1], Z = obj[3 * p + 2];
    const float xc = bR[0] * X + bR[1] * Y + bR[2] * Z + bt[0];
    const float yc = bR[3] * X + bR[4] * Y + bR[5] * Z + bt[1];
    const float zc = bR[6] * X + bR[7] * Y + bR[8] * Z + bt[2];
    const float du = img[2 * p] - ((float)cam.fu * xc / zc + (float)cam.uc);
    const float dv = img[2 * p + 1] - ((float)cam.fv * yc / zc + (float)cam.vc);
    if (du * du + dv * dv <= thr2) {
      for (int k = 0; k < 3; ++k) pw[3 * n + k] = obj[3 * p + k];
      for (int k = 0; k < 2; ++k) uv[2 * n + k] = img[2 * p + k];
      ++n;
    }
  }
  if (best >= 0 && n >= 5) {
    double R[9], t[3];
    epnp_cv(pw, uv, n, cam, R, t);
    for (int i = 0; i < 9; ++i) bR[i] = (float)R[i];
    for (int i = 0; i < 3; ++i) bt[i] = (float)t[i];
  } else if (best < 0) {
    for (int i = 0; i < 9; ++i) bR[i] = (i % 4 == 0) ? 1.f : 0.f;
    for (int i = 0; i < 3; ++i) bt[i] = 0.f;
  }
  memcpy(R_out, bR, sizeof bR);
  memcpy(t_out, bt, sizeof bt);
  return best >= 0 ? best_cnt : 0;
}

/* Diagnostics (tests/pnp_divergence.py): every hypothesis under either numerics (cv = 0: the
 * kernel-order EPnP, 1: the OpenCV-semantics one) -> f32 pose, inlier count, and per hypothesis
 * diag = approx (1..3) + 4 * (its Procrustes had det < 0) + 8 * (any approximation's did). */
void oracle_pnp_hypotheses_diag(const float* obj, const float* img, int P, const float* K4, const int* subsets,
                                int H, float thr, int cv, float* R_out, float* t_out, int* cnt_out, int* diag) {
  Cam cam = {K4[0], K4[1], K4[2], K4[3]};
  const float thr2 = thr * thr;
  for (int h = 0; h < H; ++h) {
    double spw[15], suv[10], R[9], t[3];
    for (int i = 0; i < 5; ++i) {
      const int id = subsets[5 * h + i];
      for (int k = 0; k < 3; ++k) spw[3 * i + k] = obj[3 * id + k];
      for (int k = 0; k < 2; ++k) suv[2 * i + k] = img[2 * id + k];
    }
    if (cv) epnp_cv(spw, suv, 5, cam, R, t);
    else epnp(spw, suv, 5, cam, R, t);
    float Rf[9], tf[3];
    for (int i = 0; i < 9; ++i) Rf[i] = (float)R[i];
    for (int i = 0; i < 3; ++i) tf[i] = (float)t[i];
    int cnt = 0;
    for (int p = 0; p < P; ++p) {
      const float X = obj[3 * p], Y = obj[3 * p + 1], Z = obj[3 * p + 2];
      const float xc = Rf[0] * X + Rf[1] * Y + Rf[2] * Z + tf[0];
      const float yc = Rf[3] * X + Rf[4] * Y + Rf[5] * Z + tf[1];
      const float zc = Rf[6] * X + Rf[7] * Y + Rf[8] * Z + tf[2];
      float du, dv;
      if (cv) {
        du = img[2 * p] - ((float)cam.fu * xc / zc + (float)cam.uc);
        dv = img[2 * p + 1] - ((float)cam.fv * yc / zc + (float)cam.vc);
      } else {
        const float iz = 1.0f / zc;
        du = img[2 * p] - ((float)cam.fu * xc * iz + (float)cam.uc);
        dv = img[2 * p + 1] - ((float)cam.fv * yc * iz + (float)cam.vc);
      }
      if (du * du + dv * dv <= thr2) ++cnt;
    }
    memcpy(R_out + 9 * h, Rf, sizeof Rf);
    memcpy(t_out + 3 * h, tf, sizeof tf);
    cnt_out[h] = cnt;
    diag[h] = g_diag_approx + 4 * g_diag_detneg[g_diag_approx] +
              8 * (g_diag_detneg[1] | g_diag_detneg[2] | g_diag_detneg[3]);
  }
}
