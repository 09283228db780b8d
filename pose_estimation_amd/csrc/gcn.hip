// 3D-GCN fusion kernels (FusionNetLite, lib/network/point/fusion.py:137-240).
//
//   krrn_knn_f32        get_neighbor_index / get_nearest_index (gcn3d.py:15-38) without the
//                       [n, n] distance matrix: candidates staged through LDS, top-(k+1) kept
//                       in registers, ties broken towards the lower index (the documented rule;
//                       torch.topk leaves tie order unspecified).
//   krrn_gcn_conv_f32   Conv_surface (gcn3d.py:88-112) and the gather/theta/max/sum half of
//                       Conv_layer / Conv_fuse_layer (gcn3d.py:136-216) fused with the BN1d +
//                       ReLU that FusionNetLite applies (fusion.py:183-213). The
//                       [n, k, S*C] theta / gathered / product tensors of the reference
//                       never exist: each neighbour row of the GEMM output Y is read once
//                       per (support, channel) straight from L2.
//   krrn_pool_max_f32   Pool_layer's max over the 4 neighbours (gcn3d.py:233-236), evaluated
//                       only at the randperm-sampled rows that the reference keeps (:238-241).
#include <math.h>

#include "krrn_common.h"

namespace {

constexpr int kKnnThreads = 256;
constexpr int kKnnChunk = 1024;  // candidates per LDS stage
constexpr int kKnnKmax = 16;

// Exact, FMA-free f32 expression order (documented in DESIGN.md / oracle/krrn_oracle.py):
//   inner = ((q0*c0 + q1*c1) + q2*c2) ...   (sequential over d, every op rounded)
//   |p|^2 = ((p0*p0 + p1*p1) + p2*p2) ...
//   neighbor (gcn3d.py:23): dist = ((inner * -2) + |c|^2) + |q|^2
//   nearest  (gcn3d.py:36): dist = (|c|^2 + |q|^2) - 2 * inner
template <int D>
__device__ __forceinline__ float knn_sqnorm(const float* p) {
#pragma clang fp contract(off)
  float s = p[0] * p[0];
#pragma unroll
  for (int i = 1; i < D; ++i) s = s + p[i] * p[i];
  return s;
}

template <int D>
__device__ __forceinline__ float knn_inner(const float* a, const float* b) {
#pragma clang fp contract(off)
  float s = a[0] * b[0];
#pragma unroll
  for (int i = 1; i < D; ++i) s = s + a[i] * b[i];
  return s;
}

// (d, index) lexicographic order: the stable-sort order the oracle pins (ties -> lower index).
__device__ __forceinline__ bool knn_less(float d0, int i0, float d1, int i1) {
  return d0 < d1 || (d0 == d1 && i0 < i1);
}

// One query = PARTS adjacent lanes. Lane `part` keeps the ascending top-KS of candidates
// j = part (mod PARTS) in registers (KS = k + drop rounded up to an instantiated size);
// the partial lists are then merged in (d, index) order, which equals the global stable
// top-KS because (d, index) is a total order. Block = 256 / PARTS queries. PARTS = 4 for the
// N x N level-0 search; 16 where a crop has few queries (the pools' N/4 sampled rows, level 1/2),
// so the grid still covers the CUs and each lane's serial scan is 4x shorter.
template <int D, int KS, int PARTS>
__global__ __launch_bounds__(kKnnThreads) void knn_kernel(
    const float* __restrict__ q, long long q_bs, int q_st, int nq, const int* __restrict__ qidx,
    const float* __restrict__ c, long long c_bs, int c_st, int nc, int K, int drop, int mode,
    int* __restrict__ out) {
#pragma clang fp contract(off)
  constexpr int DP = D == 3 ? 4 : 12;  // LDS record: coords + |c|^2 (+ pad)
  constexpr int QPB = kKnnThreads / PARTS;
  constexpr int STAGE = kKnnChunk * DP;
  constexpr int MERGE = kKnnThreads * KS * 2;
  __shared__ __attribute__((aligned(16))) float sc[STAGE > MERGE ? STAGE : MERGE];
  const int b = blockIdx.y;
  const int part = threadIdx.x % PARTS;
  const int ql = threadIdx.x / PARTS;
  const int t = blockIdx.x * QPB + ql;
  const bool active = t < nq;
  float qp[D];
  float qn = 0.f;
  {
    const int qi = active ? (qidx ? qidx[t] : t) : 0;
    const float* src = q + b * q_bs + (long long)qi * q_st;
#pragma unroll
    for (int i = 0; i < D; ++i) qp[i] = src[i];
    qn = knn_sqnorm<D>(qp);
  }
  float bd[KS];
  int bi[KS];
#pragma unroll
  for (int i = 0; i < KS; ++i) { bd[i] = INFINITY; bi[i] = 0x7fffffff; }

  const float* cb = c + b * c_bs;
  for (int j0 = 0; j0 < nc; j0 += kKnnChunk) {
    const int cnt = min(kKnnChunk, nc - j0);
    __syncthreads();
    for (int j = threadIdx.x; j < cnt; j += kKnnThreads) {
      const float* src = cb + (long long)(j0 + j) * c_st;
      float p[D];
#pragma unroll
      for (int i = 0; i < D; ++i) p[i] = src[i];
      float* dst = sc + j * DP;
#pragma unroll
      for (int i = 0; i < D; ++i) dst[i] = p[i];
      dst[D] = knn_sqnorm<D>(p);
    }
    __syncthreads();
    for (int j = part; j < cnt; j += PARTS) {
      const float* p = sc + j * DP;
      const float inner = knn_inner<D>(qp, p);
      const float cn = p[D];
      const float d = mode == 0 ? ((inner * -2.f) + cn) + qn : (cn + qn) - 2.f * inner;
      if (d < bd[KS - 1]) {
        // insertion in front of the first strictly larger entry (candidates of one lane arrive
        // in increasing index, so equal distances stay in index order), branch-free from the old
        // list: with c_s = d < bd[s] (monotone in s), slot s takes the old s - 1 entry where
        // c_{s-1}, the new one where c_s only, else keeps its own; the distance of that choice is
        // exactly med3(d, bd[s-1], bd[s]) (the list is sorted), one v_med3_f32 per slot
        const int ni = j0 + j;
        bool c[KS];
#pragma unroll
        for (int s2 = 0; s2 < KS; ++s2) c[s2] = d < bd[s2];
#pragma unroll
        for (int s2 = KS - 1; s2 > 0; --s2) {
          bi[s2] = c[s2 - 1] ? bi[s2 - 1] : (c[s2] ? ni : bi[s2]);
          bd[s2] = __builtin_amdgcn_fmed3f(d, bd[s2 - 1], bd[s2]);
        }
        bi[0] = c[0] ? ni : bi[0];
        bd[0] = fminf(d, bd[0]);
      }
    }
  }
  // ---- merge the kKnnParts partial lists of each query -------------------------------------
  __syncthreads();
  float* md = sc;
  int* mi = reinterpret_cast<int*>(sc + kKnnThreads * KS);
#pragma unroll
  for (int s2 = 0; s2 < KS; ++s2) {
    md[threadIdx.x * KS + s2] = bd[s2];
    mi[threadIdx.x * KS + s2] = bi[s2];
  }
  __syncthreads();
  if (!active || part != 0) return;
  const int base = threadIdx.x * KS;  // lists of lanes threadIdx.x .. threadIdx.x + PARTS - 1
  int hp[PARTS];
#pragma unroll
  for (int r = 0; r < PARTS; ++r) hp[r] = 0;
  const int ko = K - drop;
  int* o = out + ((long long)b * nq + t) * ko;
  for (int s2 = 0; s2 < K; ++s2) {
    float best_d = INFINITY;
    int best_i = 0x7fffffff, best_r = 0;
#pragma unroll
    for (int r = 0; r < PARTS; ++r) {
      if (hp[r] < KS) {
        const float dd = md[base + r * KS + hp[r]];
        const int ii = mi[base + r * KS + hp[r]];
        if (knn_less(dd, ii, best_d, best_i)) { best_d = dd; best_i = ii; best_r = r; }
      }
    }
#pragma unroll
    for (int r = 0; r < PARTS; ++r) hp[r] += (r == best_r);
    if (s2 >= drop) o[s2 - drop] = best_i;
  }
}

template <int D, int PARTS>
void knn_launch(int B, hipStream_t s, const float* q, long long q_bs, int q_st, int nq, const int* qidx,
                const float* c, long long c_bs, int c_st, int nc, int K, int drop, int mode, int* out) {
  const dim3 grid(krrn_cdiv(nq, kKnnThreads / PARTS), B);
#define KNN_CASE(KS)                                                                                          \
  hipLaunchKernelGGL((knn_kernel<D, KS, PARTS>), grid, dim3(kKnnThreads), 0, s, q, q_bs, q_st, nq, qidx, c, c_bs, \
                     c_st, nc, K, drop, mode, out)
  if (K <= 1) KNN_CASE(1);
  else if (K <= 2) KNN_CASE(2);
  else if (K <= 5) KNN_CASE(5);
  else if (K <= 8) KNN_CASE(8);
  else if (K <= 11) KNN_CASE(11);
  else KNN_CASE(16);
#undef KNN_CASE
}

}  // namespace

KRRN_API int krrn_knn_f32(const float* q, long long q_bs, int q_st, int nq, const int* qidx, const float* c,
                          long long c_bs, int c_st, int nc, int d, int k, int drop_first, int mode, int B,
                          int* out, void* stream) {
  if (!q || !c || !out) return KRRN_EARG;
  if (d != 3 && d != 9) return KRRN_ESHAPE;
  if (k < 1 || k + (drop_first ? 1 : 0) > kKnnKmax || nq < 1 || nc < 1 || B < 1) return KRRN_ESHAPE;
  if (k + (drop_first ? 1 : 0) > nc) return KRRN_ESHAPE;
  if (mode != 0 && mode != 1) return KRRN_EARG;
  const int K = k + (drop_first ? 1 : 0);
  hipStream_t s = (hipStream_t)stream;
  const int dr = drop_first ? 1 : 0;
  // lanes per query: 16 when 4 lanes would leave the grid under ~4 blocks per CU (few queries
  // per crop) AND every lane still scans >= 48 candidates (the 16-list merge is serial): the
  // pools' N/4 sampled rows against N candidates (57 -> 34 us at B = 64, N = 1000); the level-0
  // N x N search and the short level-1 / 2 / nearest scans keep 4 (profiles/bench_knn.py)
  const long long blocks4 = (long long)krrn_cdiv(nq, kKnnThreads / 4) * B;
  const bool wide = blocks4 < 1024 && nc >= 16 * 48;
  if (d == 3) {
    if (wide) knn_launch<3, 16>(B, s, q, q_bs, q_st, nq, qidx, c, c_bs, c_st, nc, K, dr, mode, out);
    else knn_launch<3, 4>(B, s, q, q_bs, q_st, nq, qidx, c, c_bs, c_st, nc, K, dr, mode, out);
  } else {
    if (wide) knn_launch<9, 16>(B, s, q, q_bs, q_st, nq, qidx, c, c_bs, c_st, nc, K, dr, mode, out);
    else knn_launch<9, 4>(B, s, q, q_bs, q_st, nq, qidx, c, c_bs, c_st, nc, K, dr, mode, out);
  }
  return krrn_launch_status();
}

// ------------------------------------------------------------------------------------------
// GCN gather-conv
// ------------------------------------------------------------------------------------------
namespace {

constexpr int kGcnThreads = 256;
constexpr int kGcnKmax = 16;
constexpr int kGcnSmax = 8;  // support_num bound of the LDS-staged 3-D form (the model uses 7)
#ifndef GCN3_WAVES
#define GCN3_WAVES 4  // waves per SIMD the 3-D form is register-bounded for (126 VGPRs, no spills)
#endif

// Block = 256 / LP points of one crop; a point is LP lanes, lane l owning channels 4l.. (+4 LP
// per step when C > 4 LP). LP = 32 for C = 128 (levels 0 / 1: 8 points per block), LP = 128 for
// C = 512 (level 2: 2 points per block, so each lane walks one channel group instead of four —
// that path is gather-latency bound, 62 points per crop). For each support s and neighbour j a
// lane reads one float4 of the neighbour's Y row (16 LP-byte coalesced per point), so every
// neighbour row segment Y[nj, C + s*C : C + (s+1)*C] is one wide read. The block -> (crop,
// points) map is XCD-aware: consecutive point groups of one crop share an XCD and its L2, where
// their overlapping neighbourhoods (choose is pixel-ordered, so neighbours have nearby indices)
// hit. KC = compile-time k (0: runtime k).
template <int D, bool HAS_Y, int KC, int LP>
__global__ __launch_bounds__(kGcnThreads) void gcn_conv_kernel(
    const int* __restrict__ idx, int n, int k, const float* __restrict__ v, long long v_bs, int v_st,
    const float* __restrict__ dn, int S, int C, const float* __restrict__ Y,
    const float* __restrict__ bn_s, const float* __restrict__ bn_b, int relu, float* __restrict__ out,
    long long o_bs, int o_st) {
  constexpr int kPts = kGcnThreads / LP;
  __shared__ float sdir[kPts * kGcnKmax * D];
  __shared__ int snb[kPts * kGcnKmax];
  const int gx = gridDim.x;
  const int lin = krrn_xcd_remap(blockIdx.x + gx * blockIdx.y, gx * gridDim.y);
  const int b = lin / gx;
  const int p0 = (lin - b * gx) * kPts;
  const int np = min(kPts, n - p0);
  const int kk = KC ? KC : k;
  const float* vb = v + b * v_bs;
  // 1) neighbour directions, F.normalize(v[j] - v[i], dim=-1) (gcn3d.py:60-69)
  for (int e = threadIdx.x; e < np * kk; e += kGcnThreads) {
    const int p = e / kk, j = e - (e / kk) * kk;
    const int pi = p0 + p;
    const int nj = idx[((long long)b * n + pi) * kk + j];
    snb[p * kGcnKmax + j] = nj;
    float dv[D];
    float ss = 0.f;
#pragma unroll
    for (int i = 0; i < D; ++i) {
      dv[i] = vb[(long long)nj * v_st + i] - vb[(long long)pi * v_st + i];
      ss += dv[i] * dv[i];
    }
    const float nr = fmaxf(sqrtf(ss), 1e-12f);
#pragma unroll
    for (int i = 0; i < D; ++i) sdir[(p * kGcnKmax + j) * D + i] = dv[i] / nr;
  }
  __syncthreads();
  const int p = threadIdx.x / LP, l = threadIdx.x % LP;
  if (p >= np) return;
  const int pi = p0 + p;
  const int SC = S * C;
  const int yrow = (S + 1) * C;  // n * yrow < 2^31 is checked on the host
  const float* yb = HAS_Y ? Y + b * (long long)n * yrow : nullptr;
  const float* dp = sdir + p * kGcnKmax * D;
  const int* nbp = snb + p * kGcnKmax;
  constexpr int KU = KC ? KC : kGcnKmax;
  // neighbour row offsets (floats, support block 0), hoisted out of the support loop
  int yo[KU];
#pragma unroll
  for (int j = 0; j < KU; ++j) yo[j] = (KC || j < kk) ? nbp[j] * yrow + C : 0;
  // 3-D directions of a fixed neighbour count (level 0 / 1: 30 floats) live in registers for the
  // whole point; the 9-D level-2 ones stay in LDS behind an opaque pointer (see below)
  constexpr bool kHoist = KC > 0 && D * KU <= 48;
  float dreg[kHoist ? KU * D : 1];
  if constexpr (kHoist) {
#pragma unroll
    for (int e = 0; e < KU * D; ++e) dreg[e] = dp[e];
  }
  for (int c = 4 * l; c < C; c += 4 * LP) {
    f32x4 acc = {0.f, 0.f, 0.f, 0.f};
    // The support loop stays rolled and, where Y is gathered, the LDS direction reads stay
    // inside it (an opaque pointer per iteration): unrolled and hoisted into paired registers
    // they took every VGPR (level 2, 9-D: occupancy 1, 170 -> 70 us per launch). The surface
    // conv (no gathers, VALU-bound) and the 3-D gathered convs (kHoist: 30 floats, occupancy 4 -> 2
    // but no flat loads in the loop; all gather-convs 1.16 -> 1.10 ms per step) keep theirs in
    // registers.
#pragma unroll 1
    for (int s = 0; s < S; ++s) {
      const int so = s * C + c;
      int dpo = p * kGcnKmax * D;
      if constexpr (HAS_Y && !kHoist) asm volatile("" : "+v"(dpo));
      const float* dps = sdir + dpo;
      f32x4 yv[HAS_Y ? KU : 1];
      if constexpr (HAS_Y) {
#pragma unroll
        for (int j = 0; j < KU; ++j)
          if (KC || j < kk) yv[j] = *reinterpret_cast<const f32x4*>(yb + yo[j] + so);
      }
      f32x4 w[D];
#pragma unroll
      for (int i = 0; i < D; ++i) w[i] = *reinterpret_cast<const f32x4*>(dn + i * SC + so);
      f32x4 m = {-INFINITY, -INFINITY, -INFINITY, -INFINITY};
#pragma unroll
      for (int j = 0; j < KU; ++j) {
        if (!KC && j >= kk) continue;  // predicated (a break here put yv in scratch memory)
        const float* dr = kHoist ? dreg + j * D : dps + j * D;
        f32x4 th = dr[0] * w[0];
#pragma unroll
        for (int i = 1; i < D; ++i) th += dr[i] * w[i];
        if constexpr (HAS_Y) {
          // act = ReLU(theta) * support (gcn3d.py:150-156)
#pragma unroll
          for (int q = 0; q < 4; ++q) th[q] = fmaxf(th[q], 0.f);
          th *= yv[j];
        }
#pragma unroll
        for (int q = 0; q < 4; ++q) m[q] = fmaxf(m[q], th[q]);
      }
      if constexpr (!HAS_Y) {
        // Conv_surface: max_k ReLU(theta) == ReLU(max_k theta) exactly (ReLU is monotone)
#pragma unroll
        for (int q = 0; q < 4; ++q) m[q] = fmaxf(m[q], 0.f);
      }
      acc += m;
    }
    f32x4 o = acc;
    if constexpr (HAS_Y) o = *reinterpret_cast<const f32x4*>(yb + pi * yrow + c) + o;
#pragma unroll
    for (int q = 0; q < 4; ++q) {
      if (bn_s) o[q] = o[q] * bn_s[c + q] + bn_b[c + q];
      if (relu) o[q] = fmaxf(o[q], 0.f);
    }
    *reinterpret_cast<f32x4*>(out + b * o_bs + (long long)pi * o_st + c) = o;
  }
}

// Level-0 / level-1 form (3-D directions, C = 128, compile-time k): the same arithmetic as
// gcn_conv_kernel<3, HAS_Y, KC, 32> (bit-identical outputs), laid out for occupancy and
// memory-level parallelism instead of register reuse:
//   * the normalised support directions dn [3][S*C] are staged in LDS once per block (10.5 KB),
//     not re-read through L1 per support by every lane;
//   * the neighbour rows are read with buffer loads: one 32-bit byte offset per neighbour (the
//     crop's Y is one buffer resource) and the support as the scalar offset, so the support loop
//     carries no 64-bit address arithmetic (the old form kept ten 64-bit pointers and stepped
//     them every support: 228 VGPRs, 2 waves per SIMD);
//   * __launch_bounds__(256, 4): >= 4 waves per SIMD, each with its k gather loads in flight.
// DBG (diagnostics build only, -DKRRN_DIAG=1: krrn_gcn_debug, csrc/krrn_diag.h; surface convs only): per-point / per-block records of what the
// block read and held in LDS, at the start and at the end of the support loop.
template <bool HAS_Y, int KC, bool DBG = false>
__global__ __launch_bounds__(256, GCN3_WAVES) void gcn_conv3_kernel(
    const int* __restrict__ idx, int n, const float* __restrict__ v, long long v_bs, int v_st,
    const float* __restrict__ dn, int S, const float* __restrict__ Y, const float* __restrict__ bn_s,
    const float* __restrict__ bn_b, int relu, float* __restrict__ out, long long o_bs, int o_st,
    unsigned* __restrict__ dbg) {
  constexpr int C = 128, LP = 32, kPts = kGcnThreads / LP;
  __shared__ f32x4 sdn[3 * kGcnSmax * C / 4];
  __shared__ float sdir[kPts * KC * 3];
  __shared__ int snb[kPts * KC];
  const int gx = gridDim.x;
  const int lin = krrn_xcd_remap(blockIdx.x + gx * blockIdx.y, gx * gridDim.y);
  const int b = lin / gx;
  const int p0 = (lin - b * gx) * kPts;
  const int np = min(kPts, n - p0);
  const float* vb = v + b * v_bs;
  const int SC = S * C;
  for (int e = threadIdx.x; e < 3 * SC / 4; e += kGcnThreads) sdn[e] = reinterpret_cast<const f32x4*>(dn)[e];
  for (int e = threadIdx.x; e < np * KC; e += kGcnThreads) {
    const int p = e / KC, j = e - (e / KC) * KC;
    const int pi = p0 + p;
    const int nj = idx[((long long)b * n + pi) * KC + j];
    snb[p * KC + j] = nj;
    float dv[3];
    float ss = 0.f;
#pragma unroll
    for (int i = 0; i < 3; ++i) {
      dv[i] = vb[(long long)nj * v_st + i] - vb[(long long)pi * v_st + i];
      ss += dv[i] * dv[i];
    }
    const float nr = fmaxf(sqrtf(ss), 1e-12f);
#pragma unroll
    for (int i = 0; i < 3; ++i) sdir[(p * KC + j) * 3 + i] = dv[i] / nr;
    if constexpr (!HAS_Y && DBG) {  // the neighbour and coordinates as read
      unsigned* r = dbg + (((long long)b * n + pi) * KC + j) * 8;
      r[0] = (unsigned)nj;
#pragma unroll
      for (int i = 0; i < 3; ++i) {
        r[1 + i] = __float_as_uint(vb[(long long)pi * v_st + i]);
        r[4 + i] = __float_as_uint(vb[(long long)nj * v_st + i]);
      }
      r[7] = (unsigned)b;
    }
  }
  __syncthreads();
  __shared__ unsigned sdig[4];
  // digest of the staged directions (sdn) and point directions (sdir) as this block's LDS holds them
  auto digest = [&](unsigned* r) {
    if (threadIdx.x == 0) sdig[0] = sdig[1] = sdig[2] = sdig[3] = 0u;
    __syncthreads();
    unsigned x = 0u, a = 0u, x2 = 0u, a2 = 0u;
    for (int e = threadIdx.x; e < 3 * SC / 4; e += kGcnThreads) {
      const f32x4 q = sdn[e];
#pragma unroll
      for (int i = 0; i < 4; ++i) {
        const unsigned u = __float_as_uint(q[i]);
        x ^= u * (unsigned)(4 * e + i + 1);
        a += u;
      }
    }
    for (int e = threadIdx.x; e < np * KC * 3; e += kGcnThreads) {
      const unsigned u = __float_as_uint(sdir[e]);
      x2 ^= u * (unsigned)(e + 1);
      a2 += u;
    }
    atomicXor(&sdig[0], x);
    atomicAdd(&sdig[1], a);
    atomicXor(&sdig[2], x2);
    atomicAdd(&sdig[3], a2);
    __syncthreads();
    if (threadIdx.x == 0) {
      r[0] = sdig[0];
      r[1] = sdig[1];
      r[2] = sdig[2];
      r[3] = sdig[3];
    }
  };
  unsigned* rblk = nullptr;
  if constexpr (!HAS_Y && DBG) {
    // per block (after the per-point records): digests at the start (0-3), XCC / HW id (4, 5), the
    // kernel arguments as read (6-13), digests after the support loop (16-19)
    rblk = dbg + (long long)gridDim.y * n * KC * 8 + (long long)lin * 20;
    digest(rblk);
    if (threadIdx.x == 0) {
      unsigned xcc, hwid;
      asm volatile("s_getreg_b32 %0, hwreg(HW_REG_XCC_ID)" : "=s"(xcc));
      asm volatile("s_getreg_b32 %0, hwreg(HW_REG_HW_ID)" : "=s"(hwid));
      const unsigned long long po = (unsigned long long)out, pd = (unsigned long long)dn, pv = (unsigned long long)v;
      rblk[4] = xcc;
      rblk[5] = hwid;
      rblk[6] = (unsigned)po;
      rblk[7] = (unsigned)(po >> 32);
      rblk[8] = (unsigned)o_bs;
      rblk[9] = (unsigned)o_st;
      rblk[10] = (unsigned)S;
      rblk[11] = (unsigned)relu;
      rblk[12] = (unsigned)pd;
      rblk[13] = (unsigned)pv;
    }
  }
  const int p = threadIdx.x / LP, l = threadIdx.x % LP;
  if constexpr (!(!HAS_Y && DBG)) {
    if (p >= np) return;
  }
  const bool live = p < np;
  const int pi = p0 + p;
  const int c = 4 * l;
  const int yrow = (S + 1) * C;
  const int dpo = p * KC * 3;  // this point's directions in sdir
  __amdgpu_buffer_rsrc_t rs;
  if constexpr (HAS_Y)
    rs = __builtin_amdgcn_make_buffer_rsrc((void*)(Y + (long long)b * n * yrow), (short)0, n * yrow * 4, 0x00020000);
  const int npo = p * KC;  // this point's neighbour rows in snb
  const unsigned cbyte = (unsigned)((C + c) * 4);
  f32x4 acc = {0.f, 0.f, 0.f, 0.f};
#pragma unroll 1
  for (int s = 0; s < S; ++s) {
    f32x4 yv[HAS_Y ? KC : 1];
    if constexpr (HAS_Y) {
      // neighbour rows re-read from LDS (broadcast) every support: 10 fewer live VGPRs. The
      // offset (not a pointer) is made opaque, so the reads stay ds_read on the LDS array
      int nbo = npo;
      asm volatile("" : "+v"(nbo));
#pragma unroll
      for (int j = 0; j < KC; ++j) {
        yv[j] = __builtin_bit_cast(
            f32x4, __builtin_amdgcn_raw_buffer_load_b128(rs, (unsigned)(snb[nbo + j] * yrow * 4) + cbyte, s * C * 4, 0));
      }
    }
    f32x4 w[3];
#pragma unroll
    for (int i = 0; i < 3; ++i) w[i] = sdn[(i * SC + s * C + c) >> 2];
    // the directions are re-read from LDS (broadcast) every support: hoisted they cost 30 VGPRs
    int dro = dpo;
    asm volatile("" : "+v"(dro));
    const float* dreg = sdir + dro;
    f32x4 m = {-INFINITY, -INFINITY, -INFINITY, -INFINITY};
#pragma unroll
    for (int j = 0; j < KC; ++j) {
      f32x4 th = dreg[j * 3] * w[0];
#pragma unroll
      for (int i = 1; i < 3; ++i) th += dreg[j * 3 + i] * w[i];
      if constexpr (HAS_Y) {
#pragma unroll
        for (int q = 0; q < 4; ++q) th[q] = fmaxf(th[q], 0.f);
        th *= yv[j];
      }
#pragma unroll
      for (int q = 0; q < 4; ++q) m[q] = fmaxf(m[q], th[q]);
    }
    if constexpr (!HAS_Y) {
#pragma unroll
      for (int q = 0; q < 4; ++q) m[q] = fmaxf(m[q], 0.f);
    }
    if constexpr (!HAS_Y && DBG) {
      // per (block, thread, support): the support's max and the first direction-weight quad as
      // this thread held them in registers (after the per-block records)
      float* rt = reinterpret_cast<float*>(dbg + (long long)gridDim.y * n * KC * 8 + (long long)gridDim.x * gridDim.y * 20) +
                  (((long long)lin * kGcnThreads + threadIdx.x) * kGcnSmax + s) * 8;
      *reinterpret_cast<f32x4*>(rt) = m;
      *reinterpret_cast<f32x4*>(rt + 4) = w[0];
    }
    acc += m;
  }
  f32x4 o = acc;
  if constexpr (HAS_Y) o = *reinterpret_cast<const f32x4*>(Y + (long long)b * n * yrow + (long long)pi * yrow + c) + o;
#pragma unroll
  for (int q = 0; q < 4; ++q) {
    if (bn_s) o[q] = o[q] * bn_s[c + q] + bn_b[c + q];
    if (relu) o[q] = fmaxf(o[q], 0.f);
  }
  if (live) *reinterpret_cast<f32x4*>(out + b * o_bs + (long long)pi * o_st + c) = o;
  if constexpr (!HAS_Y && DBG) {
    __syncthreads();
    digest(rblk + 16);
  }
}

}  // namespace

#if KRRN_DIAG
#include "krrn_diag.h"
#include <mutex>
namespace {
// krrn_gcn_debug: where the surface convs (Y == NULL) of the 3-D form dump, per (crop, point,
// neighbour), the neighbour index and both points' coordinates as the kernel read them (8 words).
// Launch i writes slot i % nslots. Diagnostics only (profiles/f0_shadow.py); off unless set.
struct GcnDebug {
  std::mutex mu;
  unsigned* buf = nullptr;
  long long slot_words = 0;
  int nslots = 1;
  long long count = 0;
} g_gcn_dbg;
}  // namespace

KRRN_API int krrn_gcn_debug(void* buf, int nslots, long long slot_words) {
  const std::lock_guard<std::mutex> lk(g_gcn_dbg.mu);
  if (buf && (nslots < 1 || slot_words < 1)) return KRRN_EARG;
  g_gcn_dbg.buf = reinterpret_cast<unsigned*>(buf);
  g_gcn_dbg.nslots = nslots < 1 ? 1 : nslots;
  g_gcn_dbg.slot_words = slot_words;
  g_gcn_dbg.count = 0;
  return KRRN_OK;
}

#endif  // KRRN_DIAG

KRRN_API int krrn_gcn_conv_f32(const int* idx, int n, int k, const float* v, long long v_bs, int v_st, int d,
                               const float* dn, int S, int C, const float* Y, const float* bn_scale,
                               const float* bn_bias, int relu, float* out, long long o_bs, int o_st, int B,
                               void* stream) {
  if (!idx || !v || !dn || !out) return KRRN_EARG;
  if ((bn_scale == nullptr) != (bn_bias == nullptr)) return KRRN_EARG;
  if (d != 3 && d != 9) return KRRN_ESHAPE;
  if (k < 1 || k > kGcnKmax || n < 1 || S < 1 || C < 1 || B < 1) return KRRN_ESHAPE;
  if ((C & 3) || (o_st & 3) || (o_bs & 3) || !krrn_aligned16(out) || !krrn_aligned16(dn)) return KRRN_EALIGN;
  if (Y && !krrn_aligned16(Y)) return KRRN_EALIGN;
  if ((long long)n * (S + 1) * C >= (1LL << 31)) return KRRN_ESHAPE;  // 32-bit row offsets per crop
  const bool wide = C >= 512;  // LP = 128 lanes per point (see the kernel comment)
  dim3 grid(krrn_cdiv(n, wide ? kGcnThreads / 128 : kGcnThreads / 32), B);
  hipStream_t s = (hipStream_t)stream;
  if (d == 3 && C == 128 && S <= kGcnSmax && (k == 10 || k == 8) &&
      (long long)n * (S + 1) * C * 4 < (1LL << 31)) {
    unsigned* dbg = nullptr;
#if KRRN_DIAG
    if (!Y && g_gcn_dbg.buf) {
      const std::lock_guard<std::mutex> lk(g_gcn_dbg.mu);
      dbg = g_gcn_dbg.buf + (g_gcn_dbg.count++ % g_gcn_dbg.nslots) * g_gcn_dbg.slot_words;
    }
#endif
#define KRRN_GCN3(HY, KC) \
  hipLaunchKernelGGL((gcn_conv3_kernel<HY, KC>), grid, dim3(kGcnThreads), 0, s, idx, n, v, v_bs, v_st, dn, S, Y, \
                     bn_scale, bn_bias, relu, out, o_bs, o_st, dbg)
#if KRRN_DIAG
    if (dbg) {
      if (k == 10)
        hipLaunchKernelGGL((gcn_conv3_kernel<false, 10, true>), grid, dim3(kGcnThreads), 0, s, idx, n, v, v_bs,
                           v_st, dn, S, Y, bn_scale, bn_bias, relu, out, o_bs, o_st, dbg);
      else
        hipLaunchKernelGGL((gcn_conv3_kernel<false, 8, true>), grid, dim3(kGcnThreads), 0, s, idx, n, v, v_bs,
                           v_st, dn, S, Y, bn_scale, bn_bias, relu, out, o_bs, o_st, dbg);
      return krrn_launch_status();
    }
#endif
    if (Y) {
      if (k == 10) KRRN_GCN3(true, 10); else KRRN_GCN3(true, 8);
    } else {
      if (k == 10) KRRN_GCN3(false, 10); else KRRN_GCN3(false, 8);
    }
#undef KRRN_GCN3
    return krrn_launch_status();
  }
#define KRRN_GCN_LAUNCH(DD, HY, KC)                                                                        \
  if (wide)                                                                                                \
    hipLaunchKernelGGL((gcn_conv_kernel<DD, HY, KC, 128>), grid, dim3(kGcnThreads), 0, s, idx, n, k, v,   \
                       v_bs, v_st, dn, S, C, Y, bn_scale, bn_bias, relu, out, o_bs, o_st);                 \
  else                                                                                                     \
    hipLaunchKernelGGL((gcn_conv_kernel<DD, HY, KC, 32>), grid, dim3(kGcnThreads), 0, s, idx, n, k, v,    \
                       v_bs, v_st, dn, S, C, Y, bn_scale, bn_bias, relu, out, o_bs, o_st)
#define KRRN_GCN_K(DD, HY)                 \
  if (k == 10) KRRN_GCN_LAUNCH(DD, HY, 10); \
  else if (k == 7) KRRN_GCN_LAUNCH(DD, HY, 7); \
  else KRRN_GCN_LAUNCH(DD, HY, 0)
  if (d == 3) {
    if (Y) { KRRN_GCN_K(3, true); } else { KRRN_GCN_K(3, false); }
  } else {
    if (Y) { KRRN_GCN_K(9, true); } else { KRRN_GCN_K(9, false); }
  }
#undef KRRN_GCN_K
#undef KRRN_GCN_LAUNCH
  return krrn_launch_status();
}

// ------------------------------------------------------------------------------------------
// Pool_layer max at the sampled rows
// ------------------------------------------------------------------------------------------
namespace {
__global__ void pool_max_kernel(const int* __restrict__ nbr, int nq, int kk, const float* __restrict__ F,
                                long long f_bs, int f_st, int C4, float* __restrict__ out, long long o_bs,
                                int o_st) {
  const int b = blockIdx.y;
  const long long e = (long long)blockIdx.x * blockDim.x + threadIdx.x;
  if (e >= (long long)nq * C4) return;
  const int t = (int)(e / C4), c4 = (int)(e - (e / C4) * C4);
  const int* nb = nbr + ((long long)b * nq + t) * kk;
  const float* fb = F + b * f_bs;
  f32x4 m = *reinterpret_cast<const f32x4*>(fb + (long long)nb[0] * f_st + 4 * c4);
  for (int j = 1; j < kk; ++j) {
    const f32x4 x = *reinterpret_cast<const f32x4*>(fb + (long long)nb[j] * f_st + 4 * c4);
    m.x = fmaxf(m.x, x.x); m.y = fmaxf(m.y, x.y); m.z = fmaxf(m.z, x.z); m.w = fmaxf(m.w, x.w);
  }
  *reinterpret_cast<f32x4*>(out + b * o_bs + (long long)t * o_st + 4 * c4) = m;
}
}  // namespace

KRRN_API int krrn_pool_max_f32(const int* nbr, int nq, int kk, const float* F, long long f_bs, int f_st, int C,
                               float* out, long long o_bs, int o_st, int B, void* stream) {
  if (!nbr || !F || !out) return KRRN_EARG;
  if (nq < 1 || kk < 1 || C < 1 || B < 1) return KRRN_ESHAPE;
  if ((C & 3) || (f_st & 3) || (o_st & 3) || (f_bs & 3) || (o_bs & 3) || !krrn_aligned16(F) || !krrn_aligned16(out))
    return KRRN_EALIGN;
  const long long tot = (long long)nq * (C / 4);
  dim3 grid((unsigned)((tot + 255) / 256), B);
  hipLaunchKernelGGL(pool_max_kernel, grid, dim3(256), 0, (hipStream_t)stream, nbr, nq, kk, F, f_bs, f_st, C / 4,
                     out, o_bs, o_st);
  return krrn_launch_status();
}
