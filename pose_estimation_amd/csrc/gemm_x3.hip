// Dense GEMM on the gfx950 bf16 matrix cores at f32 accuracy (split-bf16 operands).
//
//   out[m, n] = act( sum_k A[m, k] W[n, k] + bias[n] + res[m, n] )     (scale folded into W)
//
// The fusion's and TBase's plain GEMMs (the GCN `feature_map @ weights`,
// lib/network/point/gcn3d.py:125-127, 184-186; P1: TBase's Conv1d chain, posenet.py:51-96) are
// M = B*n points long, K = 128..1024 deep and N = 256..4096 wide. hipBLASLt's f32 kernels ran them
// at 94-140 TFLOP/s against a 157 TFLOP/s f32 MFMA peak; here each f32 operand is split into three
// exact bf16 terms (x = h + m + l, as in conv_gemm.hip / winograd.hip) and a product is summed over
// the six term pairs hh hm mh hl lh mm on v_mfma_f32_32x32x16_bf16 with f32 accumulation — the
// dropped ml lm ll are below 2^-23 |a b|, the f32 product rounding — at 2.67x the f32 MFMA rate.
//
// Tiling (MI355X-first):
//   * block = 4 waves, output tile 128 rows x 128 columns; wave w owns the 32 columns
//     [32 w, 32 w + 32) over all 128 rows (four 32x32 accumulators), so a weight fragment feeds
//     4 x 3 MFMAs and an activation fragment 3;
//   * activations: K in chunks of 32, global (float4; 8 lanes per 128-B row segment, raw buffer
//     loads so rows past M read 0) -> registers -> split into the LDS chain [h h m l] per 4 k
//     (row pitch 68 dwords = 17 16-B slots: conflict-free ds_read_b128), double buffered, one
//     barrier per chunk; the next chunk's loads are issued one group after the barrier, so they
//     have ~3 groups of MFMAs (~2300 cycles) to land;
//   * weights never touch LDS (no wave reads another's columns): the host pre-splits them into
//     wave fragments (ops.gemm_weights_x3), so one group's operand is two fully coalesced 1-KB wave
//     loads from L2, issued two groups ahead into a 4-deep register ring;
//   * epilogue: each finished 32 x 32 tile through a per-wave LDS slot, stored as float4 rows;
//   * two blocks per CU (68 KB LDS each): one block's barrier / epilogue overlaps the other's
//     MFMAs; tiles are ordered n-inner and XCD-remapped so a row block's column tiles share an L2
//     (the A rows are re-read from L2, not HBM).
//
// Gathered-A form (GA, krrn_gemm_x3_gather_f32): row m = (crop b, point i) of A is built while it is
// staged, A[m, k] = relu(P[b, ia[b, i], k] + Q[b, ib[b, i], k]), from two small per-crop row tables —
// TBase conv1 by linearity (posenet.py: the fusion's level rows times W1, BN / bias / one-hot
// column folded into them) feeding conv2 directly, so the 1024-wide h1 is never written to HBM.
#include "krrn_common.h"

namespace {

typedef __bf16 gx_bf16x8 __attribute__((ext_vector_type(8)));
typedef __bf16 gx_bf16x2 __attribute__((ext_vector_type(2)));
typedef float gx_f32x2 __attribute__((ext_vector_type(2)));
typedef unsigned gx_u32x4 __attribute__((ext_vector_type(4)));

constexpr int BM = 128, BN = 128;
constexpr int KC = 16;          // k per LDS chunk
constexpr int NG = KC / 8;      // 8-k MFMA groups per chunk
constexpr int PX = 3 * KC + 4;  // dwords per LDS row: 12 per 4 k + 4 pad (odd number of 16-B slots)

struct GemmArgs {
  const float* a;
  // GA: A[m] = relu(a[b * a_grp + ia[m] * lda] + a2[b * a2_grp + ib[m] * lda2]), b = m / npts
  const float* a2;
  const int* ia;
  const int* ib;
  long long a2_grp;
  int lda2, npts;
  const unsigned* w;  // wave fragments [N/32][K/8][2][64][4]
  const float* bias;
  const float* res;
  float* out;
  int lda, M, K, N, ldr, ldo, relu;
  long long a_grp, o_grp, r_grp;
  int mt, nt, total;  // row tiles, column tiles per group; tiles in the grid
};

__device__ __forceinline__ unsigned gx_pk(float a, float b) {
  return __builtin_bit_cast(unsigned, __builtin_convertvector(gx_f32x2{a, b}, gx_bf16x2));  // RNE
}

// 4 consecutive k of one row -> the three MFMA operand quads [h h] [h m] [m l]
__device__ __forceinline__ void gx_split(const f32x4 x, gx_u32x4& q0, gx_u32x4& q1, gx_u32x4& q2) {
  const unsigned h0 = gx_pk(x[0], x[1]), h1 = gx_pk(x[2], x[3]);
  const float r0 = x[0] - __builtin_bit_cast(float, h0 << 16), r1 = x[1] - __builtin_bit_cast(float, h0 & 0xFFFF0000u);
  const float r2 = x[2] - __builtin_bit_cast(float, h1 << 16), r3 = x[3] - __builtin_bit_cast(float, h1 & 0xFFFF0000u);
  const unsigned m0 = gx_pk(r0, r1), m1 = gx_pk(r2, r3);
  const unsigned l0 = gx_pk(r0 - __builtin_bit_cast(float, m0 << 16), r1 - __builtin_bit_cast(float, m0 & 0xFFFF0000u));
  const unsigned l1 = gx_pk(r2 - __builtin_bit_cast(float, m1 << 16), r3 - __builtin_bit_cast(float, m1 & 0xFFFF0000u));
  q0 = gx_u32x4{h0, h1, h0, h1};
  q1 = gx_u32x4{h0, h1, m0, m1};
  q2 = gx_u32x4{m0, m1, l0, l1};
}

__device__ __forceinline__ gx_bf16x8 gx_op(const gx_u32x4 v) { return __builtin_bit_cast(gx_bf16x8, v); }

template <bool GA>
__global__ __launch_bounds__(256, 2) void gemm_x3_kernel(const GemmArgs g) {
  __shared__ __attribute__((aligned(16))) unsigned smem[2 * BM * PX];

  const int tpg = g.mt * g.nt;
  const int bid = krrn_xcd_remap(blockIdx.x, g.total);
  const int grp = bid / tpg, rem = bid - grp * tpg;
  const int tm = rem / g.nt, tn = rem - tm * g.nt;
  const int m0 = tm * BM, n0 = tn * BN;
  const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
  const int frow = lane & 31, fh = lane >> 5;

  // activation staging: thread -> rows srow + 64 i (i < 2), 4 k at kq of each chunk
  const int srow = tid >> 2, kq = (tid & 3) * 4;
  const float* abase = GA ? g.a : g.a + grp * g.a_grp + (size_t)m0 * g.lda;
  const int rows = min(BM, g.M - m0);
  // GA: the two row tables are whole buffer resources (bounds checked on the host); rows past M
  // read 0 through an out-of-range offset
  const __amdgpu_buffer_rsrc_t rsA = __builtin_amdgcn_make_buffer_rsrc(
      (void*)abase, (short)0, GA ? (int)(g.a_grp * (g.M / g.npts) * 4) : ((rows - 1) * g.lda + g.K) * 4, 0x00020000);
  __amdgpu_buffer_rsrc_t rsA2;
  unsigned aoff[2], aoff2[2];
  if constexpr (GA) {
    rsA2 = __builtin_amdgcn_make_buffer_rsrc((void*)g.a2, (short)0, (int)(g.a2_grp * (g.M / g.npts) * 4),
                                             0x00020000);
#pragma unroll
    for (int i = 0; i < 2; ++i) {
      const int m = m0 + srow + 64 * i;
      if (m < g.M) {
        const int b = m / g.npts;
        aoff[i] = (unsigned)((b * g.a_grp + (long long)g.ia[m] * g.lda + kq) * 4);
        aoff2[i] = (unsigned)((b * g.a2_grp + (long long)g.ib[m] * g.lda2 + kq) * 4);
      } else {
        aoff[i] = aoff2[i] = 0x80000000u;
      }
    }
  } else {
#pragma unroll
    for (int i = 0; i < 2; ++i) aoff[i] = (unsigned)(((srow + 64 * i) * g.lda + kq) * 4);
  }

  const int G = g.K >> 3;  // 8-k groups
  const unsigned* wb = g.w + ((size_t)((n0 >> 5) + wave) * G) * 512 + lane * 4;

  // every load is unconditional (no branches in the loop body, so the waitcnts stay exact): the
  // prefetches past the last chunk / weight group reload the last one (never used), so no read
  // leaves the caller's rows: a row's k < K only, and the last row of a column-offset A (a_off
  // + K <= lda) ends inside the tensor
  const int nch = g.K / KC;  // even (K % 32 == 0)
  f32x4 ra[2][2];  // A chunks c + 1 and c + 2 in flight (2 float4 per thread per chunk)
  f32x4 rq[GA ? 2 : 1][2];  // GA: the second table's rows
  auto load_a = [&](int c, int s) {
    c = min(c, nch - 1);
#pragma unroll
    for (int i = 0; i < 2; ++i) {
      ra[s][i] = __builtin_bit_cast(
          f32x4, __builtin_amdgcn_raw_buffer_load_b128(rsA, aoff[i] + (unsigned)(c * KC * 4), 0, 0));
      if constexpr (GA)
        rq[s][i] = __builtin_bit_cast(
            f32x4, __builtin_amdgcn_raw_buffer_load_b128(rsA2, aoff2[i] + (unsigned)(c * KC * 4), 0, 0));
    }
  };
  auto store_a = [&](int s) {
    unsigned* d = smem + s * BM * PX;
#pragma unroll
    for (int i = 0; i < 2; ++i) {
      gx_u32x4 q0, q1, q2;
      f32x4 x = ra[s][i];
      if constexpr (GA) {
        x += rq[s][i];
#pragma unroll
        for (int e = 0; e < 4; ++e) x[e] = fmaxf(x[e], 0.f);
      }
      gx_split(x, q0, q1, q2);
      unsigned* p = d + (srow + 64 * i) * PX + 3 * kq;
      *reinterpret_cast<gx_u32x4*>(p) = q0;
      *reinterpret_cast<gx_u32x4*>(p + 4) = q1;
      *reinterpret_cast<gx_u32x4*>(p + 8) = q2;
    }
  };
  gx_u32x4 wr[4][2];  // weight quads of 4 groups (ring): [h h | l l]-paired P0 and [m m | h h] P1
  auto load_w = [&](int gi, int s) {
    const unsigned* p = wb + (size_t)min(gi, G - 1) * 512;
    wr[s][0] = *reinterpret_cast<const gx_u32x4*>(p);
    wr[s][1] = *reinterpret_cast<const gx_u32x4*>(p + 256);
  };

  f32x16 acc[4];
#pragma unroll
  for (int i = 0; i < 4; ++i)
#pragma unroll
    for (int r = 0; r < 16; ++r) acc[i][r] = 0.f;
  // a group's activation operands: 4 row blocks x the quads [h h] [h m] [m l], each one
  // ds_read_b128 (no register shuffles); read one group ahead of its MFMAs
  typedef gx_u32x4 Frag[4][3];
  auto read_frag = [&](int buf, int gl, Frag& f) {
    const unsigned* As = smem + buf * BM * PX;
#pragma unroll
    for (int i = 0; i < 4; ++i) {
      const unsigned* p = As + (i * 32 + frow) * PX + 12 * (2 * gl + fh);
#pragma unroll
      for (int q = 0; q < 3; ++q) f[i][q] = *reinterpret_cast<const gx_u32x4*>(p + 4 * q);
    }
  };
  auto mma = [&](const Frag& f, int s) {
    const gx_bf16x8 p0 = gx_op(wr[s][0]), p1 = gx_op(wr[s][1]);
#pragma unroll
    for (int i = 0; i < 4; ++i) {
      acc[i] = __builtin_amdgcn_mfma_f32_32x32x16_bf16(gx_op(f[i][0]), p0, acc[i], 0, 0, 0);  // hh + hl
      acc[i] = __builtin_amdgcn_mfma_f32_32x32x16_bf16(gx_op(f[i][1]), p1, acc[i], 0, 0, 0);  // hm + mh
      acc[i] = __builtin_amdgcn_mfma_f32_32x32x16_bf16(gx_op(f[i][2]), p1, acc[i], 0, 0, 0);  // mm + lh
    }
  };

  // Schedule per chunk c (2 groups, LDS buffer c & 1, weight slots 2(c & 1), 2(c & 1) + 1):
  //   phase 1: read group 1 (12 ds_read_b128) | MFMAs of group 0, with the split of chunk c + 1
  //            (~64 VALU) and its 6 ds_write_b128 into the other buffer (whose last readers,
  //            chunk c - 1, all read before this chunk's barrier) in the MFMA gaps;
  //   barrier;
  //   phase 2: read group 0 of chunk c + 1 | MFMAs of group 1.
  // sched_barrier(0) pins the phases, so every LDS read is a whole group ahead of its MFMAs and
  // the split VALU hides under MFMAs instead of serialising with them.
  static_assert(NG == 2, "the chunk schedule below is written for 2 groups per chunk");
  Frag fa, fb;
  load_a(0, 0);
  load_a(1, 1);
  load_w(0, 0);
  load_w(1, 1);
  store_a(0);
  __syncthreads();
  load_a(2, 0);
  read_frag(0, 0, fa);
  for (int c = 0; c < nch; c += 2) {
#pragma unroll
    for (int h = 0; h < 2; ++h) {  // chunk c + h
      const int gi = (c + h) * NG;
      __builtin_amdgcn_sched_barrier(0);
      load_w(gi + 2, (2 * h + 2) & 3);
      read_frag(h, 1, fb);
      store_a(1 - h);  // chunk c + h + 1 (a reloaded last chunk past the end: unused)
      mma(fa, 2 * h);
      __builtin_amdgcn_sched_group_barrier(0x020, 2, 0);   // weight loads
      __builtin_amdgcn_sched_group_barrier(0x100, 12, 0);  // DS reads
#pragma unroll
      for (int q = 0; q < 12; ++q) {
        __builtin_amdgcn_sched_group_barrier(0x008, 1, 0);  // MFMA
        __builtin_amdgcn_sched_group_barrier(0x002, 6, 0);  // VALU
        if (q < 6) __builtin_amdgcn_sched_group_barrier(0x200, 1, 0);  // DS write
      }
      __builtin_amdgcn_sched_barrier(0);
      __syncthreads();
      load_a(c + h + 3, 1 - h);
      load_w(gi + 3, (2 * h + 3) & 3);
      read_frag(1 - h, 0, fa);
      __builtin_amdgcn_sched_barrier(0);
      mma(fb, 2 * h + 1);
    }
  }
  __builtin_amdgcn_sched_barrier(0);

  // ---- epilogue: lane = column n, accumulator element r = row (r & 3) + 8 (r >> 2) + 4 fh. Each
  // 32 x 32 tile goes through this wave's LDS slot (the staging buffers are free now) and comes back
  // as 8 lanes per row: one float4 store per lane and 8 rows, whole 128-B row segments, instead of
  // 16 scalar stores per lane and tile (without any stores the family took 14 % less time) ---------
  __syncthreads();  // every wave's last reads of the staging buffers are done
  constexpr int TP = 36;  // slot pitch (floats)
  float* const ts = reinterpret_cast<float*>(smem) + wave * (32 * TP);
  const int trow = lane >> 3, tcol = 4 * (lane & 7);
  const int nq = n0 + wave * 32 + tcol;  // this lane's 4 output columns
  float bq[4];
#pragma unroll
  for (int e = 0; e < 4; ++e) bq[e] = g.bias ? g.bias[nq + e] : 0.f;
  float* ob = g.out + grp * g.o_grp + nq;
  const float* rb = g.res ? g.res + grp * g.r_grp + nq : nullptr;  // ldr = 0: one row per group
#pragma unroll
  for (int i = 0; i < 4; ++i) {
#pragma unroll
    for (int r = 0; r < 16; ++r) ts[((r & 3) + 8 * (r >> 2) + 4 * fh) * TP + frow] = acc[i][r];
    __builtin_amdgcn_wave_barrier();
    f32x4 tv[4];
#pragma unroll
    for (int j = 0; j < 4; ++j) tv[j] = *reinterpret_cast<const f32x4*>(ts + (8 * j + trow) * TP + tcol);
    __builtin_amdgcn_wave_barrier();  // the next tile's writes stay after these reads
#pragma unroll
    for (int j = 0; j < 4; ++j) {
      const int m = m0 + i * 32 + 8 * j + trow;
      if (m >= g.M) continue;
      f32x4 v = tv[j];
#pragma unroll
      for (int e = 0; e < 4; ++e) {
        v[e] += bq[e];
        if (rb) v[e] += rb[(size_t)m * g.ldr + e];
        if (g.relu) v[e] = fmaxf(v[e], 0.f);
      }
      *reinterpret_cast<f32x4*>(ob + (size_t)m * g.ldo) = v;
    }
  }
}

}  // namespace

KRRN_API int krrn_gemm_x3_f32(const float* a, int lda, int M, int K, int N, const void* w3f, const float* bias,
                              const float* res, int ldr, float* out, int ldo, int relu, int batch, long long a_grp,
                              long long o_grp, long long r_grp, void* stream) {
  if (!a || !w3f || !out) return KRRN_EARG;
  if (M < 1 || K < KC || N < BN || batch < 1) return KRRN_ESHAPE;
  if ((K % (2 * KC)) || (N % BN) || lda < K || ldo < N) return KRRN_ESHAPE;
  if ((lda & 3) || (ldo & 3) || (a_grp & 3) || (o_grp & 3)) return KRRN_EALIGN;
  if (res && ((ldr != 0 && ldr < N) || (r_grp & 3))) return KRRN_ESHAPE;
  if (!krrn_aligned16(a) || !krrn_aligned16(w3f) || !krrn_aligned16(out)) return KRRN_EALIGN;
  if ((long long)BM * lda * 4 >= 0x7FFFFFFFLL) return KRRN_ESHAPE;  // 32-bit buffer offsets
  const long long tiles = (long long)krrn_cdiv(M, BM) * (N / BN) * batch;
  if (tiles > 0x7FFFFFFFLL) return KRRN_ESHAPE;
  GemmArgs g;
  g.a = a; g.a2 = nullptr; g.ia = g.ib = nullptr; g.a2_grp = 0; g.lda2 = 0; g.npts = 1;
  g.w = reinterpret_cast<const unsigned*>(w3f); g.bias = bias; g.res = res; g.out = out;
  g.lda = lda; g.M = M; g.K = K; g.N = N; g.ldr = ldr; g.ldo = ldo; g.relu = relu;
  g.a_grp = a_grp; g.o_grp = o_grp; g.r_grp = r_grp;
  g.mt = krrn_cdiv(M, BM); g.nt = N / BN; g.total = (int)tiles;
  hipLaunchKernelGGL(gemm_x3_kernel<false>, dim3((unsigned)tiles), dim3(256), 0, (hipStream_t)stream, g);
  return krrn_launch_status();
}

KRRN_API int krrn_gemm_x3_gather_f32(const int* ia, const float* A, long long a_bs, int a_st, const int* ib,
                                     const float* A2, long long a2_bs, int a2_st, int npts, int B, int K, int N,
                                     const void* w3f, const float* bias, float* out, int ldo, int relu,
                                     void* stream) {
  if (!ia || !A || !ib || !A2 || !w3f || !out) return KRRN_EARG;
  if (npts < 1 || B < 1 || K < KC || N < BN) return KRRN_ESHAPE;
  if ((K % (2 * KC)) || (N % BN) || a_st < K || a2_st < K || ldo < N) return KRRN_ESHAPE;
  if ((a_st & 3) || (a2_st & 3) || (a_bs & 3) || (a2_bs & 3) || (ldo & 3)) return KRRN_EALIGN;
  if (!krrn_aligned16(A) || !krrn_aligned16(A2) || !krrn_aligned16(w3f) || !krrn_aligned16(out)) return KRRN_EALIGN;
  // 32-bit buffer offsets over the whole row tables; the kernel trusts ia / ib to index rows of
  // their crop's table (a_bs / a_st floats), as krrn_gather2_add_f32 does
  if ((long long)B * a_bs * 4 >= 0x7FFFFFFFLL || (long long)B * a2_bs * 4 >= 0x7FFFFFFFLL) return KRRN_ESHAPE;
  const long long M = (long long)B * npts;
  const long long tiles = (long long)krrn_cdiv(M, BM) * (N / BN);
  if (M > 0x7FFFFFFFLL || tiles > 0x7FFFFFFFLL) return KRRN_ESHAPE;
  GemmArgs g;
  g.a = A; g.a2 = A2; g.ia = ia; g.ib = ib; g.a_grp = a_bs; g.a2_grp = a2_bs; g.lda = a_st; g.lda2 = a2_st;
  g.npts = npts;
  g.w = reinterpret_cast<const unsigned*>(w3f); g.bias = bias; g.res = nullptr; g.out = out;
  g.M = (int)M; g.K = K; g.N = N; g.ldr = 0; g.ldo = ldo; g.relu = relu;
  g.o_grp = 0; g.r_grp = 0;
  g.mt = krrn_cdiv(g.M, BM); g.nt = N / BN; g.total = (int)tiles;
  hipLaunchKernelGGL(gemm_x3_kernel<true>, dim3((unsigned)tiles), dim3(256), 0, (hipStream_t)stream, g);
  return krrn_launch_status();
}
