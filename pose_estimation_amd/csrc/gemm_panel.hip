// Short-K GEMM (K = 64 / 128) streaming its output: the fusion's level-0 / level-1 GCN
// `feature_map @ weights + bias` of Conv_layer (lib/network/point/gcn3d.py:136-164, SURVEY §8a G6:
// M = B*N points, K = 128, N = (support_num + 1) * 128 = 1024 columns).
//
//   out[m, n] = act( sum_k A[m, k] W[n, k] + bias[n] + res[m, n] )       (scale folded into W)
//
// The output (262 MB at B = 64, N = 1000, per branch) is 8x the input, so the kernel is a write
// stream with 128 k of f32-accurate matrix work per output element: split-bf16 operands (x = h + m
// + l, the three bf16 terms of gemm_x3.hip) on v_mfma_f32_32x32x16_bf16, six term products per f32
// product. Layout (MI355X-first, "A-stationary"):
//   * a wave owns 32 rows for the whole launch: it loads its 32 x K activation panel once (one
//     float4 per lane per 8-k group), splits it into two MFMA operand quads per group, [h m] and
//     [h l], and keeps them in VGPRs (K = 128: 128 registers) while it walks its column tiles;
//   * per 32-column tile and 8-k group the weights are three host-split quads [h m] [m h] [l h]
//     (ops.gemm_weights_panel), one fully coalesced 1-KB wave load each, read from L1 / L2 (the four
//     waves of a block walk the same tiles): [h m]x[h m] = hh + mm, [h m]x[m h] = hm + mh,
//     [h l]x[l h] = hl + lh -- three MFMAs per 8 k, no LDS and no barrier anywhere;
//   * the 32x32 accumulator of a tile is stored as it stands (one register = two 128-B row
//     segments), bias / residual / ReLU fused; two waves per SIMD overlap one wave's store tail
//     with the other's MFMAs.
// The row panels of a launch split into `csplit` column ranges when the panels alone cannot fill
// the chip (level 1: M = 16000 -> 125 panels x 4 column ranges).
#include "krrn_common.h"

namespace {

typedef __bf16 gp_bf16x8 __attribute__((ext_vector_type(8)));
typedef __bf16 gp_bf16x2 __attribute__((ext_vector_type(2)));
typedef float gp_f32x2 __attribute__((ext_vector_type(2)));
typedef unsigned gp_u32x4 __attribute__((ext_vector_type(4)));

struct PanelArgs {
  const float* a;
  const unsigned* w;  // [N/32][K/8][3][64][4] u32
  const float* bias;
  const float* res;
  float* out;
  int lda, M, N, ldr, ldo, relu;
  int ntile_per_split;  // column tiles (32 wide) per blockIdx.y
};

__device__ __forceinline__ unsigned gp_pk(float a, float b) {
  return __builtin_bit_cast(unsigned, __builtin_convertvector(gp_f32x2{a, b}, gp_bf16x2));  // RNE
}

__device__ __forceinline__ gp_bf16x8 gp_op(const gp_u32x4 v) { return __builtin_bit_cast(gp_bf16x8, v); }

template <int KT>
__global__ __launch_bounds__(256, 2) void gemm_panel_x3_kernel(const PanelArgs g) {
  constexpr int G = KT / 8;  // 8-k groups
  const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
  const int nl = lane & 31, fh = lane >> 5;
  const int m0 = blockIdx.x * 128 + wave * 32;
  if (m0 >= g.M) return;  // whole idle waves only (no barrier in this kernel)

  // ---- the wave's activation panel: row m0 + nl, k = 8 gi + 4 fh .. + 3 of every group ------
  gp_u32x4 qa[G][2];  // [h m] and [h l] per group
  {
    const int row = m0 + nl;
    const float* ap = g.a + (size_t)row * g.lda + 4 * fh;
    f32x4 x[G];
#pragma unroll
    for (int gi = 0; gi < G; ++gi)
      x[gi] = row < g.M ? *reinterpret_cast<const f32x4*>(ap + 8 * gi) : f32x4{0.f, 0.f, 0.f, 0.f};
#pragma unroll
    for (int gi = 0; gi < G; ++gi) {
      const f32x4 v = x[gi];
      const unsigned h0 = gp_pk(v[0], v[1]), h1 = gp_pk(v[2], v[3]);
      const float r0 = v[0] - __builtin_bit_cast(float, h0 << 16), r1 = v[1] - __builtin_bit_cast(float, h0 & 0xFFFF0000u);
      const float r2 = v[2] - __builtin_bit_cast(float, h1 << 16), r3 = v[3] - __builtin_bit_cast(float, h1 & 0xFFFF0000u);
      const unsigned mm0 = gp_pk(r0, r1), mm1 = gp_pk(r2, r3);
      const unsigned l0 = gp_pk(r0 - __builtin_bit_cast(float, mm0 << 16), r1 - __builtin_bit_cast(float, mm0 & 0xFFFF0000u));
      const unsigned l1 = gp_pk(r2 - __builtin_bit_cast(float, mm1 << 16), r3 - __builtin_bit_cast(float, mm1 & 0xFFFF0000u));
      qa[gi][0] = gp_u32x4{h0, h1, mm0, mm1};
      qa[gi][1] = gp_u32x4{h0, h1, l0, l1};
    }
  }

  const int ct0 = blockIdx.y * g.ntile_per_split;
  const int ct1 = min(ct0 + g.ntile_per_split, g.N >> 5);
  // rows of accumulator element r: (r & 3) + 8 (r >> 2) + 4 fh
  for (int ct = ct0; ct < ct1; ++ct) {
    const unsigned* wp = g.w + (size_t)ct * G * 768 + lane * 4;
    f32x16 acc;
#pragma unroll
    for (int r = 0; r < 16; ++r) acc[r] = 0.f;
#pragma unroll
    for (int gi = 0; gi < G; ++gi) {
      const gp_u32x4 b0 = *reinterpret_cast<const gp_u32x4*>(wp + gi * 768);
      const gp_u32x4 b1 = *reinterpret_cast<const gp_u32x4*>(wp + gi * 768 + 256);
      const gp_u32x4 b2 = *reinterpret_cast<const gp_u32x4*>(wp + gi * 768 + 512);
      acc = __builtin_amdgcn_mfma_f32_32x32x16_bf16(gp_op(qa[gi][0]), gp_op(b0), acc, 0, 0, 0);  // hh + mm
      acc = __builtin_amdgcn_mfma_f32_32x32x16_bf16(gp_op(qa[gi][0]), gp_op(b1), acc, 0, 0, 0);  // hm + mh
      acc = __builtin_amdgcn_mfma_f32_32x32x16_bf16(gp_op(qa[gi][1]), gp_op(b2), acc, 0, 0, 0);  // hl + lh
    }
    const int n = ct * 32 + nl;
    const float bi = g.bias ? g.bias[n] : 0.f;
    float* ob = g.out + (size_t)m0 * g.ldo + n;
    const float* rb = g.res ? g.res + (size_t)m0 * g.ldr + n : nullptr;
#pragma unroll
    for (int r = 0; r < 16; ++r) {
      const int mr = (r & 3) + 8 * (r >> 2) + 4 * fh;
      if (m0 + mr >= g.M) continue;
      float v = acc[r] + bi;
      if (rb) v += rb[(size_t)mr * g.ldr];
      if (g.relu) v = fmaxf(v, 0.f);
      ob[(size_t)mr * g.ldo] = v;
    }
  }
}

}  // namespace

KRRN_API int krrn_gemm_panel_x3_f32(const float* a, int lda, int M, int K, int N, const void* wpf, const float* bias,
                                    const float* res, int ldr, float* out, int ldo, int relu, int csplit,
                                    void* stream) {
  if (!a || !wpf || !out) return KRRN_EARG;
  if (M < 1 || (K != 64 && K != 128) || N < 32 || (N & 31) || csplit < 1) return KRRN_ESHAPE;
  if (lda < K || ldo < N || (res && ldr < N)) return KRRN_ESHAPE;
  if ((lda & 3) || !krrn_aligned16(a) || !krrn_aligned16(wpf)) return KRRN_EALIGN;
  const int ntiles = N >> 5;
  const int per = krrn_cdiv(ntiles, csplit);
  PanelArgs g;
  g.a = a; g.w = reinterpret_cast<const unsigned*>(wpf); g.bias = bias; g.res = res; g.out = out;
  g.lda = lda; g.M = M; g.N = N; g.ldr = ldr; g.ldo = ldo; g.relu = relu;
  g.ntile_per_split = per;
  const dim3 grid((unsigned)krrn_cdiv(M, 128), (unsigned)krrn_cdiv(ntiles, per));
  hipStream_t s = (hipStream_t)stream;
  if (K == 128)
    hipLaunchKernelGGL(gemm_panel_x3_kernel<128>, grid, dim3(256), 0, s, g);
  else
    hipLaunchKernelGGL(gemm_panel_x3_kernel<64>, grid, dim3(256), 0, s, g);
  return krrn_launch_status();
}
