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
#include <stdlib.h>

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

// The same GEMM with the weight tiles shared through LDS: a block of 8 waves owns 256 rows (each wave
// its 32-row register panel as above) and walks the column tiles together; each 32-column tile's
// three split quads per 8-k group (48 KB at K = 128) are staged into a double-buffered LDS ring by
// all 512 threads (6 b128 global loads each, issued one tile ahead, written after the tile's MFMAs),
// then read by every wave with ds_read_b128 -- one L2 read of the weights per 256 rows instead of one
// per 32 rows per wave (the register-only form above re-streamed 768 KB of fragments per wave from
// L2: 3 GB per level-0 launch). One barrier per tile; 96 KB LDS, 2 waves per SIMD.
template <int KT, bool RES, int DIAG = 0>  // DIAG (measurements only): 1 = no MFMAs, 2 = no output stores
__global__ __launch_bounds__(512, 1) void gemm_plds_x3_kernel(const PanelArgs g) {
  constexpr int G = KT / 8;
  constexpr int TILE_U32 = G * 3 * 256;  // one 32-column tile of split fragments
  constexpr int PIECES = TILE_U32 / 4 / 512;
  static_assert(PIECES * 4 * 512 == TILE_U32, "tile staging");
  __shared__ __attribute__((aligned(16))) unsigned sb[2][TILE_U32];
  const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
  const int nl = lane & 31, fh = lane >> 5;
  const int m0 = blockIdx.x * 256 + wave * 32;

  // ---- the wave's activation panel (rows past M are zero; every wave stays for the barriers) ----
  gp_u32x4 qa[G][2];
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
  gp_u32x4 stg[PIECES];
  auto load_tile = [&](int ct) {
    const gp_u32x4* src = reinterpret_cast<const gp_u32x4*>(g.w + (size_t)ct * TILE_U32);
#pragma unroll
    for (int i = 0; i < PIECES; ++i) stg[i] = src[tid + i * 512];
  };
  auto store_tile = [&](int buf) {
    gp_u32x4* dst = reinterpret_cast<gp_u32x4*>(sb[buf]);
#pragma unroll
    for (int i = 0; i < PIECES; ++i) dst[tid + i * 512] = stg[i];
  };
  if (ct0 < ct1) {
    load_tile(ct0);
    store_tile(0);
  }
  __syncthreads();
  const bool live = m0 < g.M;
  // software pipeline: tile ct's 48 MFMAs issue while tile ct - 1's accumulator is stored (its 16
  // stores + bias adds sit in the MFMA gaps, one per 8-k group), so the matrix pipe and the write
  // stream overlap inside every wave (with one barrier per tile, the 8 waves of the block otherwise
  // alternate MFMA and store phases in lockstep)
  // the previous tile's output column pointer and bias, so its epilogue reads no global memory
  float* obp = g.out + (size_t)m0 * g.ldo + ct0 * 32 + nl;
  float bip = 0.f;
  const int rows_left = g.M - m0;
  auto epilogue = [&](const f32x16& acc, int r) {
    const int mr = (r & 3) + 8 * (r >> 2) + 4 * fh;
    if (mr >= rows_left) return;
    float v = acc[r] + bip;
    if constexpr (RES) v += g.res[(obp - g.out) + (size_t)mr * g.ldr - (size_t)m0 * (g.ldo - g.ldr)];
    if (g.relu) v = fmaxf(v, 0.f);
    obp[(size_t)mr * g.ldo] = v;
  };
  f32x16 accp;
#pragma unroll
  for (int r = 0; r < 16; ++r) accp[r] = 0.f;
  for (int ct = ct0; ct <= ct1; ++ct) {
    const int buf = (ct - ct0) & 1;
    const bool has = ct < ct1;
    const float bi_cur = (has && g.bias) ? g.bias[ct * 32 + nl] : 0.f;
    if (ct + 1 < ct1) load_tile(ct + 1);  // in flight under this tile's MFMAs
    f32x16 acc;
#pragma unroll
    for (int r = 0; r < 16; ++r) acc[r] = 0.f;
    const unsigned* bp = sb[buf] + lane * 4;
#pragma unroll
    for (int gi = 0; gi < G; ++gi) {
      if (live && has && DIAG != 1) {
        const gp_u32x4 b0 = *reinterpret_cast<const gp_u32x4*>(bp + gi * 768);
        const gp_u32x4 b1 = *reinterpret_cast<const gp_u32x4*>(bp + gi * 768 + 256);
        const gp_u32x4 b2 = *reinterpret_cast<const gp_u32x4*>(bp + gi * 768 + 512);
        acc = __builtin_amdgcn_mfma_f32_32x32x16_bf16(gp_op(qa[gi][0]), gp_op(b0), acc, 0, 0, 0);  // hh + mm
        acc = __builtin_amdgcn_mfma_f32_32x32x16_bf16(gp_op(qa[gi][0]), gp_op(b1), acc, 0, 0, 0);  // hm + mh
        acc = __builtin_amdgcn_mfma_f32_32x32x16_bf16(gp_op(qa[gi][1]), gp_op(b2), acc, 0, 0, 0);  // hl + lh
      }
      if (live && ct > ct0 && DIAG != 2) {
        // the previous tile's rows, G of its 16 accumulator registers per... spread over the groups
#pragma unroll
        for (int r = gi * 16 / G; r < (gi + 1) * 16 / G; ++r) epilogue(accp, r);
      }
    }
    if (DIAG == 2 && live) {
      float sum = 0.f;
#pragma unroll
      for (int r = 0; r < 16; ++r) sum += acc[r];
      if (sum == 1234.5f) g.out[0] = sum;  // keeps the MFMAs alive
    }
    accp = acc;
    if (ct > ct0) obp += 32;
    bip = bi_cur;
    if (ct + 1 < ct1) store_tile(buf ^ 1);  // its last readers (tile ct - 1) passed the previous barrier
    __syncthreads();
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
  hipStream_t s = (hipStream_t)stream;
  static const int form = [] {
    const char* e = getenv("KRRN_PANEL_FORM");  // 0: register-only form (diagnostics)
    return e ? atoi(e) : 1;
  }();
  if (form >= 1) {
    const dim3 grid((unsigned)krrn_cdiv(M, 256), (unsigned)krrn_cdiv(ntiles, per));
    if (K == 128 && !res) {
      if (form == 2) hipLaunchKernelGGL((gemm_plds_x3_kernel<128, false, 1>), grid, dim3(512), 0, s, g);
      else if (form == 3) hipLaunchKernelGGL((gemm_plds_x3_kernel<128, false, 2>), grid, dim3(512), 0, s, g);
      else hipLaunchKernelGGL((gemm_plds_x3_kernel<128, false, 0>), grid, dim3(512), 0, s, g);
    } else if (K == 128) {
      // a residual at K = 128 does not fit the LDS form's register budget; the register-only form
      // that has room for it gave gather-conv outputs differing from the serial run beside the
      // gather-conv and stays a diagnostic (KRRN_PANEL_FORM=0)
      return KRRN_EUNSUPPORTED;
    } else if (res) {
      hipLaunchKernelGGL((gemm_plds_x3_kernel<64, true, 0>), grid, dim3(512), 0, s, g);
    } else {
      hipLaunchKernelGGL((gemm_plds_x3_kernel<64, false, 0>), grid, dim3(512), 0, s, g);
    }
    return krrn_launch_status();
  }
  const dim3 grid((unsigned)krrn_cdiv(M, 128), (unsigned)krrn_cdiv(ntiles, per));
  if (K == 128)
    hipLaunchKernelGGL(gemm_panel_x3_kernel<128>, grid, dim3(256), 0, s, g);
  else
    hipLaunchKernelGGL(gemm_panel_x3_kernel<64>, grid, dim3(256), 0, s, g);
  return krrn_launch_status();
}
