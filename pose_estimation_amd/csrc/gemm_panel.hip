// Short-K GEMM (K = 64 / 128) streaming its output: the fusion's level-0 / level-1 GCN
// `feature_map @ weights + bias` of Conv_layer (lib/network/point/gcn3d.py:136-164, SURVEY §8a G6:
// M = B*N points, K = 128, N = (support_num + 1) * 128 = 1024 columns) and layer1's 64 -> 256 1x1
// convs (myhrnet.py:65-103, K = 64, with the residual).
//
//   out[m, n] = act( sum_k A[m, k] W[n, k] + bias[n] + res[m, n] )       (scale folded into W)
//
// The output (262 MB at B = 64, N = 1000, per branch) is 8x the input, so the kernel is a write
// stream with 128 k of f32-accurate matrix work per output element: split-bf16 operands (x = h + m
// + l, the three bf16 terms of gemm_x3.hip) on v_mfma_f32_32x32x16_bf16, six term products per f32
// product. Layout (MI355X-first, "A-stationary"):
//   * a block of 8 waves owns 256 rows; a wave loads its 32 x K activation panel once (one float4
//     per lane per 8-k group), splits it into two MFMA operand quads per group, [h m] and [h l], and
//     keeps them in VGPRs (K = 128: 128 registers) while the block walks its column tiles;
//   * per 32-column tile the three host-split weight quads per 8-k group ([h m] [m h] [l h],
//     ops.gemm_weights_panel; 48 KB at K = 128) are staged into a double-buffered LDS ring by all 512
//     threads one tile ahead, then read by every wave with ds_read_b128 (one L2 read of the weights per
//     256 rows): [h m]x[h m] = hh + mm, [h m]x[m h] = hm + mh, [h l]x[l h] = hl + lh -- three MFMAs per
//     8 k, one barrier per tile; 96 KB LDS, 2 waves per SIMD;
//   * the previous tile's accumulator is stored in the current tile's MFMA gaps as 4 float4 per lane
//     (operands swapped so a lane holds 4 consecutive columns), bias / residual / ReLU fused.
// The row panels of a launch split into `csplit` column ranges when the panels alone cannot fill
// the chip (level 1: M = 16000 -> 63 panels x 4 column ranges).
#include "krrn_common.h"

namespace {

constexpr int kPanelMaxN = 2048;  // columns whose bias a block stages in LDS (gemm_pdma_x3_kernel)

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
  int vec;              // float4 epilogue: out / res / bias 16-B aligned, ldo / ldr % 4 == 0
};

__device__ __forceinline__ unsigned gp_pk(float a, float b) {
  return __builtin_bit_cast(unsigned, __builtin_convertvector(gp_f32x2{a, b}, gp_bf16x2));  // RNE
}

__device__ __forceinline__ gp_bf16x8 gp_op(const gp_u32x4 v) { return __builtin_bit_cast(gp_bf16x8, v); }

// (The round-3 register-only form without the LDS ring re-streamed 768 KB of weight fragments per
// wave from L2, 3 GB per level-0 launch, and was removed in round 4.)
typedef unsigned gp_u32x8 __attribute__((ext_vector_type(8)));
typedef unsigned gp_u32x2 __attribute__((ext_vector_type(2)));
__device__ __forceinline__ gp_bf16x8 gp_sub4(const gp_u32x8& c, int o) {
  return __builtin_bit_cast(gp_bf16x8, gp_u32x4{c[o], c[o + 1], c[o + 2], c[o + 3]});
}

// CH (chain layout, KRRN_PANEL_CHAIN): per 8-k group the weights are one [m h] quad + one [l] pair
// per lane (ops.gemm_weights_panel_chain: 24 B instead of the three quads' 48 B), the activations a
// register chain [h h m l]; the MFMAs take register slices, W[2:5] x A[0:3] = hh + lh,
// W[0:3] x A[2:5] = mh + hm, W[0:3] x A[4:7] = mm + hl -- half the LDS bytes per MFMA.
template <int KT, bool RES, int DIAG = 0, bool CH = false>  // DIAG (measurements only): 1 = no MFMAs, 2 = no stores
__global__ __launch_bounds__(512, 1) void gemm_plds_x3_kernel(const PanelArgs g) {
  constexpr int G = KT / 8;
  constexpr int GU32 = CH ? 384 : 768;   // u32 per 8-k group of one 32-column tile
  constexpr int TILE_U32 = G * GU32;     // one 32-column tile of split fragments
  constexpr int P4 = TILE_U32 / 4;       // 16-B pieces per tile
  constexpr int PIECES = (P4 + 511) / 512;
  __shared__ __attribute__((aligned(16))) unsigned sb[2][TILE_U32];
  const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
  const int nl = lane & 31, fh = lane >> 5;
  const int m0 = blockIdx.x * 256 + wave * 32;

  // ---- the wave's activation panel (rows past M are zero; every wave stays for the barriers) ----
  gp_u32x4 qa[CH ? 1 : G][2];
  gp_u32x8 ca[CH ? G : 1];
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
      if constexpr (CH) {
        ca[gi] = gp_u32x8{h0, h1, h0, h1, mm0, mm1, l0, l1};
      } else {
        qa[gi][0] = gp_u32x4{h0, h1, mm0, mm1};
        qa[gi][1] = gp_u32x4{h0, h1, l0, l1};
      }
    }
  }

  const int ct0 = blockIdx.y * g.ntile_per_split;
  const int ct1 = min(ct0 + g.ntile_per_split, g.N >> 5);
  gp_u32x4 stg[PIECES];
  auto load_tile = [&](int ct) {
    const gp_u32x4* src = reinterpret_cast<const gp_u32x4*>(g.w + (size_t)ct * TILE_U32);
#pragma unroll
    for (int i = 0; i < PIECES; ++i)
      if (P4 % 512 == 0 || tid + i * 512 < P4) stg[i] = src[tid + i * 512];
  };
  auto store_tile = [&](int buf) {
    gp_u32x4* dst = reinterpret_cast<gp_u32x4*>(sb[buf]);
#pragma unroll
    for (int i = 0; i < PIECES; ++i)
      if (P4 % 512 == 0 || tid + i * 512 < P4) dst[tid + i * 512] = stg[i];
  };
  if (ct0 < ct1) {
    load_tile(ct0);
    store_tile(0);
  }
  __syncthreads();
  const bool live = m0 < g.M;
  // software pipeline: tile ct's 48 MFMAs issue while tile ct - 1's accumulator is stored (its
  // stores + bias adds sit in the MFMA gaps), so the matrix pipe and the write stream overlap inside
  // every wave (with one barrier per tile, the 8 waves of the block otherwise alternate MFMA and
  // store phases in lockstep).
  // Operands swapped (weights as the MFMA's A, activations as B: D = (A W^T)^T, the same products):
  // lane l then holds output row m0 + l % 32 and, in accumulator registers 4q .. 4q + 3, the 4
  // consecutive columns 8q + 4 (l / 32) .. + 3 of the tile -- the epilogue is 4 float4 stores per lane
  // and tile (each wave-instruction 1 KB) instead of 16 dword stores (256 B each): the store issue,
  // not the bytes, had paced the write stream (MI355X_MICROARCH.md: epilogue store tails)
  const int rows_left = g.M - m0;
  const int mrow = nl;  // this lane's output row in the wave's panel
  float* orow = g.out + (size_t)(m0 + mrow) * g.ldo;
  const float* rrow = RES ? g.res + (size_t)(m0 + mrow) * g.ldr : nullptr;
  const bool row_ok = mrow < rows_left;
  auto epilogue = [&](const f32x16& acc, int ctp, int q) {
    if (!row_ok) return;
    const int n = ctp * 32 + 8 * q + 4 * fh;
    f32x4 v = {acc[4 * q], acc[4 * q + 1], acc[4 * q + 2], acc[4 * q + 3]};
    if (g.vec) {
      if (g.bias) v += *reinterpret_cast<const f32x4*>(g.bias + n);
      if constexpr (RES) v += *reinterpret_cast<const f32x4*>(rrow + n);
      if (g.relu) {
#pragma unroll
        for (int e = 0; e < 4; ++e) v[e] = fmaxf(v[e], 0.f);
      }
      *reinterpret_cast<f32x4*>(orow + n) = v;
    } else {
#pragma unroll
      for (int e = 0; e < 4; ++e) {
        float x = v[e] + (g.bias ? g.bias[n + e] : 0.f);
        if constexpr (RES) x += rrow[n + e];
        if (g.relu) x = fmaxf(x, 0.f);
        orow[n + e] = x;
      }
    }
  };
  f32x16 accp;
#pragma unroll
  for (int r = 0; r < 16; ++r) accp[r] = 0.f;
  for (int ct = ct0; ct <= ct1; ++ct) {
    const int buf = (ct - ct0) & 1;
    const bool has = ct < ct1;
    if (ct + 1 < ct1) load_tile(ct + 1);  // in flight under this tile's MFMAs
    f32x16 acc;
#pragma unroll
    for (int r = 0; r < 16; ++r) acc[r] = 0.f;
    const unsigned* bp = sb[buf] + lane * 4;
#pragma unroll
    for (int gi = 0; gi < G; ++gi) {
      if (live && has && DIAG != 1) {
        if constexpr (CH) {
          const gp_u32x4 mh = *reinterpret_cast<const gp_u32x4*>(bp + gi * 384);
          const unsigned* lp = sb[buf] + gi * 384 + 256 + lane * 2;
          const gp_u32x8 wc = {mh[0], mh[1], mh[2], mh[3], lp[0], lp[1], 0u, 0u};  // [m h l]
          acc = __builtin_amdgcn_mfma_f32_32x32x16_bf16(gp_sub4(wc, 2), gp_sub4(ca[gi], 0), acc, 0, 0, 0);  // hh + lh
          acc = __builtin_amdgcn_mfma_f32_32x32x16_bf16(gp_sub4(wc, 0), gp_sub4(ca[gi], 2), acc, 0, 0, 0);  // mh + hm
          acc = __builtin_amdgcn_mfma_f32_32x32x16_bf16(gp_sub4(wc, 0), gp_sub4(ca[gi], 4), acc, 0, 0, 0);  // mm + hl
        } else {
          const gp_u32x4 b0 = *reinterpret_cast<const gp_u32x4*>(bp + gi * 768);
          const gp_u32x4 b1 = *reinterpret_cast<const gp_u32x4*>(bp + gi * 768 + 256);
          const gp_u32x4 b2 = *reinterpret_cast<const gp_u32x4*>(bp + gi * 768 + 512);
          acc = __builtin_amdgcn_mfma_f32_32x32x16_bf16(gp_op(b0), gp_op(qa[gi][0]), acc, 0, 0, 0);  // mm + hh
          acc = __builtin_amdgcn_mfma_f32_32x32x16_bf16(gp_op(b1), gp_op(qa[gi][0]), acc, 0, 0, 0);  // mh + hm
          acc = __builtin_amdgcn_mfma_f32_32x32x16_bf16(gp_op(b2), gp_op(qa[gi][1]), acc, 0, 0, 0);  // lh + hl
        }
      }
      // the previous tile's 4 float4 stores, one every G / 4 groups
      if (live && ct > ct0 && DIAG != 2 && gi % (G / 4) == 0) epilogue(accp, ct - 1, gi / (G / 4));
    }
    if (DIAG == 2 && live) {
      float sum = 0.f;
#pragma unroll
      for (int r = 0; r < 16; ++r) sum += acc[r];
      if (sum == 1234.5f) g.out[0] = sum;  // keeps the MFMAs alive
    }
    accp = acc;
    if (ct + 1 < ct1) store_tile(buf ^ 1);  // its last readers (tile ct - 1) passed the previous barrier
    __syncthreads();
  }
}


// ---- Two blocks per CU, weights staged by LDS DMA (gemm_pdma_x3_kernel, KRRN_PANEL_DMA=1) ---------
// The 8-wave form runs one block per CU whose barrier makes every wave wait for the slowest wave's
// stores and weight staging each tile (measured at the level-0 GCN GEMM: 211 us = 105 us without the
// stores + 86 us without the MFMAs). Here a block is 4 waves / 128 rows in the chain layout (24 KB per
// weight tile, 48 KB ring + 8 KB bias), so two independent blocks share a CU and one's store / staging
// phase overlaps the other's MFMAs. The weight tile is copied global -> LDS by global_load_lds_dwordx4
// (no staging registers: each wave instruction moves 1 KB), the bias sits in LDS (a global load in
// the store loop would wait for every earlier store: vmcnt retires in order) and the residual quads
// are loaded before the tile's DMA. Ring halves are two separate LDS arrays, so the compiler can see
// that the DMA into one does not alias the reads of the other.
typedef __attribute__((address_space(3))) void gp_lds_void;

template <int KT, bool RES>
__global__ __launch_bounds__(256, 2) void gemm_pdma_x3_kernel(const PanelArgs g) {
  constexpr int G = KT / 8;
  constexpr int TILE_U32 = G * 384;
  constexpr int NI = TILE_U32 / 256 / 4;  // 1-KB DMA instructions per wave and tile
  static_assert(NI * 4 * 256 == TILE_U32, "tile DMA split");
  __shared__ __attribute__((aligned(16))) unsigned sbA[TILE_U32];
  __shared__ __attribute__((aligned(16))) unsigned sbB[TILE_U32];
  __shared__ float sbias[kPanelMaxN];
  const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
  const int nl = lane & 31, fh = lane >> 5;
  const int m0 = blockIdx.x * 128 + wave * 32;

  gp_u32x8 ca[G];
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
      ca[gi] = gp_u32x8{h0, h1, h0, h1, mm0, mm1, l0, l1};
    }
  }

  const int ct0 = blockIdx.y * g.ntile_per_split;
  const int ct1 = min(ct0 + g.ntile_per_split, g.N >> 5);
  for (int n = ct0 * 32 + tid; n < ct1 * 32; n += 256) sbias[n] = g.bias ? g.bias[n] : 0.f;
  // this wave's NI 1-KB pieces of tile ct: global u32 offset ct * TILE_U32 + (wave * NI + i) * 256
  auto dma_tile = [&](int ct, unsigned* dst) {
    const unsigned* src = g.w + (size_t)ct * TILE_U32 + lane * 4;
#pragma unroll
    for (int i = 0; i < NI; ++i)
      __builtin_amdgcn_global_load_lds((void*)(src + (wave * NI + i) * 256), (gp_lds_void*)(dst + (wave * NI + i) * 256),
                                       16, 0, 0);
  };
  if (ct0 < ct1) dma_tile(ct0, sbA);
  asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
  __syncthreads();

  const bool live = m0 < g.M;
  const int rows_left = g.M - m0;
  const int mrow = nl;
  float* orow = g.out + (size_t)(m0 + mrow) * g.ldo;
  const float* rrow = RES ? g.res + (size_t)(m0 + mrow) * g.ldr : nullptr;
  const bool row_ok = mrow < rows_left;
  f32x4 rv[RES ? 4 : 1];
  auto epilogue = [&](const f32x16& acc, int ctp, int q) {
    if (!row_ok) return;
    const int n = ctp * 32 + 8 * q + 4 * fh;
    f32x4 v = {acc[4 * q], acc[4 * q + 1], acc[4 * q + 2], acc[4 * q + 3]};
    if (g.vec) {
      v += *reinterpret_cast<const f32x4*>(sbias + n);
      if constexpr (RES) v += rv[q];
      if (g.relu) {
#pragma unroll
        for (int e = 0; e < 4; ++e) v[e] = fmaxf(v[e], 0.f);
      }
      *reinterpret_cast<f32x4*>(orow + n) = v;
    } else {
#pragma unroll
      for (int e = 0; e < 4; ++e) {
        float x = v[e] + sbias[n + e];
        if constexpr (RES) x += rrow[n + e];
        if (g.relu) x = fmaxf(x, 0.f);
        orow[n + e] = x;
      }
    }
  };
  f32x16 accp;
#pragma unroll
  for (int r = 0; r < 16; ++r) accp[r] = 0.f;
  // one tile: MFMAs on cur (tile ct) with tile ct - 1's stores in their gaps, tile ct + 1 DMA'd into nxt
  auto step = [&](int ct, const unsigned* cur, unsigned* nxt) {
    const bool has = ct < ct1;
    const bool st = live && ct > ct0;
    if constexpr (RES) {
      if (g.vec && st && row_ok) {
#pragma unroll
        for (int q = 0; q < 4; ++q) rv[q] = *reinterpret_cast<const f32x4*>(rrow + (ct - 1) * 32 + 8 * q + 4 * fh);
      }
    }
    if (ct + 1 < ct1) dma_tile(ct + 1, nxt);  // its last readers (tile ct - 1) passed the previous barrier
    f32x16 acc;
#pragma unroll
    for (int r = 0; r < 16; ++r) acc[r] = 0.f;
    const unsigned* bp = cur + lane * 4;
#pragma unroll
    for (int gi = 0; gi < G; ++gi) {
      if (live && has) {
        const gp_u32x4 mh = *reinterpret_cast<const gp_u32x4*>(bp + gi * 384);  // [m h]
        const gp_u32x2 lp = *reinterpret_cast<const gp_u32x2*>(cur + gi * 384 + 256 + lane * 2);
        const gp_u32x4 hl = {mh[2], mh[3], lp[0], lp[1]};  // [h l]
        acc = __builtin_amdgcn_mfma_f32_32x32x16_bf16(gp_op(hl), gp_sub4(ca[gi], 0), acc, 0, 0, 0);  // hh + lh
        acc = __builtin_amdgcn_mfma_f32_32x32x16_bf16(gp_op(mh), gp_sub4(ca[gi], 2), acc, 0, 0, 0);  // mh + hm
        acc = __builtin_amdgcn_mfma_f32_32x32x16_bf16(gp_op(mh), gp_sub4(ca[gi], 4), acc, 0, 0, 0);  // mm + hl
      }
      if (st && gi % (G / 4) == 0) epilogue(accp, ct - 1, gi / (G / 4));
    }
    accp = acc;
    // this wave's DMA into nxt must have landed before any wave reads it: vmcnt retires in order and
    // only the tile's 4 stores (issued by a live wave past its first tile) follow the DMA
    if (st) asm volatile("s_waitcnt vmcnt(4)" ::: "memory");
    else asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    __syncthreads();
  };
  for (int ct = ct0; ct <= ct1; ct += 2) {
    step(ct, sbA, sbB);
    if (ct + 1 <= ct1) step(ct + 1, sbB, sbA);
  }
}
}  // namespace

// KRRN_PANEL_CHAIN=1: the chain weight layout (ops.gemm_weights_panel_chain) and kernel form
static bool krrn_panel_chain() {
  static const bool on = [] {
    const char* e = getenv("KRRN_PANEL_CHAIN");
    const char* d = getenv("KRRN_PANEL_DMA");
    return (e && atoi(e) == 1) || (d && atoi(d) == 1);
  }();
  return on;
}

// KRRN_PANEL_DMA=1 (implies the chain layout): gemm_pdma_x3_kernel, two 4-wave blocks per CU
static bool krrn_panel_dma() {
  static const bool on = [] {
    const char* e = getenv("KRRN_PANEL_DMA");
    return e && atoi(e) == 1;
  }();
  return on;
}

KRRN_API int krrn_gemm_panel_x3_f32(const float* a, int lda, int M, int K, int N, const void* wpf, const float* bias,
                                    const float* res, int ldr, float* out, int ldo, int relu, int csplit,
                                    void* stream) {
  if (!a || !wpf || !out) return KRRN_EARG;
  if (M < 1 || (K != 64 && K != 128) || N < 32 || (N & 31) || N > kPanelMaxN || csplit < 1) return KRRN_ESHAPE;
  if (lda < K || ldo < N || (res && ldr < N)) return KRRN_ESHAPE;
  if ((lda & 3) || !krrn_aligned16(a) || !krrn_aligned16(wpf)) return KRRN_EALIGN;
  const int ntiles = N >> 5;
  const int per = krrn_cdiv(ntiles, csplit);
  PanelArgs g;
  g.a = a; g.w = reinterpret_cast<const unsigned*>(wpf); g.bias = bias; g.res = res; g.out = out;
  g.lda = lda; g.M = M; g.N = N; g.ldr = ldr; g.ldo = ldo; g.relu = relu;
  g.ntile_per_split = per;
  g.vec = krrn_aligned16(out) && !(ldo & 3) && (!res || (krrn_aligned16(res) && !(ldr & 3))) &&
          (!bias || krrn_aligned16(bias)) ? 1 : 0;
  hipStream_t s = (hipStream_t)stream;
  const dim3 grid((unsigned)krrn_cdiv(M, 256), (unsigned)krrn_cdiv(ntiles, per));
  if (K == 128 && res) {
    // a residual at K = 128 does not fit the kernel's register budget (the round-3 register-only
    // form that had room for it was removed: DESIGN.md §5)
    return KRRN_EUNSUPPORTED;
  }
  // KRRN_PANEL_DIAG (timing experiments only, outputs wrong): 1 = no MFMAs, 2 = no output stores
  static const int diag = [] {
    const char* e = getenv("KRRN_PANEL_DIAG");
    return e ? atoi(e) : 0;
  }();
  if (krrn_panel_dma()) {
    const dim3 grid2((unsigned)krrn_cdiv(M, 128), (unsigned)krrn_cdiv(ntiles, per));
    if (K == 128) hipLaunchKernelGGL((gemm_pdma_x3_kernel<128, false>), grid2, dim3(256), 0, s, g);
    else if (res) hipLaunchKernelGGL((gemm_pdma_x3_kernel<64, true>), grid2, dim3(256), 0, s, g);
    else hipLaunchKernelGGL((gemm_pdma_x3_kernel<64, false>), grid2, dim3(256), 0, s, g);
    return krrn_launch_status();
  }
  if (krrn_panel_chain()) {
    if (K == 128 && diag == 1) hipLaunchKernelGGL((gemm_plds_x3_kernel<128, false, 1, true>), grid, dim3(512), 0, s, g);
    else if (K == 128 && diag == 2) hipLaunchKernelGGL((gemm_plds_x3_kernel<128, false, 2, true>), grid, dim3(512), 0, s, g);
    else if (K == 128) hipLaunchKernelGGL((gemm_plds_x3_kernel<128, false, 0, true>), grid, dim3(512), 0, s, g);
    else if (res) hipLaunchKernelGGL((gemm_plds_x3_kernel<64, true, 0, true>), grid, dim3(512), 0, s, g);
    else hipLaunchKernelGGL((gemm_plds_x3_kernel<64, false, 0, true>), grid, dim3(512), 0, s, g);
    return krrn_launch_status();
  }
  if (K == 128 && diag == 1) hipLaunchKernelGGL((gemm_plds_x3_kernel<128, false, 1>), grid, dim3(512), 0, s, g);
  else if (K == 128 && diag == 2) hipLaunchKernelGGL((gemm_plds_x3_kernel<128, false, 2>), grid, dim3(512), 0, s, g);
  else if (K == 128) hipLaunchKernelGGL((gemm_plds_x3_kernel<128, false, 0>), grid, dim3(512), 0, s, g);
  else if (res) hipLaunchKernelGGL((gemm_plds_x3_kernel<64, true, 0>), grid, dim3(512), 0, s, g);
  else hipLaunchKernelGGL((gemm_plds_x3_kernel<64, false, 0>), grid, dim3(512), 0, s, g);
  return krrn_launch_status();
}
