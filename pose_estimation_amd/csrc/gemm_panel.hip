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
//   * a block of 4 waves owns 128 rows; a wave loads its 32 x K activation panel once (one float4
//     per lane per 8-k group), splits it into the register chain [h h m l] per group and keeps it
//     (K = 128: 128 VGPRs) while the block walks its 32-column tiles;
//   * per tile the host-split weights (ops.gemm_weights_panel: per 8-k group one [m h] quad and one
//     [l] pair per lane, 24 KB at K = 128) are copied into a 2-slot LDS ring one tile ahead by LDS DMA;
//     every wave reads them with one ds_read_b128 + one ds_read_b64 per group, and the three MFMAs
//     per 8 k take register slices, W[h l] x A[h h] = hh + lh, W[m h] x A[h m] = mh + hm,
//     W[m h] x A[m l] = mm + hl; one barrier per tile, two blocks per CU (74 KB LDS per block at K = 128:
//     48 KB weight ring + 8 KB bias + 18 KB store-transpose slots; 2 waves per SIMD);
//   * the previous tile's accumulator is stored in the current tile's MFMA gaps as 4 float4 per lane
//     (operands swapped so a lane holds 4 consecutive columns; transposed through LDS first so each
//     store instruction writes whole 128-B row segments), bias (from LDS) / residual / ReLU fused.
// The row panels of a launch split into `csplit` column ranges when the panels alone cannot fill
// the chip (level 1: M = 16000 -> 125 panels x 4 column ranges).
#include "krrn_common.h"

namespace {

constexpr int kPanelMaxN = 2048;  // columns whose bias a block stages in LDS
#ifndef KRRN_GP_EXP
#define KRRN_GP_EXP 0  // timing experiments only (results wrong): 1 no output stores, 2 no MFMAs
#endif
#ifndef KRRN_GP_NW128
// waves (32-row panels) per block at K = 128: 4 (two blocks per CU) or 8 (one; half the weight-tile
// copies into LDS, measured no faster: DESIGN.md "Next (after round 6)")
#define KRRN_GP_NW128 4
#endif

typedef __bf16 gp_bf16x8 __attribute__((ext_vector_type(8)));
typedef __bf16 gp_bf16x2 __attribute__((ext_vector_type(2)));
typedef float gp_f32x2 __attribute__((ext_vector_type(2)));
typedef unsigned gp_u32x2 __attribute__((ext_vector_type(2)));
typedef unsigned gp_u32x4 __attribute__((ext_vector_type(4)));
typedef unsigned gp_u32x8 __attribute__((ext_vector_type(8)));

struct PanelArgs {
  const float* a;
  const unsigned* w;  // [N/32][K/8][384] u32 (ops.gemm_weights_panel)
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
__device__ __forceinline__ gp_bf16x8 gp_sub4(const gp_u32x8& c, int o) {
  return __builtin_bit_cast(gp_bf16x8, gp_u32x4{c[o], c[o + 1], c[o + 2], c[o + 3]});
}

// ---- Two blocks per CU, weights staged by LDS DMA (gemm_pdma_x3_kernel) --------------------------
// Round 3's 8-wave form (one block per CU, 48-B weight quads staged through registers) made every
// wave wait at each tile's barrier for the slowest wave's stores and staging: at the level-0 GCN GEMM
// 211 us = 105 us without its stores + 86 us without its MFMAs. Measured (profiles/bench_fusion_kernels.py):
// level 0 (M = 64000) 194 -> 140 us, level 1 (M = 16000, csplit 4) 39 -> 37 us; step +1.5 %. Here a block is 4 waves / 128 rows in the chain layout (24 KB per
// weight tile, 48 KB ring + 8 KB bias), so two independent blocks share a CU and one's store / staging
// phase overlaps the other's MFMAs. The weight tile is copied global -> LDS by buffer_load_dwordx4 ... lds
// (no staging registers: each wave instruction moves 1 KB), the bias sits in LDS (a global load in
// the store loop would wait for every earlier store: vmcnt retires in order) and the residual quads
// are loaded before the tile's DMA. Ring halves are two separate LDS arrays, so the compiler can see
// that the DMA into one does not alias the reads of the other.
typedef __attribute__((address_space(3))) void gp_lds_void;

// Transposed stores: a lane's accumulator is
// 4 float4 of ONE row, so a direct store instruction writes 32 rows x 32 B; the tile instead goes
// through a per-wave LDS slot and comes back as 8 lanes per row, and each store instruction writes 8
// whole 128-B row segments. The stores are buffer stores through a per-wave resource bounded by the
// wave's valid rows: rows past M are dropped by the hardware, so a live wave always issues its 4
// stores per tile (the vmcnt(4) accounting below depends on it).
constexpr int kTP = 36;  // LDS pitch of a transposed tile row (floats; conflict-free b128 writes)

template <int KT, bool RES, int NW>
__global__ __launch_bounds__(64 * NW, 8 / NW) void gemm_pdma_x3_kernel(const PanelArgs g) {
  constexpr int G = KT / 8;
  constexpr int TILE_U32 = G * 384;
  constexpr int NI = TILE_U32 / 256 / NW;  // 1-KB DMA instructions per wave and tile
  static_assert(NI * NW * 256 == TILE_U32, "tile DMA split");
  __shared__ __attribute__((aligned(16))) unsigned sbA[TILE_U32];
  __shared__ __attribute__((aligned(16))) unsigned sbB[TILE_U32];
  __shared__ __attribute__((aligned(16))) float sbias[kPanelMaxN];  // read as f32x4 (ds_read_b128)
  __shared__ __attribute__((aligned(16))) float stile[NW][32 * kTP];
  const int tid = threadIdx.x, lane = tid & 63;
  const int wave = __builtin_amdgcn_readfirstlane(tid >> 6);
  const int nl = lane & 31, fh = lane >> 5;
  const int m0 = blockIdx.x * (32 * NW) + wave * 32;

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
  for (int n = ct0 * 32 + tid; n < ct1 * 32; n += 64 * NW) sbias[n] = g.bias ? g.bias[n] : 0.f;
  // this wave's NI 1-KB pieces of tile ct: byte offset (ct * TILE_U32 + (wave * NI + i) * 256) * 4,
  // through a buffer resource (per-lane 32-bit voffset, the tile part in soffset: no 64-bit address
  // registers)
  const __amdgpu_buffer_rsrc_t rsW = __builtin_amdgcn_make_buffer_rsrc(
      (void*)g.w, (short)0, (int)min((long long)(g.N >> 5) * TILE_U32 * 4, 0x7FFFFFFFLL), 0x00020000);
  auto dma_tile = [&](int ct, unsigned* dst) {
#pragma unroll
    for (int i = 0; i < NI; ++i)
      __builtin_amdgcn_raw_ptr_buffer_load_lds(rsW, (gp_lds_void*)(dst + (wave * NI + i) * 256), 16,
                                               (unsigned)(lane * 16),
                                               (unsigned)((ct * TILE_U32 + (wave * NI + i) * 256) * 4), 0, 0);
  };
  if (ct0 < ct1) dma_tile(ct0, sbA);
  asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
  __syncthreads();

  const bool live = m0 < g.M;
  const int rows_left = g.M - m0;
  f32x4 rv[RES ? 4 : 1];
  float* const tw = stile[wave];
  const int trow = lane >> 3, tcol = 4 * (lane & 7);  // store j: row 8 j + trow, columns tcol .. + 3
  const int vrows = live ? min(32, rows_left) : 0;
  const __amdgpu_buffer_rsrc_t rsO = __builtin_amdgcn_make_buffer_rsrc(
      (void*)(g.out + (size_t)(live ? m0 : 0) * g.ldo), (short)0, vrows * g.ldo * 4, 0x00020000);
  const __amdgpu_buffer_rsrc_t rsR = __builtin_amdgcn_make_buffer_rsrc(
      (void*)(RES && g.res ? g.res + (size_t)(live ? m0 : 0) * g.ldr : g.out), (short)0,
      RES && g.res ? vrows * g.ldr * 4 : 0, 0x00020000);
  f32x4 tv[4];
  auto epilogue_t = [&](int ctp, int j) {
    const int n = ctp * 32 + tcol;
    f32x4 v = tv[j] + *reinterpret_cast<const f32x4*>(sbias + n);
    if constexpr (RES) v += rv[j];
    if (g.relu) {
#pragma unroll
      for (int e = 0; e < 4; ++e) v[e] = fmaxf(v[e], 0.f);
    }
    const unsigned vo = (unsigned)(((8 * j + trow) * g.ldo + tcol) * 4);
    if (KRRN_GP_EXP & 1) {
      if (v[0] == 1234.5f) g.out[0] = v[1];
    } else if (g.vec) {
      __builtin_amdgcn_raw_buffer_store_b128(__builtin_bit_cast(gp_u32x4, v), rsO, vo, ctp * 128, 0);
    } else {
      // out / ldo not 16-B aligned: four dword stores. (Not __builtin_bit_cast(unsigned, v[e]): on an
      // ext_vector element clang (ROCm 7.2) reads element 0 whatever e is -- the IR extracts lane 0 for
      // all four -- so this path stored v[0] four times; found by
      // tests/test_gpu_gemm.py::test_gemm_panel_scalar_epilogue.)
#pragma unroll
      for (int e = 0; e < 4; ++e)
        __builtin_amdgcn_raw_buffer_store_b32(__float_as_uint(v[e]), rsO, vo + 4 * e, ctp * 128, 0);
    }
  };
  f32x16 accp;
#pragma unroll
  for (int r = 0; r < 16; ++r) accp[r] = 0.f;
  // one tile: MFMAs on cur (tile ct) with tile ct - 1's stores in their gaps, tile ct + 1 DMA'd into nxt
  auto step = [&](int ct, const unsigned* cur, unsigned* nxt) {
    const bool has = ct < ct1;
    const bool st = live && ct > ct0;
    if (st) {
      // tile ct - 1 through the wave's LDS slot: written as (row nl, columns 8 q + 4 fh), read back as
      // (row 8 j + trow, columns tcol); the slot is this wave's alone and a wave's LDS accesses stay in order
#pragma unroll
      for (int q = 0; q < 4; ++q)
        *reinterpret_cast<f32x4*>(tw + nl * kTP + 8 * q + 4 * fh) =
            f32x4{accp[4 * q], accp[4 * q + 1], accp[4 * q + 2], accp[4 * q + 3]};
      __builtin_amdgcn_wave_barrier();
#pragma unroll
      for (int j = 0; j < 4; ++j) tv[j] = *reinterpret_cast<const f32x4*>(tw + (8 * j + trow) * kTP + tcol);
      __builtin_amdgcn_wave_barrier();
      if constexpr (RES) {
#pragma unroll
        for (int j = 0; j < 4; ++j) {
          const unsigned ro = (unsigned)(((8 * j + trow) * g.ldr + tcol) * 4);
          if (g.vec) {
            rv[j] = __builtin_bit_cast(f32x4, __builtin_amdgcn_raw_buffer_load_b128(rsR, ro, (ct - 1) * 128, 0));
          } else {
#pragma unroll
            for (int e = 0; e < 4; ++e)
              rv[j][e] = __builtin_bit_cast(float, __builtin_amdgcn_raw_buffer_load_b32(rsR, ro + 4 * e, (ct - 1) * 128, 0));
          }
        }
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
#if KRRN_GP_EXP & 2
        acc[gi & 15] += __uint_as_float(hl[0] ^ mh[1] ^ ca[gi][0]);
#else
        acc = __builtin_amdgcn_mfma_f32_32x32x16_bf16(gp_op(hl), gp_sub4(ca[gi], 0), acc, 0, 0, 0);  // hh + lh
        acc = __builtin_amdgcn_mfma_f32_32x32x16_bf16(gp_op(mh), gp_sub4(ca[gi], 2), acc, 0, 0, 0);  // mh + hm
        acc = __builtin_amdgcn_mfma_f32_32x32x16_bf16(gp_op(mh), gp_sub4(ca[gi], 4), acc, 0, 0, 0);  // mm + hl
#endif
      }
      if (st && gi % (G / 4) == 0) epilogue_t(ct - 1, gi / (G / 4));
    }
    accp = acc;
    // this wave's DMA into nxt must have landed before any wave reads it: vmcnt retires in order and
    // only the tile's 4 stores (issued by a live wave past its first tile) follow the DMA
    if (st && !(KRRN_GP_EXP & 1)) asm volatile("s_waitcnt vmcnt(4)" ::: "memory");
    else asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    __syncthreads();
  };
  for (int ct = ct0; ct <= ct1; ct += 2) {
    step(ct, sbA, sbB);
    if (ct + 1 <= ct1) step(ct + 1, sbB, sbA);
  }
}
}  // namespace

KRRN_API int krrn_gemm_panel_x3_f32(const float* a, int lda, int M, int K, int N, const void* wpf, const float* bias,
                                    const float* res, int ldr, float* out, int ldo, int relu, int csplit,
                                    void* stream) {
  if (!a || !wpf || !out) return KRRN_EARG;
  if (M < 1 || (K != 64 && K != 128) || N < 32 || (N & 31) || N > kPanelMaxN || csplit < 1) return KRRN_ESHAPE;
  if (lda < K || ldo < N || (res && ldr < N)) return KRRN_ESHAPE;
  if ((lda & 3) || !krrn_aligned16(a) || !krrn_aligned16(wpf)) return KRRN_EALIGN;
  // a residual at K = 128 does not fit the kernel's register budget (128 VGPRs of activation chain)
  if (K == 128 && res) return KRRN_EUNSUPPORTED;
  const int ntiles = N >> 5;
  const int per = krrn_cdiv(ntiles, csplit);
  PanelArgs g;
  g.a = a; g.w = reinterpret_cast<const unsigned*>(wpf); g.bias = bias; g.res = res; g.out = out;
  g.lda = lda; g.M = M; g.N = N; g.ldr = ldr; g.ldo = ldo; g.relu = relu;
  g.ntile_per_split = per;
  g.vec = krrn_aligned16(out) && !(ldo & 3) && (!res || (krrn_aligned16(res) && !(ldr & 3))) &&
          (!bias || krrn_aligned16(bias)) ? 1 : 0;
  hipStream_t s = (hipStream_t)stream;
  const unsigned gy = (unsigned)krrn_cdiv(ntiles, per);
  if (K == 128)
    hipLaunchKernelGGL((gemm_pdma_x3_kernel<128, false, KRRN_GP_NW128>),
                       dim3((unsigned)krrn_cdiv(M, 32 * KRRN_GP_NW128), gy), dim3(64 * KRRN_GP_NW128), 0, s, g);
  else if (res) hipLaunchKernelGGL((gemm_pdma_x3_kernel<64, true, 4>), dim3((unsigned)krrn_cdiv(M, 128), gy), dim3(256), 0, s, g);
  else hipLaunchKernelGGL((gemm_pdma_x3_kernel<64, false, 4>), dim3((unsigned)krrn_cdiv(M, 128), gy), dim3(256), 0, s, g);
  return krrn_launch_status();
}
