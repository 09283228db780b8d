// The heads' final 1x1 convs with NCHW output: xyz_final (128 -> mask | region | xyz logits, 72
// channels for one class) and nml_final (128 -> 3 C normals), lib/network/krrn.py:97-98 / 80-84,
// SURVEY §8a D1 / D2. The API returns NCHW maps, so the store runs along pixels.
//
// A short-K (128), narrow-N GEMM over ~1M pixels: the implicit-GEMM conv ran it at 40 TFLOP/s
// (4 k-tiles per block, its prologue / epilogue dominating). Here a tile = 64 consecutive pixels
// of one image x all N output channels (NT 16-channel tiles): the 64 pixel rows (all K channels,
// one contiguous NHWC run each) are staged in LDS beside the block's weights, then each wave
// runs its 16 pixels x NT tiles over the whole K on v_mfma_f32_16x16x4_f32 with channels as the
// MFMA rows and pixels as its columns, so a lane group's 16 results of one channel are 16
// consecutive pixels: the NCHW store is a 64-B run per channel. One ds_read_b128 of a pixel's
// (or a weight row's) 4 k-values feeds 4 MFMAs (k = 4g + s over the 4 lane groups).
#include "krrn_common.h"

namespace {

constexpr int kPx = 64;       // pixels per block (16 per wave)
constexpr int kOP = kPx + 4;  // output staging pitch (floats)

// Persistent blocks: the weights are staged once per block, then the block walks its 64-pixel
// tiles (b, px0), the next tile's pixel rows loaded into registers while the current tile's
// MFMAs run (8 float4 per thread), written to LDS after the barrier.
template <int NT>
__global__ __launch_bounds__(256) void conv1x1_nchw_kernel(const float* __restrict__ in, int in_cs, int in_co, int B,
                                                           int HW, int K, int Kp, const float* __restrict__ wt, int N,
                                                           int n_store, const float* __restrict__ scale,
                                                           const float* __restrict__ bias, float* __restrict__ out,
                                                           int out_cs, int out_co, int vec) {
  extern __shared__ __attribute__((aligned(16))) float lds[];
  const int pitch = Kp + 4;  // odd number of 16-B slots per row: conflict-free b128 reads
  float* sx = lds;                  // [kPx][pitch]
  float* sw = lds + kPx * pitch;    // [16 NT][pitch]
  const int tid = threadIdx.x;
  const int kq = Kp / 4;
  const int tpi = krrn_cdiv(HW, kPx), ntiles = B * tpi;
  for (int e = tid; e < 16 * NT * kq; e += 256) {
    const int n = e / kq, q = e - (e / kq) * kq;
    f32x4 v = {0.f, 0.f, 0.f, 0.f};
    if (n < N && 4 * q < K) v = *reinterpret_cast<const f32x4*>(wt + (long long)n * K + 4 * q);
    *reinterpret_cast<f32x4*>(sw + n * pitch + 4 * q) = v;
  }
  // this thread's staging elements: e = tid + 256 u over kPx * kq (<= 64 * 64 / 256 = 16 float4)
  constexpr int kMaxU = 16;
  const int nu = krrn_cdiv(kPx * kq, 256);
  auto load_x = [&](int tile, f32x4 (&r)[kMaxU]) {
    const int b = tile / tpi, px0 = (tile - b * tpi) * kPx;
    const float* xb = in + ((long long)b * HW) * in_cs + in_co;
#pragma unroll
    for (int u = 0; u < kMaxU; ++u) {
      r[u] = f32x4{0.f, 0.f, 0.f, 0.f};
      const int e = tid + 256 * u;
      if (u < nu && e < kPx * kq) {
        const int p = e / kq, q = e - (e / kq) * kq;
        if (px0 + p < HW && 4 * q < K) r[u] = *reinterpret_cast<const f32x4*>(xb + (long long)(px0 + p) * in_cs + 4 * q);
      }
    }
  };
  const int lane = tid & 63, wave = tid >> 6;
  const int fr = lane & 15, g = lane >> 4;
  const float* xr = sx + (16 * wave + fr) * pitch + 4 * g;  // this lane's pixel, k-quad g
  const float* wr = sw + fr * pitch + 4 * g;                 // channel fr of tile t at + t * 16 * pitch
  f32x4 xn[kMaxU];
  if (blockIdx.x < ntiles) load_x(blockIdx.x, xn);
  for (int tile = blockIdx.x; tile < ntiles; tile += gridDim.x) {
    __syncthreads();  // the previous tile's MFMAs are done reading sx (and sw is staged)
#pragma unroll
    for (int u = 0; u < kMaxU; ++u) {
      const int e = tid + 256 * u;
      if (u < nu && e < kPx * kq) {
        const int p = e / kq, q = e - (e / kq) * kq;
        *reinterpret_cast<f32x4*>(sx + p * pitch + 4 * q) = xn[u];
      }
    }
    __syncthreads();
    if (tile + (int)gridDim.x < ntiles) load_x(tile + gridDim.x, xn);  // in flight under the MFMAs
    f32x4 acc[NT];
#pragma unroll
    for (int t = 0; t < NT; ++t) acc[t] = f32x4{0.f, 0.f, 0.f, 0.f};
    for (int k0 = 0; k0 < Kp; k0 += 16) {
      const f32x4 xv = *reinterpret_cast<const f32x4*>(xr + k0);
#pragma unroll
      for (int t = 0; t < NT; ++t) {
        const f32x4 wv = *reinterpret_cast<const f32x4*>(wr + t * 16 * pitch + k0);
#pragma unroll
        for (int s2 = 0; s2 < 4; ++s2) acc[t] = __builtin_amdgcn_mfma_f32_16x16x4f32(wv[s2], xv[s2], acc[t], 0, 0, 0);
      }
    }
    // acc[t][i] = (channel 16 t + 4 g + i, pixel 16 wave + fr)
    const int b = tile / tpi, px0 = (tile - b * tpi) * kPx;
    if (vec) {
      // transposed through LDS (sx is free once every wave's MFMAs are done): each channel's 64
      // pixels leave as one 256-B run of float4 stores instead of four 64-B lane-group runs
      __syncthreads();
      float* so = sx;  // [16 NT][kOP]
#pragma unroll
      for (int t = 0; t < NT; ++t)
#pragma unroll
        for (int i = 0; i < 4; ++i) so[(16 * t + 4 * g + i) * kOP + 16 * wave + fr] = acc[t][i];
      __syncthreads();
      float* ob = out + ((long long)b * out_cs + out_co) * HW + px0;
      for (int e = tid; e < n_store * (kPx / 4); e += 256) {
        const int n = e / (kPx / 4), q = e - n * (kPx / 4);
        if (px0 + 4 * q >= HW) continue;  // HW % 4 == 0: a float4 is all in or all out
        const float sc = scale ? scale[n] : 1.f, bi = bias ? bias[n] : 0.f;
        f32x4 v = *reinterpret_cast<const f32x4*>(so + n * kOP + 4 * q);
#pragma unroll
        for (int i = 0; i < 4; ++i) v[i] = v[i] * sc + bi;
        *reinterpret_cast<f32x4*>(ob + (long long)n * HW + 4 * q) = v;
      }
      continue;
    }
    const int px = px0 + 16 * wave + fr;
    if (px < HW) {
      float* ob = out + ((long long)b * out_cs + out_co) * HW + px;
#pragma unroll
      for (int t = 0; t < NT; ++t)
#pragma unroll
        for (int i = 0; i < 4; ++i) {
          const int n = 16 * t + 4 * g + i;
          if (n < n_store) ob[(long long)n * HW] = acc[t][i] * (scale ? scale[n] : 1.f) + (bias ? bias[n] : 0.f);
        }
    }
  }
}

// Split-bf16 form (X3) for the wide head (xyz_final: K = 128, N = 72 -> 5 channel tiles): block =
// NT waves, wave w owns channel tile w for the whole K with its [m h l] weight chains in registers
// for the block's life (8 steps x 6 VGPRs, loaded once), so LDS holds only the staged pixel rows,
// split into [h h] / [m l] planes (67.6 KB: two blocks per CU). Per 16 k and 16-pixel subtile three
// v_mfma_f32_16x16x32_bf16 (W[h l] x X[h h], W[m h] x X[h m], W[m h] x X[m l]: the six term
// products hh lh mh hm mm hl at f32 accuracy, 2.67x the f32 MFMA rate). Same output layout and
// NCHW store path as the f32 kernel.
typedef __bf16 nx_bf16x8 __attribute__((ext_vector_type(8)));
typedef __bf16 nx_bf16x2 __attribute__((ext_vector_type(2)));
typedef float nx_f32x2 __attribute__((ext_vector_type(2)));
typedef unsigned nx_u32x4 __attribute__((ext_vector_type(4)));
typedef unsigned nx_u32x2 __attribute__((ext_vector_type(2)));

__device__ __forceinline__ unsigned nx_pk(float a, float b) {
  return __builtin_bit_cast(unsigned, __builtin_convertvector(nx_f32x2{a, b}, nx_bf16x2));  // RNE
}
__device__ __forceinline__ void nx_split(const f32x4 x, nx_u32x4& p0, nx_u32x4& p1) {
  const unsigned h0 = nx_pk(x[0], x[1]), h1 = nx_pk(x[2], x[3]);
  const float r0 = x[0] - __builtin_bit_cast(float, h0 << 16), r1 = x[1] - __builtin_bit_cast(float, h0 & 0xFFFF0000u);
  const float r2 = x[2] - __builtin_bit_cast(float, h1 << 16), r3 = x[3] - __builtin_bit_cast(float, h1 & 0xFFFF0000u);
  const unsigned m0 = nx_pk(r0, r1), m1 = nx_pk(r2, r3);
  const unsigned l0 = nx_pk(r0 - __builtin_bit_cast(float, m0 << 16), r1 - __builtin_bit_cast(float, m0 & 0xFFFF0000u));
  const unsigned l1 = nx_pk(r2 - __builtin_bit_cast(float, m1 << 16), r3 - __builtin_bit_cast(float, m1 & 0xFFFF0000u));
  p0 = nx_u32x4{h0, h1, h0, h1};
  p1 = nx_u32x4{m0, m1, l0, l1};
}
__device__ __forceinline__ nx_bf16x8 nx_op(const nx_u32x4 v) { return __builtin_bit_cast(nx_bf16x8, v); }

constexpr int kX3Steps = 8;          // K = 128: 8 steps of 16 k (4 channel quads x 4 lane groups)
constexpr int kX3Q = 4 * kX3Steps;   // channel quads per pixel
constexpr int kX3Pitch = kX3Q + 1;   // 16-B slots per staged pixel and plane (odd: conflict-free)

template <int NT>
__global__ __launch_bounds__(64 * NT) void conv1x1_nchw_x3_kernel(const float* __restrict__ in, int in_cs, int in_co,
                                                                  int B, int HW, const unsigned* __restrict__ w3,
                                                                  int n_store, const float* __restrict__ scale,
                                                                  const float* __restrict__ bias, float* __restrict__ out,
                                                                  int out_cs, int out_co, int vec) {
  constexpr int kThreads = 64 * NT;
  extern __shared__ __attribute__((aligned(16))) float lds[];
  nx_u32x4* sx0 = reinterpret_cast<nx_u32x4*>(lds);  // [kPx][kX3Pitch] planes [h h], then [m l]
  nx_u32x4* sx1 = sx0 + kPx * kX3Pitch;
  const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
  const int fr = lane & 15, g = lane >> 4;
  const int tpi = krrn_cdiv(HW, kPx), ntiles = B * tpi;
  // this wave's weight chains for the whole K (record = channel x quad; quads of step st: 4 st + g)
  const unsigned nrec = (unsigned)(16 * NT * kX3Q);
  const nx_u32x4* wmh_g = reinterpret_cast<const nx_u32x4*>(w3);
  const nx_u32x2* wl_g = reinterpret_cast<const nx_u32x2*>(w3 + 4 * nrec);
  nx_u32x4 wmh[kX3Steps];
  nx_u32x2 wl[kX3Steps];
#pragma unroll
  for (int st = 0; st < kX3Steps; ++st) {
    const int r = (16 * wave + fr) * kX3Q + 4 * st + g;
    wmh[st] = wmh_g[r];
    wl[st] = wl_g[r];
  }
  constexpr int kItems = kPx * kX3Q;  // float4 per tile
  constexpr int kU = (kItems + kThreads - 1) / kThreads;
  auto load_x = [&](int tile, f32x4 (&r)[kU]) {
    const int b = tile / tpi, px0 = (tile - b * tpi) * kPx;
    const float* xb = in + ((long long)b * HW) * in_cs + in_co;
#pragma unroll
    for (int u = 0; u < kU; ++u) {
      const int e = tid + kThreads * u;
      const int p = e / kX3Q, q = e - (e / kX3Q) * kX3Q;
      r[u] = (e < kItems && px0 + p < HW) ? *reinterpret_cast<const f32x4*>(xb + (long long)(px0 + p) * in_cs + 4 * q)
                                          : f32x4{0.f, 0.f, 0.f, 0.f};
    }
  };
  f32x4 xn[kU];
  if (blockIdx.x < ntiles) load_x(blockIdx.x, xn);
  for (int tile = blockIdx.x; tile < ntiles; tile += gridDim.x) {
    __syncthreads();  // the previous tile's MFMAs / output transpose are done with the planes
#pragma unroll
    for (int u = 0; u < kU; ++u) {
      const int e = tid + kThreads * u;
      if (e < kItems) {
        const int p = e / kX3Q, q = e - (e / kX3Q) * kX3Q;
        nx_u32x4 p0, p1;
        nx_split(xn[u], p0, p1);
        sx0[p * kX3Pitch + q] = p0;
        sx1[p * kX3Pitch + q] = p1;
      }
    }
    __syncthreads();
    if (tile + (int)gridDim.x < ntiles) load_x(tile + gridDim.x, xn);  // in flight under the MFMAs
    f32x4 acc[4];
#pragma unroll
    for (int s = 0; s < 4; ++s) acc[s] = f32x4{0.f, 0.f, 0.f, 0.f};
#pragma unroll
    for (int st = 0; st < kX3Steps; ++st) {
      const nx_u32x4 whl = nx_u32x4{wmh[st][2], wmh[st][3], wl[st][0], wl[st][1]};
#pragma unroll
      for (int s = 0; s < 4; ++s) {
        const int e = (16 * s + fr) * kX3Pitch + 4 * st + g;
        const nx_u32x4 x0 = sx0[e], x1 = sx1[e];
        const nx_u32x4 xhm = nx_u32x4{x0[0], x0[1], x1[0], x1[1]};
        acc[s] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(nx_op(whl), nx_op(x0), acc[s], 0, 0, 0);
        acc[s] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(nx_op(wmh[st]), nx_op(xhm), acc[s], 0, 0, 0);
        acc[s] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(nx_op(wmh[st]), nx_op(x1), acc[s], 0, 0, 0);
      }
    }
    // acc[s][i] = (channel 16 wave + 4 g + i, pixel 16 s + fr)
    const int b = tile / tpi, px0 = (tile - b * tpi) * kPx;
    if (vec) {
      __syncthreads();
      float* so = lds;  // [16 NT][kOP], over the planes (every wave's MFMAs are done)
#pragma unroll
      for (int s = 0; s < 4; ++s)
#pragma unroll
        for (int i = 0; i < 4; ++i) so[(16 * wave + 4 * g + i) * kOP + 16 * s + fr] = acc[s][i];
      __syncthreads();
      float* ob = out + ((long long)b * out_cs + out_co) * HW + px0;
      for (int e = tid; e < n_store * (kPx / 4); e += kThreads) {
        const int n = e / (kPx / 4), q = e - n * (kPx / 4);
        if (px0 + 4 * q >= HW) continue;  // HW % 4 == 0: a float4 is all in or all out
        const float sc = scale ? scale[n] : 1.f, bi = bias ? bias[n] : 0.f;
        f32x4 v = *reinterpret_cast<const f32x4*>(so + n * kOP + 4 * q);
#pragma unroll
        for (int i = 0; i < 4; ++i) v[i] = v[i] * sc + bi;
        *reinterpret_cast<f32x4*>(ob + (long long)n * HW + 4 * q) = v;
      }
      continue;
    }
    float* ob = out + ((long long)b * out_cs + out_co) * HW + px0;
#pragma unroll
    for (int s = 0; s < 4; ++s) {
      const int px = 16 * s + fr;
      if (px0 + px >= HW) continue;
#pragma unroll
      for (int i = 0; i < 4; ++i) {
        const int n = 16 * wave + 4 * g + i;
        if (n < n_store) ob[(long long)n * HW + px] = acc[s][i] * (scale ? scale[n] : 1.f) + (bias ? bias[n] : 0.f);
      }
    }
  }
}

}  // namespace

KRRN_API int krrn_conv1x1_nchw_x3_f32(const float* in, int in_cs, int in_co, int B, int HW, int cin, const void* w3,
                                      int N, int n_store, const float* scale, const float* bias, float* out, int out_cs,
                                      int out_co, void* stream) {
  if (!in || !w3 || !out) return KRRN_EARG;
  if (B < 1 || HW < 1 || N < 1 || N > 80 || n_store < 1 || n_store > N) return KRRN_ESHAPE;
  if (cin != 4 * kX3Q) return KRRN_ESHAPE;  // the heads' 128-channel input (weights in registers)
  if ((in_cs & 3) || (in_co & 3) || in_co + cin > in_cs) return KRRN_EALIGN;
  if (!krrn_aligned16(in) || !krrn_aligned16(w3)) return KRRN_EALIGN;
  if (out_co + n_store > out_cs || (long long)B * HW * in_cs >= (1LL << 40)) return KRRN_ESHAPE;
  if ((long long)B * krrn_cdiv(HW, kPx) > 0x7fffffffLL) return KRRN_ESHAPE;
  const int nt = (N + 15) / 16;
  const size_t lds = 2 * sizeof(nx_u32x4) * (size_t)kPx * kX3Pitch;  // >= the output tile 16 nt x kOP floats
  const int ntiles = B * krrn_cdiv(HW, kPx);
  const dim3 grid(min(ntiles, 256 * 2));
  hipStream_t s = (hipStream_t)stream;
  const int vec = (HW % 4 == 0) && krrn_aligned16(out) ? 1 : 0;
#define KRRN_1X1X3(NTV)                                                                                        \
  if (nt == NTV) {                                                                                             \
    const hipError_t e = hipFuncSetAttribute((const void*)conv1x1_nchw_x3_kernel<NTV>,                         \
                                             hipFuncAttributeMaxDynamicSharedMemorySize, (int)lds);           \
    if (e != hipSuccess) return (int)e;                                                                        \
    hipLaunchKernelGGL(conv1x1_nchw_x3_kernel<NTV>, grid, dim3(64 * NTV), lds, s, in, in_cs, in_co, B, HW,     \
                       reinterpret_cast<const unsigned*>(w3), n_store, scale, bias, out, out_cs, out_co, vec); \
    return krrn_launch_status();                                                                               \
  }
  KRRN_1X1X3(1) KRRN_1X1X3(2) KRRN_1X1X3(3) KRRN_1X1X3(4) KRRN_1X1X3(5)
#undef KRRN_1X1X3
  return KRRN_ESHAPE;
}

KRRN_API int krrn_conv1x1_nchw_f32(const float* in, int in_cs, int in_co, int B, int HW, int cin, const float* wt,
                                   int N, int n_store, const float* scale, const float* bias, float* out, int out_cs,
                                   int out_co, void* stream) {
  if (!in || !wt || !out) return KRRN_EARG;
  if (B < 1 || HW < 1 || cin < 4 || N < 1 || N > 80 || n_store < 1 || n_store > N) return KRRN_ESHAPE;
  if ((cin & 3) || (in_cs & 3) || (in_co & 3) || in_co + cin > in_cs) return KRRN_EALIGN;
  if (!krrn_aligned16(in) || !krrn_aligned16(wt)) return KRRN_EALIGN;
  if (out_co + n_store > out_cs || (long long)B * HW * in_cs >= (1LL << 40)) return KRRN_ESHAPE;
  if (cin > 256 || (long long)B * krrn_cdiv(HW, kPx) > 0x7fffffffLL) return KRRN_ESHAPE;  // kMaxU float4 per thread
  const int Kp = (cin + 15) / 16 * 16;
  const int nt = (N + 15) / 16;
  const size_t lds = sizeof(float) * (size_t)(kPx + 16 * nt) * (Kp + 4);
  if (lds > 160 * 1024) return KRRN_ESHAPE;
  const int ntiles = B * krrn_cdiv(HW, kPx);
  const int per_cu = (int)((160 * 1024) / lds);
  const dim3 grid(min(ntiles, 256 * (per_cu < 1 ? 1 : per_cu)));
  hipStream_t s = (hipStream_t)stream;
  // float4 NCHW stores when every channel plane starts 16-B aligned and the staging tile
  // (16 nt x kOP floats) fits the pixel-row region sx (kPx x (Kp + 4)): the heads' K = 128
  const int vec = (HW % 4 == 0) && krrn_aligned16(out) && kPx * (Kp + 4) >= 16 * nt * kOP ? 1 : 0;
#define KRRN_1X1(NTV)                                                                                                   \
  if (nt == NTV) {                                                                                                      \
    if (lds > 64 * 1024) {                                                                                              \
      const hipError_t e = hipFuncSetAttribute((const void*)conv1x1_nchw_kernel<NTV>,                                  \
                                               hipFuncAttributeMaxDynamicSharedMemorySize, (int)lds);                  \
      if (e != hipSuccess) return (int)e;                                                                               \
    }                                                                                                                   \
    hipLaunchKernelGGL(conv1x1_nchw_kernel<NTV>, grid, dim3(256), lds, s, in, in_cs, in_co, B, HW, cin, Kp, wt, N,     \
                       n_store, scale, bias, out, out_cs, out_co, vec);                                                 \
    return krrn_launch_status();                                                                                        \
  }
  KRRN_1X1(1) KRRN_1X1(2) KRRN_1X1(3) KRRN_1X1(4) KRRN_1X1(5)
#undef KRRN_1X1
  return KRRN_ESHAPE;
}
