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

// Split-bf16 form (X3) for the wide head (xyz_final: K = 128, N = 72 -> 5 channel tiles). The
// block-staged form above is latency-bound on its input (one 32-KB tile in flight per block between
// barriers: ~2.6 TB/s); here every wave streams its own 16-pixel subtiles with no block barrier
// after the weight fill: the block's LDS holds all NT channel tiles' split weights in lane order
// ([tile][step][64 lanes], conflict-free 16 / 8-B reads), a lane loads its pixel's channel quad of
// each step straight from HBM (next subtile's 8 quads prefetched into registers) and splits it
// in registers into [h h] / [m l] operands. Per 16 k and channel tile three
// v_mfma_f32_16x16x32_bf16 (W[h l] x X[h h], W[m h] x X[h m], W[m h] x X[m l]: the six term
// products hh lh mh hm mm hl at f32 accuracy).
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

constexpr int kX3Steps = 8;         // K = 128: 8 steps of 16 k (4 channel quads x 4 lane groups)
constexpr int kX3Q = 4 * kX3Steps;  // channel quads per pixel
constexpr int kX3Waves = 8;

template <int NT>
__global__ __launch_bounds__(64 * kX3Waves) __attribute__((amdgpu_waves_per_eu(4))) void conv1x1_nchw_x3_kernel(const float* __restrict__ in, int in_cs,
                                                                        int in_co, int B, int HW,
                                                                        const unsigned* __restrict__ w3, int n_store,
                                                                        const float* __restrict__ scale,
                                                                        const float* __restrict__ bias,
                                                                        float* __restrict__ out, int out_cs,
                                                                        int out_co) {
  __shared__ nx_u32x4 smh[NT * kX3Steps * 64];  // [tile][step][lane]: m0..m3 h0..h3
  __shared__ nx_u32x2 sl[NT * kX3Steps * 64];   // l0..l3
  __shared__ float ssc[16 * NT], sbi[16 * NT];
  const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
  const int fr = lane & 15, g = lane >> 4;
  {
    const unsigned nrec = (unsigned)(16 * NT * kX3Q);
    const nx_u32x4* wmh_g = reinterpret_cast<const nx_u32x4*>(w3);
    const nx_u32x2* wl_g = reinterpret_cast<const nx_u32x2*>(w3 + 4 * nrec);
    for (int e = tid; e < NT * kX3Steps * 64; e += 64 * kX3Waves) {
      const int l = e & 63, ts = e >> 6, t = ts / kX3Steps, st = ts - t * kX3Steps;
      const int r = (16 * t + (l & 15)) * kX3Q + 4 * st + (l >> 4);
      smh[e] = wmh_g[r];
      sl[e] = wl_g[r];
    }
    for (int n = tid; n < 16 * NT; n += 64 * kX3Waves) {
      ssc[n] = n < n_store && scale ? scale[n] : 1.f;
      sbi[n] = n < n_store && bias ? bias[n] : 0.f;
    }
  }
  __syncthreads();
  const int spi = krrn_cdiv(HW, 16), nsub = B * spi;
  const __amdgpu_buffer_rsrc_t rso =
      __builtin_amdgcn_make_buffer_rsrc((void*)out, (short)0, (int)((long long)B * out_cs * HW * 4), 0x00020000);
  auto x_ptr = [&](int c, bool& ok) {
    const int b = c / spi, px = (c - b * spi) * 16 + fr;
    ok = px < HW;
    return in + ((long long)b * HW + px) * in_cs + in_co + 4 * g;
  };
  const int stride = gridDim.x * kX3Waves;
  int c = blockIdx.x * kX3Waves + wave;
  // xr[st]: this subtile's quad of step st; once steps 2j and 2j + 1 are split, their registers take
  // the next subtile's quads (in flight for a whole subtile of MFMAs)
  f32x4 xr[kX3Steps];
  if (c < nsub) {
    bool ok;
    const float* xp = x_ptr(c, ok);
#pragma unroll
    for (int st = 0; st < kX3Steps; ++st)
      xr[st] = ok ? *reinterpret_cast<const f32x4*>(xp + 16 * st) : f32x4{0.f, 0.f, 0.f, 0.f};
  }
  for (; c < nsub; c += stride) {
    const bool more = c + stride < nsub;
    bool nok = false;
    const float* np = more ? x_ptr(c + stride, nok) : in;
    nok = nok && more;
    f32x4 acc[NT];
#pragma unroll
    for (int t = 0; t < NT; ++t) acc[t] = f32x4{0.f, 0.f, 0.f, 0.f};
    int wl_off = lane;  // made opaque per step: keeps the weight reads in the loop, one step live at a time
#pragma unroll
    for (int st = 0; st < kX3Steps; ++st) {
      asm volatile("" : "+v"(wl_off));
      nx_u32x4 x0, x1;
      nx_split(xr[st], x0, x1);
      if (more && (st & 1)) {  // steps 2j, 2j + 1 are the two halves of one 128-B line: request them together
        xr[st - 1] = nok ? *reinterpret_cast<const f32x4*>(np + 16 * (st - 1)) : f32x4{0.f, 0.f, 0.f, 0.f};
        xr[st] = nok ? *reinterpret_cast<const f32x4*>(np + 16 * st) : f32x4{0.f, 0.f, 0.f, 0.f};
      }
      const nx_u32x4 xhm = nx_u32x4{x0[0], x0[1], x1[0], x1[1]};
#pragma unroll
      for (int t = 0; t < NT; ++t) {
        const nx_u32x4 wmh = smh[(t * kX3Steps + st) * 64 + wl_off];
        const nx_u32x2 wl = sl[(t * kX3Steps + st) * 64 + wl_off];
        const nx_u32x4 whl = nx_u32x4{wmh[2], wmh[3], wl[0], wl[1]};
        acc[t] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(nx_op(whl), nx_op(x0), acc[t], 0, 0, 0);
        acc[t] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(nx_op(wmh), nx_op(xhm), acc[t], 0, 0, 0);
        acc[t] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(nx_op(wmh), nx_op(x1), acc[t], 0, 0, 0);
      }
    }
    // acc[t][i] = (channel 16 t + 4 g + i, pixel 16 (c % spi) + fr): 64-B NCHW runs per channel.
    // Buffer stores: the lane's channel-group / pixel part in one 32-bit voffset, the (t, i) channel
    // part (16 t + i) HW in the scalar offset -- with plain 64-bit addresses LLVM hoisted all 20
    // per-channel offsets out of the subtile loop (40 VGPRs) and spilled 28 B / lane to scratch.
    const int b = c / spi, px = (c - b * spi) * 16 + fr;
    if (px < HW) {
      const unsigned vo = (unsigned)((((b * out_cs + out_co) + 4 * g) * HW + px) * 4);
#pragma unroll
      for (int t = 0; t < NT; ++t)
#pragma unroll
        for (int i = 0; i < 4; ++i) {
          const int n = 16 * t + 4 * g + i;
          if (n < n_store)
            __builtin_amdgcn_raw_buffer_store_b32(__builtin_bit_cast(unsigned, acc[t][i] * ssc[n] + sbi[n]), rso, vo,
                                                  (16 * t + i) * HW * 4, 0);  // the f32 bits (b32 takes a u32)
        }
    }
  }
}

// Narrow form (N <= 4 weight rows: the normal head's 3-channel conv, krrn.py:80-84): a pure HBM
// read of the 128-channel rows, so no MFMA tile (16 of 16 rows would idle) and no LDS staging:
// 8 lanes per pixel each read KQL channel quads (one 128-B run per 8 lanes and load), dot them
// against their quads of the <= 4 weight rows held in registers, and an xor butterfly sums the 8
// partials; each wave walks 32-pixel chunks (4 rounds of 8 pixels, all loads issued up front) and
// writes them through a per-wave LDS row as 128-B NCHW runs.
constexpr int kNarrowPx = 32;
constexpr int kNarrowPitch = kNarrowPx + 4;

template <int KQL>
__global__ __launch_bounds__(256) void conv1x1_nchw_narrow_kernel(const float* __restrict__ in, int in_cs, int in_co,
                                                                  int B, int HW, const float* __restrict__ wt, int N,
                                                                  int n_store, const float* __restrict__ scale,
                                                                  const float* __restrict__ bias,
                                                                  float* __restrict__ out, int out_cs, int out_co,
                                                                  int vec) {
  constexpr int cin = 32 * KQL;
  __shared__ __attribute__((aligned(16))) float so_all[4][4 * kNarrowPitch];
  const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
  const int j = lane & 7, k = lane >> 3;
  float* so = so_all[wave];
  f32x4 w[4][KQL];
#pragma unroll
  for (int n = 0; n < 4; ++n)
#pragma unroll
    for (int t = 0; t < KQL; ++t)
      w[n][t] = n < N ? *reinterpret_cast<const f32x4*>(wt + n * cin + 4 * (j + 8 * t)) : f32x4{0.f, 0.f, 0.f, 0.f};
  const int cpi = krrn_cdiv(HW, kNarrowPx), nch = B * cpi;
  for (int c = blockIdx.x * 4 + wave; c < nch; c += gridDim.x * 4) {
    const int b = c / cpi, px0 = (c - b * cpi) * kNarrowPx;
    f32x4 x[4][KQL];
#pragma unroll
    for (int it = 0; it < 4; ++it) {
      const int p = px0 + 8 * it + k;
      const float* xp = in + ((long long)b * HW + p) * in_cs + in_co + 4 * j;
#pragma unroll
      for (int t = 0; t < KQL; ++t)
        x[it][t] = p < HW ? *reinterpret_cast<const f32x4*>(xp + 32 * t) : f32x4{0.f, 0.f, 0.f, 0.f};
    }
    float acc[4][4];
#pragma unroll
    for (int it = 0; it < 4; ++it)
#pragma unroll
      for (int n = 0; n < 4; ++n) {
        float a = 0.f;
#pragma unroll
        for (int t = 0; t < KQL; ++t)
#pragma unroll
          for (int i = 0; i < 4; ++i) a = fmaf(x[it][t][i], w[n][t][i], a);
        acc[it][n] = a;
      }
#pragma unroll
    for (int off = 1; off < 8; off <<= 1)
#pragma unroll
      for (int it = 0; it < 4; ++it)
#pragma unroll
        for (int n = 0; n < 4; ++n) acc[it][n] += __shfl_xor(acc[it][n], off);
    // every lane of pixel group k holds its 16 sums: lane j writes channel j & 3 of rounds 2 (j >> 2) + {0, 1}
    {
      const int n = j & 3;
      const float sc = n < n_store && scale ? scale[n] : 1.f, bi = n < n_store && bias ? bias[n] : 0.f;
#pragma unroll
      for (int r = 0; r < 2; ++r) {
        const int it = 2 * (j >> 2) + r;
        float v = 0.f;
#pragma unroll
        for (int q = 0; q < 4; ++q)
#pragma unroll
          for (int nn = 0; nn < 4; ++nn) v = (q == it && nn == n) ? acc[q][nn] : v;
        so[n * kNarrowPitch + 8 * it + k] = v * sc + bi;
      }
    }
    __builtin_amdgcn_wave_barrier();
    float* ob = out + ((long long)b * out_cs + out_co) * HW + px0;
    if (vec) {
      const int n = lane >> 3, q = lane & 7;  // lanes 0..31: 4 channels x 8 float4
      if (n < n_store && px0 + 4 * q < HW)
        *reinterpret_cast<f32x4*>(ob + (long long)n * HW + 4 * q) = *reinterpret_cast<const f32x4*>(so + n * kNarrowPitch + 4 * q);
    } else if (lane < kNarrowPx && px0 + lane < HW) {
      for (int n = 0; n < n_store; ++n) ob[(long long)n * HW + lane] = so[n * kNarrowPitch + lane];
    }
    __builtin_amdgcn_wave_barrier();
  }
}

}  // namespace

KRRN_API int krrn_conv1x1_nchw_x3_f32(const float* in, int in_cs, int in_co, int B, int HW, int cin, const void* w3,
                                      int N, int n_store, const float* scale, const float* bias, float* out, int out_cs,
                                      int out_co, void* stream) {
  if (!in || !w3 || !out) return KRRN_EARG;
  // 3..5 channel tiles (the weight LDS and the accumulators sized for them)
  if (B < 1 || HW < 1 || N <= 32 || N > 80 || n_store < 1 || n_store > N) return KRRN_ESHAPE;
  if (cin != 4 * kX3Q) return KRRN_ESHAPE;  // the heads' 128-channel input (8 k steps)
  if ((in_cs & 3) || (in_co & 3) || in_co + cin > in_cs) return KRRN_EALIGN;
  if (!krrn_aligned16(in) || !krrn_aligned16(w3)) return KRRN_EALIGN;
  if (out_co + n_store > out_cs || (long long)B * HW * in_cs >= (1LL << 40)) return KRRN_ESHAPE;
  if ((long long)B * krrn_cdiv(HW, 16) > 0x3fffffffLL) return KRRN_ESHAPE;  // subtile index + grid stride fit int
  if ((long long)B * out_cs * HW * 4 >= 0x7FFFFFFFLL) return KRRN_ESHAPE;      // 32-bit buffer-store offsets
  const int nt = (N + 15) / 16;
  const int nsub = B * krrn_cdiv(HW, 16);
  const dim3 grid(min(krrn_cdiv(nsub, kX3Waves), 256 * 2));
  hipStream_t s = (hipStream_t)stream;
#define KRRN_1X1X3(NTV)                                                                                      \
  if (nt == NTV) {                                                                                           \
    hipLaunchKernelGGL(conv1x1_nchw_x3_kernel<NTV>, grid, dim3(64 * kX3Waves), 0, s, in, in_cs, in_co, B, HW, \
                       reinterpret_cast<const unsigned*>(w3), n_store, scale, bias, out, out_cs, out_co);     \
    return krrn_launch_status();                                                                             \
  }
  KRRN_1X1X3(3) KRRN_1X1X3(4) KRRN_1X1X3(5)
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
  if (N <= 4 && cin % 32 == 0 && cin <= 128) {  // the narrow (normal) head: VALU dot products, HBM-bound
    const int nch = B * krrn_cdiv(HW, kNarrowPx);
    const dim3 grid(min(krrn_cdiv(nch, 4), 256 * 3));
    const int vec = (HW % 4 == 0) && krrn_aligned16(out) ? 1 : 0;
    hipStream_t s = (hipStream_t)stream;
#define KRRN_1X1N(KQ)                                                                                      \
  if (cin == 32 * KQ) {                                                                                    \
    hipLaunchKernelGGL(conv1x1_nchw_narrow_kernel<KQ>, grid, dim3(256), 0, s, in, in_cs, in_co, B, HW, wt, \
                       N, n_store, scale, bias, out, out_cs, out_co, vec);                                 \
    return krrn_launch_status();                                                                           \
  }
    KRRN_1X1N(1) KRRN_1X1N(2) KRRN_1X1N(4)
#undef KRRN_1X1N
  }
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
