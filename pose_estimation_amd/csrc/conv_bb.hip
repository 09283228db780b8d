// One HRNet BasicBlock per launch (lib/network/hrnet/myhrnet.py:34-63):
//
//   y = ReLU( BN2(conv3x3(ReLU(BN1(conv3x3(x))))) + x )       (no downsample: the branch blocks)
//
// The branch blocks (18/36/72/144 channels at S/4 .. S/32, 208 convs per step at W18) were two
// latency-bound conv_small launches each (13-20 us for 3-6 us of f32 matrix work; a launch's
// staging, weight-latency and epilogue phases were ~9 us of it, profiles/bench_small.py). Here a
// block owns T output rows of one image and keeps everything between the two convs on chip:
//
//   stage   input rows [y0-2, y0+T+2) (zero outside the image) -> LDS, split into bf16 terms
//   conv1   mid rows [y0-1, y0+T+1) ∩ image, BN1 + ReLU, split -> LDS (zero rows / columns around)
//   conv2   output rows [y0, y0+T), BN2 + residual (x, from L2) + ReLU -> HBM
//
// so the intermediate never leaves the CU, one staging latency and one launch serve both convs,
// and the halo rows conv2 needs are recomputed (T = 4 at 30 px: 1.5x conv1 rows).
//
// Matrix math: the split-bf16 scheme of winograd.hip / gemm_x3.hip at f32 accuracy (x = x_h + x_m
// + x_l exactly, six term products hh hm mh hl lh mm on v_mfma_f32_16x16x32_bf16, f32
// accumulation; the dropped ml lm ll are below 2^-23 |w x|). The weights are the MFMA's first
// operand (rows = 16 output channels) and the activations its second (columns = 16 pixels), so a
// lane's accumulator is 4 consecutive channels of one pixel — exactly the 16-byte channel quad the
// next stage stores (LDS chains for conv2, a float4 for the output). A lane group's 8 k-slots are
// 2 term kinds x one channel quad (4 channels of one tap): per 16 k of the flattened reduction
// (k = tap * C + c) three MFMAs,
//   W[h l] x X[h h] = hh + lh,   W[m h] x X[h m] = mh + hm,   W[m h] x X[m l] = mm + hl.
// Activations live in LDS as two 16-byte planes per (pixel, channel quad), [h h] and [m l], with an
// odd pixel pitch (conflict-free ds_read_b128); weights are pre-split on the host into a 16-byte
// [m h] plane and an 8-byte [l] plane per (channel, quad), read from L2 four steps ahead.
//
// Work split per conv: NTt = C / 16 channel tiles; with NTt >= 4 each wave owns a range of NT
// channel tiles and walks every pixel tile (weights amortised over pixels), else each wave owns
// all channel tiles and every 4th pixel tile (activation reads amortised over channels).
#include "krrn_common.h"

namespace {

typedef __bf16 bb_bf16x8 __attribute__((ext_vector_type(8)));
typedef __bf16 bb_bf16x2 __attribute__((ext_vector_type(2)));
typedef float bb_f32x2 __attribute__((ext_vector_type(2)));
typedef unsigned bb_u32x4 __attribute__((ext_vector_type(4)));
typedef unsigned bb_u32x2 __attribute__((ext_vector_type(2)));
typedef unsigned bb_u32x8 __attribute__((ext_vector_type(8)));

struct BBArgs {
  const float* in;
  int in_cs, in_co;
  int B, H, W, Q;  // image; Q = C / 4 channel quads (C = padded channel count, multiple of 4)
  int T;           // output rows per block
  int tiles_y;     // ceil(H / T)
  int qp;          // LDS pixel pitch per plane in 16-B units: Q rounded up to odd
  int xrows, mrows;  // LDS rows of the input / mid tiles (max over blocks)
  const unsigned* w1;  // split weights: [m h] plane [NTt*16][KQp][4 u32], then [l] plane [..][2 u32]
  const unsigned* w2;
  int kqp;             // k-quads per weight row, padded to a multiple of 16 (steps, a multiple of 4, * 4)
  const float* s1;
  const float* b1;
  const float* s2;
  const float* b2;
  float* out;
  int out_cs, out_co;
  int ntt;  // channel tiles
  int nsplit;  // 1: waves split channel tiles, 0: waves split pixel tiles
};

__device__ __forceinline__ unsigned bb_pk(float a, float b) {
  return __builtin_bit_cast(unsigned, __builtin_convertvector(bb_f32x2{a, b}, bb_bf16x2));  // RNE
}

// 4 channels -> planes [h h] and [m l] (packed bf16 pairs)
__device__ __forceinline__ void bb_split(const f32x4 x, bb_u32x4& p0, bb_u32x4& p1) {
  const unsigned h0 = bb_pk(x[0], x[1]), h1 = bb_pk(x[2], x[3]);
  const float r0 = x[0] - __builtin_bit_cast(float, h0 << 16), r1 = x[1] - __builtin_bit_cast(float, h0 & 0xFFFF0000u);
  const float r2 = x[2] - __builtin_bit_cast(float, h1 << 16), r3 = x[3] - __builtin_bit_cast(float, h1 & 0xFFFF0000u);
  const unsigned m0 = bb_pk(r0, r1), m1 = bb_pk(r2, r3);
  const unsigned l0 = bb_pk(r0 - __builtin_bit_cast(float, m0 << 16), r1 - __builtin_bit_cast(float, m0 & 0xFFFF0000u));
  const unsigned l1 = bb_pk(r2 - __builtin_bit_cast(float, m1 << 16), r3 - __builtin_bit_cast(float, m1 & 0xFFFF0000u));
  p0 = bb_u32x4{h0, h1, h0, h1};
  p1 = bb_u32x4{m0, m1, l0, l1};
}

__device__ __forceinline__ bb_bf16x8 bb_op(const bb_u32x4 v) { return __builtin_bit_cast(bb_bf16x8, v); }
// registers o .. o + 3 of an 8-register chain as one MFMA operand (the chains are laid out so every
// operand is a contiguous slice: no copies)
__device__ __forceinline__ bb_bf16x8 bb_sub(const bb_u32x8& c, int o) {
  return __builtin_bit_cast(bb_bf16x8, bb_u32x4{c[o], c[o + 1], c[o + 2], c[o + 3]});
}

// One 3x3 conv of the block: out pixels [0, P) of a W-wide row range whose first row is `orow`
// (image row), reading the source tile (LDS planes, first row `srow`, zero columns 0 and W + 1).
// EPI(p, c4, f32x4 acc) consumes each valid (pixel, channel quad).
template <int MT, int NT, class Epi>
__device__ __forceinline__ void bb_conv(const BBArgs& a, const unsigned* wt, const bb_u32x4* src, int splane,
                                        int orow, int srow, int P, Epi epi) {
  const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
  const int fr = lane & 15, g = lane >> 4;
  const int W2 = a.W + 2, Q = a.Q, qp = a.qp;
  const int mtt = (P + 15) >> 4;
  const int nsteps = a.kqp >> 2;
  const int KQ = 9 * Q;
  // this wave's channel tiles and pixel-tile walk
  const int n0 = a.nsplit ? wave * NT : 0;
  const int mfirst = a.nsplit ? 0 : wave, mstep = a.nsplit ? MT : 4 * MT, mstride = a.nsplit ? 1 : 4;
  if (n0 >= a.ntt) return;
  const long long nrows = (long long)a.ntt * 16 * a.kqp;  // weight records
  const __amdgpu_buffer_rsrc_t rsMH =
      __builtin_amdgcn_make_buffer_rsrc((void*)wt, (short)0, (int)(nrows * 16), 0x00020000);
  const __amdgpu_buffer_rsrc_t rsL =
      __builtin_amdgcn_make_buffer_rsrc((void*)(wt + nrows * 4), (short)0, (int)(nrows * 8), 0x00020000);
  unsigned wrow[NT];
#pragma unroll
  for (int j = 0; j < NT; ++j) {
    const int nt = min(n0 + j, a.ntt - 1);  // past the last tile: a duplicate, never stored
    wrow[j] = (unsigned)((nt * 16 + fr) * a.kqp + g);
  }
  const int W2q = W2 * qp;
  for (int mc = mfirst; mc < mtt; mc += mstep) {
    // pixel tiles mc + mstride * i (i < MT) of this chunk: centre-tap LDS offsets (16-B units);
    // tiles past the last one recompute a valid tile (no branches in the K loop), never stored
    int pxq[MT];
#pragma unroll
    for (int i = 0; i < MT; ++i) {
      const int mt = min(mc + mstride * i, mtt - 1);
      const int p = min(mt * 16 + fr, P - 1);
      const int y = p / a.W, x = p - (p / a.W) * a.W;
      pxq[i] = ((orow + y - srow) * W2 + x + 1) * qp;
    }
    f32x4 acc[MT][NT];
#pragma unroll
    for (int i = 0; i < MT; ++i)
#pragma unroll
      for (int j = 0; j < NT; ++j) acc[i][j] = f32x4{0.f, 0.f, 0.f, 0.f};
    // weights KPF steps ahead in a register ring, as 6-register chains [m h l]; the activation
    // chains [h h m l] one step ahead
#ifndef KRRN_BB_KPF
#define KRRN_BB_KPF 4
#endif
    constexpr int KPF = KRRN_BB_KPF;
    bb_u32x8 wr[KPF][NT];
    auto wload = [&](int st, int slot) {
      const unsigned kq = (unsigned)(min(st, nsteps - 1) * 4);
#pragma unroll
      for (int j = 0; j < NT; ++j) {
        const unsigned r = wrow[j] + kq;
        const bb_u32x4 mh = __builtin_bit_cast(bb_u32x4, __builtin_amdgcn_raw_buffer_load_b128(rsMH, r * 16u, 0, 0));
        const bb_u32x2 l = __builtin_bit_cast(bb_u32x2, __builtin_amdgcn_raw_buffer_load_b64(rsL, r * 8u, 0, 0));
        wr[slot][j] = bb_u32x8{mh[0], mh[1], mh[2], mh[3], l[0], l[1], 0u, 0u};
      }
    };
#pragma unroll
    for (int u = 0; u < KPF; ++u) wload(u, u);
    // the next step to read: k-quad kq = tap * Q + c4 (Q >= 4: at most one wrap per step)
    int kq = g, tap = g / Q, c4 = g - (g / Q) * Q;
    bb_u32x8 xa[2][MT];
    auto aread = [&](int buf) {
      const bool kok = kq < KQ;
      const int t = kok ? tap : 4;  // past the reduction: the centre tap (zero weights)
      // tap -> (row + 1, column + 1) from 2-bit tables (no division by 3)
      const int ty1 = (0x2A540 >> (2 * t)) & 3, tx1 = (0x24924 >> (2 * t)) & 3;
      const int toffq = (int)__umul24(ty1, W2q) + (int)__umul24(tx1, qp) - W2q - qp;
      const int cc = kok ? c4 : 0;
#pragma unroll
      for (int i = 0; i < MT; ++i) {
        const int e = pxq[i] + toffq + cc;
        const bb_u32x4 x0 = src[e], x1 = src[splane + e];
        xa[buf][i] = bb_u32x8{x0[0], x0[1], x0[2], x0[3], x1[0], x1[1], x1[2], x1[3]};
      }
      kq += 4;
      c4 += 4;
      const bool wrap = c4 >= Q;
      c4 -= wrap ? Q : 0;
      tap += wrap ? 1 : 0;
    };
    aread(0);
    // nsteps is a multiple of KPF (zero-padded weight quads): whole groups, no early exits
    for (int st0 = 0; st0 < nsteps; st0 += KPF) {
#pragma unroll
      for (int u = 0; u < KPF; ++u) {
        aread((u + 1) & 1);
#pragma unroll
        for (int i = 0; i < MT; ++i) {
          const bb_u32x8& xc = xa[u & 1][i];
#pragma unroll
          for (int j = 0; j < NT; ++j) {
            const bb_u32x8& wc = wr[u][j];
            acc[i][j] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(bb_sub(wc, 2), bb_sub(xc, 0), acc[i][j], 0, 0, 0);  // hh + lh
            acc[i][j] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(bb_sub(wc, 0), bb_sub(xc, 2), acc[i][j], 0, 0, 0);  // mh + hm
            acc[i][j] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(bb_sub(wc, 0), bb_sub(xc, 4), acc[i][j], 0, 0, 0);  // mm + hl
          }
        }
        wload(st0 + u + KPF, u);
      }
    }
    // acc[i][j][r] = channel 16 (n0 + j) + 4 g + r of pixel 16 mt + fr
#pragma unroll
    for (int i = 0; i < MT; ++i) {
      if (mc + mstride * i >= mtt) continue;
      const int p = (mc + mstride * i) * 16 + fr;
      if (p >= P) continue;
#pragma unroll
      for (int j = 0; j < NT; ++j) {
        const int cq = (n0 + j) * 4 + g;
        if (n0 + j < a.ntt && cq < Q) epi(p, cq, acc[i][j]);
      }
    }
  }
}

template <int MT, int NT>
__global__ __launch_bounds__(256) void basic_block_x3_kernel(const BBArgs a) {
  extern __shared__ __attribute__((aligned(16))) bb_u32x4 lds[];
  const int b = blockIdx.x / a.tiles_y, ty = blockIdx.x - (blockIdx.x / a.tiles_y) * a.tiles_y;
  const int y0 = ty * a.T, y1 = min(y0 + a.T, a.H);
  const int W = a.W, W2 = W + 2, Q = a.Q, qp = a.qp;
  // tile rows: input [xr0, xr1), mid [mr0, mr1), clipped to one zero row outside the image
  const int xr0 = max(y0 - 2, -1), xr1 = min(y1 + 2, a.H + 1);
  const int mr0 = max(y0 - 1, -1), mr1 = min(y1 + 1, a.H + 1);
  const int xplane = a.xrows * W2 * qp, mplane = a.mrows * W2 * qp;
  bb_u32x4* X = lds;
  bb_u32x4* Mid = lds + 2 * xplane;
  const float* inb = a.in + (size_t)b * a.H * W * a.in_cs + a.in_co;

  // ---- stage the input rows (split) and zero the mid tile -----------------------------------
  const int nx = (xr1 - xr0) * W2 * Q;
  constexpr int kU = 4;
  for (int e0 = threadIdx.x; e0 < nx; e0 += 256 * kU) {
    f32x4 v[kU];
    int dst[kU];
#pragma unroll
    for (int u = 0; u < kU; ++u) {
      const int e = e0 + 256 * u;
      const int pix = e / Q, c4 = e - (e / Q) * Q;
      const int r = pix / W2, c = pix - (pix / W2) * W2;
      const int y = xr0 + r, x = c - 1;
      const bool ok = e < nx && y >= 0 && y < a.H && x >= 0 && x < W;
      v[u] = ok ? *reinterpret_cast<const f32x4*>(inb + ((size_t)y * W + x) * a.in_cs + 4 * c4) : f32x4{0.f, 0.f, 0.f, 0.f};
      dst[u] = e < nx ? pix * qp + c4 : -1;
    }
#pragma unroll
    for (int u = 0; u < kU; ++u) {
      if (dst[u] < 0) continue;
      bb_u32x4 p0, p1;
      bb_split(v[u], p0, p1);
      X[dst[u]] = p0;
      X[xplane + dst[u]] = p1;
    }
  }
  const int nm = (mr1 - mr0) * W2 * qp;
  for (int e = threadIdx.x; e < nm; e += 256) {
    Mid[e] = bb_u32x4{0u, 0u, 0u, 0u};
    Mid[mplane + e] = bb_u32x4{0u, 0u, 0u, 0u};
  }
  __syncthreads();

  // ---- conv1 on the mid rows inside the image: BN1 + ReLU, split into the mid tile ------------
  const int m0 = max(y0 - 1, 0), m1 = min(y1 + 1, a.H);
  bb_conv<MT, NT>(a, a.w1, X, xplane, m0, xr0, (m1 - m0) * W, [&](int p, int cq, f32x4 acc) {
    const int y = m0 + p / W, x = p - (p / W) * W;
    const f32x4 s = *reinterpret_cast<const f32x4*>(a.s1 + 4 * cq);
    const f32x4 bi = *reinterpret_cast<const f32x4*>(a.b1 + 4 * cq);
    f32x4 v;
#pragma unroll
    for (int r = 0; r < 4; ++r) v[r] = fmaxf(acc[r] * s[r] + bi[r], 0.f);
    bb_u32x4 p0, p1;
    bb_split(v, p0, p1);
    const int d = ((y - mr0) * W2 + x + 1) * qp + cq;
    Mid[d] = p0;
    Mid[mplane + d] = p1;
  });
  __syncthreads();

  // ---- conv2 on the output rows: BN2 + residual + ReLU -> out ----------------------------------
  float* ob = a.out + (size_t)b * a.H * W * a.out_cs + a.out_co;
  bb_conv<MT, NT>(a, a.w2, Mid, mplane, y0, mr0, (y1 - y0) * W, [&](int p, int cq, f32x4 acc) {
    const int y = y0 + p / W, x = p - (p / W) * W;
    const f32x4 s = *reinterpret_cast<const f32x4*>(a.s2 + 4 * cq);
    const f32x4 bi = *reinterpret_cast<const f32x4*>(a.b2 + 4 * cq);
    const f32x4 res = *reinterpret_cast<const f32x4*>(inb + ((size_t)y * W + x) * a.in_cs + 4 * cq);
    f32x4 v;
#pragma unroll
    for (int r = 0; r < 4; ++r) v[r] = fmaxf(acc[r] * s[r] + bi[r] + res[r], 0.f);
    *reinterpret_cast<f32x4*>(ob + ((size_t)y * W + x) * a.out_cs + 4 * cq) = v;
  });
}

long long bb_lds_bytes(int T, int H, int W, int Q) {
  const int qp = Q | 1;
  const int xr = min(T + 4, H + 2), mr = min(T + 2, H + 2);
  return 2LL * (xr + mr) * (W + 2) * qp * 16;
}

}  // namespace

KRRN_API int krrn_basic_block_x3_f32(const float* in, int in_cs, int in_co, int B, int H, int W, int C,
                                     const void* w1, const float* s1, const float* b1, const void* w2,
                                     const float* s2, const float* b2, float* out, int out_cs, int out_co, int T,
                                     void* stream) {
  if (!in || !w1 || !w2 || !s1 || !b1 || !s2 || !b2 || !out) return KRRN_EARG;
  if (B < 1 || H < 1 || W < 1 || T < 1 || C < 16) return KRRN_ESHAPE;  // Q >= 4 (one wrap per step)
  if ((C & 3) || (in_cs & 3) || (in_co & 3) || (out_cs & 3) || (out_co & 3) || in_co + C > in_cs ||
      out_co + C > out_cs)
    return KRRN_EALIGN;
  if (!krrn_aligned16(in) || !krrn_aligned16(out) || !krrn_aligned16(w1) || !krrn_aligned16(w2) ||
      !krrn_aligned16(s1) || !krrn_aligned16(b1) || !krrn_aligned16(s2) || !krrn_aligned16(b2))
    return KRRN_EALIGN;
  if ((const void*)in == (const void*)out) return KRRN_EARG;  // the residual is re-read from `in`
  if ((long long)B * H * W * in_cs >= (1LL << 31) || (long long)B * H * W * out_cs >= (1LL << 31)) return KRRN_ESHAPE;
  const long long lds = bb_lds_bytes(T, H, W, C / 4);
  if (lds > 160 * 1024) return KRRN_ESHAPE;
  BBArgs a;
  a.in = in; a.in_cs = in_cs; a.in_co = in_co; a.B = B; a.H = H; a.W = W; a.Q = C / 4; a.T = T;
  a.tiles_y = krrn_cdiv(H, T);
  a.qp = a.Q | 1;
  a.xrows = min(T + 4, H + 2);
  a.mrows = min(T + 2, H + 2);
  a.w1 = reinterpret_cast<const unsigned*>(w1);
  a.w2 = reinterpret_cast<const unsigned*>(w2);
  a.kqp = krrn_cdiv(9 * a.Q, 16) * 16;
  a.s1 = s1; a.b1 = b1; a.s2 = s2; a.b2 = b2;
  a.out = out; a.out_cs = out_cs; a.out_co = out_co;
  a.ntt = krrn_cdiv(C, 16);
  a.nsplit = a.ntt >= 4;
  if ((long long)B * a.tiles_y > 0x7fffffffLL) return KRRN_ESHAPE;
  // per-wave register tiles: channel-split NT = ceil(ntt / 4), pixel-split NT = ntt (<= 3)
  const int nt = a.nsplit ? krrn_cdiv(a.ntt, 4) : a.ntt;
  const int P1 = min(T + 2, H) * W;  // conv1 pixels of the largest block
  const int mtt = krrn_cdiv(P1, 16);
  const int mt = a.nsplit ? min(mtt, 3) : min(krrn_cdiv(mtt, 4), 3);
  hipStream_t s = (hipStream_t)stream;
  const dim3 grid((unsigned)(B * a.tiles_y)), blk(256);
#define KRRN_BB(MTV, NTV)                                                                              \
  if (mt == MTV && nt == NTV) {                                                                        \
    if (lds > 64 * 1024) {                                                                             \
      const hipError_t e = hipFuncSetAttribute((const void*)basic_block_x3_kernel<MTV, NTV>,          \
                                               hipFuncAttributeMaxDynamicSharedMemorySize, (int)lds); \
      if (e != hipSuccess) return (int)e;                                                              \
    }                                                                                                  \
    hipLaunchKernelGGL((basic_block_x3_kernel<MTV, NTV>), grid, blk, (size_t)lds, s, a);               \
    return krrn_launch_status();                                                                       \
  }
  KRRN_BB(1, 1) KRRN_BB(2, 1) KRRN_BB(3, 1)
  KRRN_BB(1, 2) KRRN_BB(2, 2) KRRN_BB(3, 2)
  KRRN_BB(1, 3) KRRN_BB(2, 3) KRRN_BB(3, 3)
  KRRN_BB(1, 4) KRRN_BB(2, 4) KRRN_BB(3, 4)
#undef KRRN_BB
  return KRRN_ESHAPE;  // more than 64 channel tiles per wave range (C > 256)
}
