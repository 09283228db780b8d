// Winograd F(4x4, 3x3) convolution on the bf16 matrix cores at f32 accuracy (split-bf16, as in
// winograd.hip), for the heads' wide 128 -> 128 3x3 convs at S/2 and S (XYZNet / NMLNet,
// lib/network/krrn.py:52-63, 74-81).
//
//   per 4x4 output tile t and input channel c: V = B^T d B      (d = the 6x6 input patch, pad 0)
//   per output channel n:                      U = G g G^T      (host, f64, once per plan)
//   M[xi][t][n] = sum_c V[xi][t][c] U[xi][c][n]                 (36 GEMMs, xi = 6u + v)
//   Y = A^T M A (4x4), then out = act(scale[n] * Y + bias[n] (+ res))
//
// with points (0, +-1, +-2) (Lavin & Gray 2016):
//   B^T = [4 0 -5 0 1 0; 0 -4 -4 1 1 0; 0 4 -4 -1 1 0; 0 -2 -1 2 1 0; 0 2 -1 -2 1 0; 0 4 0 -5 0 1]
//   A^T = [1 1 1 1 1 0; 0 1 -1 2 -2 0; 0 1 1 4 4 0; 0 1 -1 8 -8 1]
// 36 products per 16 outputs: 2.25 per output against 4 for F(2x2) and 9 for the direct conv.
//
// Why this block. The F(2x2) kernel moves ~30 B/clk/CU from L2 (TA busy
// 75 %, PMC), 86 % of it split weights: each weight is reused over the 32 tiles = 128 output pixels
// of a wave's MFMA rows, 0.75 B of weights per output MAC. Here a wave's weight registers serve 32
// tiles = 512 output pixels: 36 * 6 B / 512 = 0.42 B per output MAC. Accumulators: 36 components x
// 32 tiles x 64 channels = 9 components x one 32x32 accumulator per wave over 8 waves (144 registers
// each, 2 waves per SIMD, one block per CU). The input transform is done ONCE per (tile, channel)
// for all 64 output channels of the block, by the block cooperatively, into LDS:
//
//   block = 16 x 2 tiles (64 x 8 output pixels of one image) x 64 output channels, 512 threads.
//   Per 8-channel chunk ck (one barrier per chunk):
//     raw  : the 10 x 66 x 8 input region of chunk ck + 2 goes by LDS-DMA (3 buffer_load ... lds
//            per wave, no staging registers) into a 2-slot ring (padded slots: conflict-free patch
//            reads), requested after component 6 of chunk ck;
//     T    : the transform of chunk ck + 1, interleaved with M(ck) (its steps sit in the MFMA gaps of
//            each component): waves 0..5 own columns v = 0..5 of the 6x6 transform (waves 6, 7
//            only multiply; KRRN_W4_TSPLIT); lane (tile, channel
//            half h) forms e[r] = B_v(d[r][.]) for the 6 patch rows, then V[u][v] = B_u(e[.]), splits
//            each into the three bf16 terms and writes the MFMA operand chain [V_m V_h | V_l]
//            (b128 + b64) to a 2-slot V buffer; V[comp][h][tile] = lane order, so the consumer's read
//            is the producer's write address;
//     M    : wave (g = wave & 3, nh = wave >> 2) owns the 3x3 component sub-grid g
//            (u in 3(g>>1)+0..2, v in 3(g&1)+0..2) for output channels 32 nh .. +31: per component
//            one b128 + one b64 V read (one component ahead), three v_mfma_f32_32x32x16_bf16
//            (mm+hh, mh+hl, hm+lh as in winograd.hip), then the weights of the component 3 ahead
//            are loaded into a rolling 3-component register buffer.
//   Epilogue: 2 passes of 16 tiles through LDS ([comp][tile][n]); thread (channel quad, tile, output
//   row i) forms t[v] = A_i(M[.][v]) and Y[i][j] = A_j(t), applies BN / bias / residual / ReLU and
//   stores float4 channel runs.
// Where the time goes (profiles/w4_trace.py, per-wave cycle stamps): the chunk
// loop 75 %, the epilogue 14 % (VALU-bound A^T transform), the prologue 8 %; the chip runs at
// ~1.5 GHz under this kernel against ~2.1 GHz with either the MFMAs or the transform removed.
#include <type_traits>

#include "krrn_common.h"

namespace {

typedef __bf16 bf16x8 __attribute__((ext_vector_type(8)));
typedef __bf16 bf16x2 __attribute__((ext_vector_type(2)));
typedef float f32x2 __attribute__((ext_vector_type(2)));
typedef unsigned u32x4 __attribute__((ext_vector_type(4)));
typedef unsigned u32x2 __attribute__((ext_vector_type(2)));
typedef unsigned u32x3 __attribute__((ext_vector_type(3)));
typedef unsigned u32x6 __attribute__((ext_vector_type(6)));

constexpr int kGX = 16, kGY = 2, kT = kGX * kGY;  // tiles per block
constexpr int kN = 64;                            // output channels per block
constexpr int kC = 8;                             // input channels per chunk
constexpr int kRR = 4 * kGY + 2, kRC = 4 * kGX + 2;  // raw rows / cols: 10 x 66
constexpr int kRS = 152;                          // 16-B slots per raw row: 2 col + h + col / 4, padded
constexpr int kRing = 1536;                       // slots per ring slot (10 x 152 = 1520, 3 per thread)
constexpr int kRingF = kRing * 4;                 // floats per ring slot
constexpr int kVMH = 36 * 64 * 4;                 // u32 per V buffer, plane [V_m V_h]
constexpr int kVL = 36 * 64 * 2;                  // u32 per V buffer, plane [V_l]
constexpr int kET = kN * 4;                       // epilogue bytes per (component, tile): [64 n] f32
constexpr unsigned kOOB = 0xFFFF0000u;
// timing experiments only (results wrong; profiles/build_variant.sh), a bit mask: 1 no MFMAs, 2 no weight reloads,
// 4 no transform, 8 no raw staging after the prologue, 16 no epilogue, 32 no output stores,
// 64 one transform tap read per patch row (the VALU unchanged)
#ifndef KRRN_W4_EXP
#define KRRN_W4_EXP 0
#endif
#ifndef KRRN_W4_TSPLIT
// 0 (default): waves 0-5 own transform columns 0-5, waves 6, 7 skip the transform; 1: waves 4 / 6 and
// 5 / 7 split columns 4 / 5 (each SIMD the same transform VALU, but both waves of a pair redo the
// column's row steps): 0.9 % slower under sustained load (760 vs 753 us per 120-px launch)
#define KRRN_W4_TSPLIT 0
#endif
#ifndef KRRN_W4_TPAIR
// 1: waves 2 pr + h (pr < 3) transform the column pair (2 pr, 2 pr + 1) of channel half h, one channel
// pair per lane: 5 ds_read_b64 per patch row shared by both columns instead of 4 ds_read_b128 per column
// (-37 % transform LDS-array cycles, but 6 ds_write_b32 per output for 2): 0.8 % slower under sustained
// load (762 / 765 vs 756 / 759 us per 120-px launch, profiles/r6_tpair_ab.txt), so 0 (default)
#define KRRN_W4_TPAIR 0
#endif
static_assert(!(KRRN_W4_TPAIR && KRRN_W4_TSPLIT), "one transform split");
#ifndef KRRN_W4_SKIP3
// 1: waves 0 / 5 skip the zero-coefficient 4th tap read of rows 1-5. The uniform branch splits the
// chunk body's scheduling regions: 1.9 % slower under sustained load (772 vs 758 us, r6_w4_skip3_ab.txt)
#define KRRN_W4_SKIP3 0
#endif
#ifndef KRRN_W4_TRACE
#define KRRN_W4_TRACE 0  // 1: per-wave cycle stamps of the first 256 blocks (profiles/w4_trace.py; timing study only)
#endif
#ifndef KRRN_W4_RAWK
#define KRRN_W4_RAWK 6
#endif
#ifndef KRRN_W4_GAP
#define KRRN_W4_GAP 6
#endif
constexpr int kRawK = KRRN_W4_RAWK;  // component slot after which the raw chunk two ahead is requested
constexpr int kGap = KRRN_W4_GAP;    // transform VALU instructions placed in each MFMA gap
static_assert(kRR * kRS <= kRing && kRing == 3 * 512, "raw ring");
static_assert(2 * (kRC - 1) + 1 + (kRC - 1) / 4 < kRS && (kRS * 4) % 16 == 0, "padded raw row");
// LDS bytes: V plane MH x 2 | V plane L x 2 | raw ring x 2 (the epilogue's [36][64][12] f32 reuses
// the V planes). Every access is one per-lane base register + a compile-time offset < 64 KB.
constexpr int kOffL = 2 * kVMH * 4;              // 73728
constexpr int kOffR = kOffL + 2 * kVL * 4;       // 110592
constexpr int kLdsBytes = kOffR + 2 * kRingF * 4;  // 159744
static_assert(36 * 16 * kET <= kLdsBytes, "epilogue (16 tiles) fits the LDS");

struct Wino4Args {
  const float* in;
  int in_cs, in_co;
  int B, H, W, cin;
  long long img;    // elements per input image
  const void* U3;   // split weights: plane MH [nck][36][N][2][16 B], then plane L [..][8 B]
  int N, n_store;
  const float* scale;
  const float* bias;
  const float* res;
  int res_cs, res_co;
  float* out;
  int out_cs, out_co;
  int relu;
  int vec;          // out / res / scale / bias allow float4 channel runs
  int Ht, Wt;       // tiles per column / row
  // head form (krrn_conv3x3_wino4_x3_head_f32): the activated conv output is not stored; its dot with
  // the 4 rows of w1 ([4][N], the following 1x1 conv) over this block's 64 channels goes to
  // part[nb][pixel][4], summed over the n-blocks in order by wino4_head_finish_kernel
  const float* w1;
  float* part;
};

// x of the lane the DPP control names (within a row of 16 lanes)
template <int CTRL>
__device__ __forceinline__ float dpp_f(float x) {
  return __int_as_float(__builtin_amdgcn_update_dpp(0, __float_as_int(x), CTRL, 0xF, 0xF, false));
}

__device__ __forceinline__ unsigned pk_bf16(float a, float b) {
  return __builtin_bit_cast(unsigned, __builtin_convertvector(f32x2{a, b}, bf16x2));  // RNE
}
__device__ __forceinline__ float bf_lo(unsigned p) { return __builtin_bit_cast(float, p << 16); }
__device__ __forceinline__ float bf_hi(unsigned p) { return __builtin_bit_cast(float, p & 0xFFFF0000u); }

// x (4 channels) -> the operand chain [x_m x_h x_l] as packed bf16 pairs (winograd.hip split3_chain)
__device__ __forceinline__ u32x6 split3(const f32x4 x) {
  const unsigned h0 = pk_bf16(x[0], x[1]), h1 = pk_bf16(x[2], x[3]);
  const float r0 = x[0] - bf_lo(h0), r1 = x[1] - bf_hi(h0);
  const float r2 = x[2] - bf_lo(h1), r3 = x[3] - bf_hi(h1);
  const unsigned m0 = pk_bf16(r0, r1), m1 = pk_bf16(r2, r3);
  const unsigned l0 = pk_bf16(r0 - bf_lo(m0), r1 - bf_hi(m0)), l1 = pk_bf16(r2 - bf_lo(m1), r3 - bf_hi(m1));
  return u32x6{m0, m1, h0, h1, l0, l1};
}

__device__ __forceinline__ bf16x8 sub4(const u32x6& c, int o) {
  return __builtin_bit_cast(bf16x8, u32x4{c[o], c[o + 1], c[o + 2], c[o + 3]});
}

// x (a channel pair) -> its packed bf16 terms {m, h, l}
__device__ __forceinline__ u32x3 split3_pair(const f32x2 x) {
  const unsigned hh = pk_bf16(x[0], x[1]);
  const float r0 = x[0] - bf_lo(hh), r1 = x[1] - bf_hi(hh);
  const unsigned m = pk_bf16(r0, r1);
  return u32x3{m, hh, pk_bf16(r0 - bf_lo(m), r1 - bf_hi(m))};
}

// row K of B^T applied to x[0..5] (scalar f32, element-wise over the vector's channels)
template <int K, typename V>
__device__ __forceinline__ V bt_row(const V (&x)[6]) {
  V y;
#pragma unroll
  for (int e = 0; e < (int)(sizeof(V) / 4); ++e) {
    if constexpr (K == 0) y[e] = __builtin_fmaf(4.f, x[0][e], __builtin_fmaf(-5.f, x[2][e], x[4][e]));
    if constexpr (K == 1) y[e] = __builtin_fmaf(-4.f, x[1][e] + x[2][e], x[3][e] + x[4][e]);
    if constexpr (K == 2) y[e] = __builtin_fmaf(4.f, x[1][e] - x[2][e], x[4][e] - x[3][e]);
    if constexpr (K == 3) y[e] = __builtin_fmaf(2.f, x[3][e] - x[1][e], x[4][e] - x[2][e]);
    if constexpr (K == 4) y[e] = __builtin_fmaf(2.f, x[1][e] - x[3][e], x[4][e] - x[2][e]);
    if constexpr (K == 5) y[e] = __builtin_fmaf(4.f, x[1][e], __builtin_fmaf(-5.f, x[3][e], x[5][e]));
  }
  return y;
}
// the columns row K of B^T reads
template <int K>
__device__ __forceinline__ constexpr bool bt_uses(int c) {
  return K == 0 ? (c == 0 || c == 2 || c == 4) : (K == 5 ? (c == 1 || c == 3 || c == 5) : (c >= 1 && c <= 4));
}

// row I of A^T applied to x[0..5]
template <int I>
__device__ __forceinline__ f32x4 at_row(const f32x4 (&x)[6]) {
  f32x4 y;
#pragma unroll
  for (int e = 0; e < 4; ++e) {
    if constexpr (I == 0) y[e] = ((x[0][e] + x[1][e]) + x[2][e]) + (x[3][e] + x[4][e]);
    if constexpr (I == 1) y[e] = __builtin_fmaf(2.f, x[3][e] - x[4][e], x[1][e] - x[2][e]);
    if constexpr (I == 2) y[e] = __builtin_fmaf(4.f, x[3][e] + x[4][e], x[1][e] + x[2][e]);
    if constexpr (I == 3) y[e] = __builtin_fmaf(8.f, x[3][e] - x[4][e], x[1][e] - x[2][e]) + x[5][e];
  }
  return y;
}
template <int I>
__device__ __forceinline__ constexpr bool at_uses(int u) {
  return I == 0 ? (u <= 4) : (I == 3 ? (u >= 1) : (u >= 1 && u <= 4));
}

// epilogue: output row I of local tile tl (of the pass's 16), channels ng .. ng + 3;
// E = [36][16 tiles][64 n] f32
template <int I, int HP>
__device__ __forceinline__ void epi_row(const Wino4Args& a, const char* E, int nq, int tl, int pass, int b, int ty0,
                                        int tx0, int ng, int nb) {
  const char* eb = E + tl * kET + nq * 16;
  f32x4 t[6];
#pragma unroll
  for (int v = 0; v < 6; ++v) {
    f32x4 m[6];
#pragma unroll
    for (int u = 0; u < 6; ++u)
      m[u] = at_uses<I>(u) ? *reinterpret_cast<const f32x4*>(eb + (6 * u + v) * 16 * kET) : f32x4{0.f, 0.f, 0.f, 0.f};
    t[v] = at_row<I>(m);
    asm volatile("" : "+v"(t[v])::"memory");  // one column's reads at a time (register budget)
  }
  f32x4 y[4];  // y[j]: output column j, 4 channels
  y[0] = at_row<0>(t);
  y[1] = at_row<1>(t);
  y[2] = at_row<2>(t);
  y[3] = at_row<3>(t);
  const int tile = 16 * pass + tl;
  const int ty = ty0 + (tile >> 4), tx = tx0 + (tile & 15);
  const int oy = 4 * ty + I;
  const int nj = min(4, a.W - 4 * tx);  // output columns of this tile inside the image
  if constexpr (HP > 0) {
    // the 16 lanes of a DPP row are the 16 channel quads of one tile: every lane takes part in the
    // row sums (no early exit), invalid pixels / channels contribute zeros
    const bool ok = ty < a.Ht && oy < a.H && nj > 0 && ng < a.n_store;  // n_store = N % 4 == 0
    const f32x4 zero = {0.f, 0.f, 0.f, 0.f};
    const f32x4 scl = ok && a.scale ? *reinterpret_cast<const f32x4*>(a.scale + ng) : f32x4{1.f, 1.f, 1.f, 1.f};
    const f32x4 bia = ok && a.bias ? *reinterpret_cast<const f32x4*>(a.bias + ng) : zero;
    f32x4 w[HP];
#pragma unroll
    for (int o = 0; o < HP; ++o) w[o] = ok ? *reinterpret_cast<const f32x4*>(a.w1 + (size_t)o * a.N + ng) : zero;
    const long long pix = ((long long)b * a.H + oy) * a.W + 4 * tx;
    float s[4][HP];  // this lane's 4-channel partial dot of pixel j with w1 row o
#pragma unroll
    for (int j = 0; j < 4; ++j) {
      const bool okj = ok && j < nj;
      f32x4 v;
#pragma unroll
      for (int e = 0; e < 4; ++e) v[e] = __builtin_fmaf(y[j][e], scl[e], bia[e]);
      if (a.res && okj) v += *reinterpret_cast<const f32x4*>(a.res + (pix + j) * a.res_cs + a.res_co + ng);
      if (a.relu) {
#pragma unroll
        for (int e = 0; e < 4; ++e) v[e] = fmaxf(v[e], 0.f);
      }
      if (!okj) v = zero;
#pragma unroll
      for (int o = 0; o < HP; ++o) s[j][o] = v[0] * w[o][0] + v[1] * w[o][1] + v[2] * w[o][2] + v[3] * w[o][3];
    }
    // sum over the 16 channel quads as a reduce-scatter: two exchange levels leave lane nq the 4-lane
    // partials of pixel j = nq & 3 (the partner gets the other half of the values), two rotations
    // of the DPP row then add the 4 lanes of each class
    const bool b0 = nq & 1, b1 = (nq >> 1) & 1;
    float t1[2][HP];
#pragma unroll
    for (int jj = 0; jj < 2; ++jj)
#pragma unroll
      for (int o = 0; o < HP; ++o) {
        const float keep = b0 ? s[2 * jj + 1][o] : s[2 * jj][o], send = b0 ? s[2 * jj][o] : s[2 * jj + 1][o];
        t1[jj][o] = keep + dpp_f<0xB1>(send);  // quad [1 0 3 2]
      }
    float t2[HP];
#pragma unroll
    for (int o = 0; o < HP; ++o) {
      const float keep = b1 ? t1[1][o] : t1[0][o], send = b1 ? t1[0][o] : t1[1][o];
      t2[o] = keep + dpp_f<0x4E>(send);  // quad [2 3 0 1]
      t2[o] += dpp_f<0x128>(t2[o]);      // row_ror 8
      t2[o] += dpp_f<0x124>(t2[o]);      // row_ror 4
    }
    const int j = nq & 3;
    if (nq >= 4 || !(ty < a.Ht && oy < a.H && j < nj)) return;
    const long long M = (long long)a.B * a.H * a.W;
    f32x4 r = {0.f, 0.f, 0.f, 0.f};
#pragma unroll
    for (int o = 0; o < HP; ++o) r[o] = t2[o];
    *reinterpret_cast<f32x4*>(a.part + ((size_t)nb * M + pix + j) * 4) = r;
    return;
  }
  if (ty >= a.Ht || oy >= a.H || nj <= 0 || ng >= a.n_store) return;
  const long long pix = ((long long)b * a.H + oy) * a.W + 4 * tx;
  float* o = a.out + pix * a.out_cs + a.out_co + ng;
  const float* rs = a.res ? a.res + pix * a.res_cs + a.res_co + ng : nullptr;
  if (a.vec && ng + 4 <= a.n_store) {
    const f32x4 scl = a.scale ? *reinterpret_cast<const f32x4*>(a.scale + ng) : f32x4{1.f, 1.f, 1.f, 1.f};
    const f32x4 bia = a.bias ? *reinterpret_cast<const f32x4*>(a.bias + ng) : f32x4{0.f, 0.f, 0.f, 0.f};
#pragma unroll
    for (int j = 0; j < 4; ++j) {
      if (j >= nj) break;
      f32x4 v;
#pragma unroll
      for (int e = 0; e < 4; ++e) v[e] = __builtin_fmaf(y[j][e], scl[e], bia[e]);
      if (rs) v += *reinterpret_cast<const f32x4*>(rs + j * a.res_cs);
      if (a.relu) {
#pragma unroll
        for (int e = 0; e < 4; ++e) v[e] = fmaxf(v[e], 0.f);
      }
      if (!(KRRN_W4_EXP & 32) || v[0] == 1234.5f) *reinterpret_cast<f32x4*>(o + j * a.out_cs) = v;
    }
    return;
  }
#pragma unroll
  for (int e = 0; e < 4; ++e) {
    if (ng + e >= a.n_store) break;
    const float scl = a.scale ? a.scale[ng + e] : 1.f, bia = a.bias ? a.bias[ng + e] : 0.f;
#pragma unroll
    for (int j = 0; j < 4; ++j) {
      if (j >= nj) break;
      float v = __builtin_fmaf(y[j][e], scl, bia);
      if (rs) v += rs[j * a.res_cs + e];
      if (a.relu) v = fmaxf(v, 0.f);
      o[j * a.out_cs + e] = v;
    }
  }
}

// out[b][o][p] = sum over n-blocks (in order) of part[nb][b * HW + p][o] + b1[o], o < p1
__global__ __launch_bounds__(256) void wino4_head_finish_kernel(const float* __restrict__ part, int nbn, long long M,
                                                                int HW, const float* __restrict__ b1, int p1,
                                                                float* __restrict__ out, int out_c) {
  const long long m = (long long)blockIdx.x * 256 + threadIdx.x;
  if (m >= M) return;
  f32x4 v = *reinterpret_cast<const f32x4*>(part + m * 4);
  for (int nb = 1; nb < nbn; ++nb) v += *reinterpret_cast<const f32x4*>(part + ((size_t)nb * M + m) * 4);
  const long long b = m / HW, p = m - b * HW;
#pragma unroll
  for (int o = 0; o < 4; ++o)
    if (o < p1) out[(b * out_c + o) * HW + p] = v[o] + (b1 ? b1[o] : 0.f);
}

#if KRRN_W4_TRACE
constexpr int kTrN = 52;  // per wave: [16 chunks][start, after component 4, before the barrier], 4 more
__device__ unsigned g_w4_trace[256 * 8 * kTrN];
#define W4_MARK(i)                                                  \
  do {                                                              \
    const unsigned t_ = (unsigned)__builtin_readcyclecounter();     \
    if (lane == 0 && (i) < kTrN) trace_lds[wave * kTrN + (i)] = t_; \
  } while (0)
#else
#define W4_MARK(i) \
  do {             \
  } while (0)
#endif

template <int HP>  // 0: conv output stored; 1..4: head form, HP rows of w1
__global__ __launch_bounds__(512, 1) void wino_f43_x3_kernel(const Wino4Args a) {
  __shared__ __attribute__((aligned(16))) char smem[kLdsBytes];
  const int tid = threadIdx.x, lane = tid & 63;
  const int wave = __builtin_amdgcn_readfirstlane(tid >> 6);
#if KRRN_W4_TRACE
  __shared__ unsigned trace_lds[8 * kTrN];
#endif
  W4_MARK(48);
  const int gxn = krrn_cdiv(a.Wt, kGX), gyn = krrn_cdiv(a.Ht, kGY), nbn = krrn_cdiv(a.N, kN);
  const int per_img = gxn * gyn;
  const int bid = krrn_xcd_remap(blockIdx.x, a.B * per_img * nbn);
  const int sp = bid / nbn, nb = bid - (bid / nbn) * nbn;
  const int b = sp / per_img, r2 = sp - (sp / per_img) * per_img;
  const int by = r2 / gxn, bx = r2 - (r2 / gxn) * gxn;
  const int n0 = nb * kN;
  const int ty0 = by * kGY, tx0 = bx * kGX;
  const int nck = a.cin / kC;

  // raw staging: this thread's 3 ring slots t, t + 512, t + 1024 (padding slots load zeros)
  const __amdgpu_buffer_rsrc_t rsA = __builtin_amdgcn_make_buffer_rsrc(
      (void*)(a.in + (size_t)b * a.img + a.in_co), (short)0, (int)min(a.img * 4 - (long long)a.in_co * 4, 0x7FFFFFFFLL),
      0x00020000);
  unsigned roff[3];
#pragma unroll
  for (int i = 0; i < 3; ++i) {
    const int s = 192 * wave + 64 * i + lane;  // LDS-DMA: wave instruction i fills slots 64 (3 wave + i) ..
    const int r = s / kRS, q = s - (s / kRS) * kRS;
    const int g4 = q / 9, w9 = q - (q / 9) * 9;
    const int col = 4 * g4 + (w9 >> 1), hh = w9 & 1;
    const int iy = 4 * ty0 - 1 + r, ix = 4 * tx0 - 1 + col;
    const bool ok = r < kRR && w9 < 8 && col < kRC && iy >= 0 && iy < a.H && ix >= 0 && ix < a.W;
    roff[i] = ok ? (unsigned)((((long long)iy * a.W + ix) * a.in_cs + 4 * hh) * 4) : kOOB;
  }
  // raw chunk ck straight into ring slot `slot` by LDS-DMA (buffer_load_dwordx4 ... lds: 1 KB per
  // wave instruction, no staging registers); padding slots receive zeros
  auto dma_raw = [&](int ck, int slot) {
    char* dst = smem + kOffR + slot * (kRingF * 4) + 3 * 1024 * wave;
#pragma unroll
    for (int i = 0; i < 3; ++i)
      __builtin_amdgcn_raw_ptr_buffer_load_lds(rsA, (__attribute__((address_space(3))) void*)(dst + 1024 * i), 16,
                                               roff[i], ck * kC * 4, 0, 0);
  };

  // M: wave (g, nh), components (u, v) = (3 (g >> 1) + k / 3, 3 (g & 1) + k % 3), k = 0..8
  const int g = wave & 3, nh = wave >> 2;
  const int cu0 = 3 * (g >> 1), cv0 = 3 * (g & 1);
  const int fr = lane & 31, h = lane >> 5;
  const long long nrec = (long long)nck * 36 * a.N * 2;
  const char* u3 = reinterpret_cast<const char*>(a.U3);
  const __amdgpu_buffer_rsrc_t rsMH =
      __builtin_amdgcn_make_buffer_rsrc((void*)u3, (short)0, (int)min(nrec * 16, 0x7FFFFFFFLL), 0x00020000);
  const __amdgpu_buffer_rsrc_t rsL =
      __builtin_amdgcn_make_buffer_rsrc((void*)(u3 + nrec * 16), (short)0, (int)min(nrec * 8, 0x7FFFFFFFLL), 0x00020000);
  const unsigned wrec = (unsigned)(2 * min(n0 + 32 * nh + fr, a.N - 1) + h);  // lanes past N read channel N-1
  // weights: a rolling buffer of 3 components (slot k % 3); component k + 3 (or k - 6 of the next
  // chunk) is loaded as soon as component k's MFMAs have issued
  u32x4 wmh[3];
  u32x2 wl[3];
  auto load_w = [&](int ck, int k) {
    ck = min(ck, nck - 1);
    const int comp = 6 * (cu0 + k / 3) + cv0 + k % 3;
    const unsigned srec = (unsigned)((ck * 36 + comp) * a.N * 2);  // uniform
    wmh[k % 3] = __builtin_bit_cast(u32x4, __builtin_amdgcn_raw_buffer_load_b128(rsMH, wrec * 16u, srec * 16u, 0));
    wl[k % 3] = __builtin_bit_cast(u32x2, __builtin_amdgcn_raw_buffer_load_b64(rsL, wrec * 8u, srec * 8u, 0));
  };

  f32x16 acc[9];
#pragma unroll
  for (int k = 0; k < 9; ++k)
#pragma unroll
    for (int r = 0; r < 16; ++r) acc[k][r] = 0.f;

#if KRRN_W4_TPAIR
  // T, column pairs: wave 2 pr + th (pr < 3) transforms columns 2 pr and 2 pr + 1 of channel half th;
  // lane (tile = lane >> 1, channel pair tq = lane & 1) reads 5 taps per patch row as f32x2 (one tile
  // row per 32-lane ds_read_b64 group: 16 slots 36 dwords apart x 2 halves, conflict-free) in an order
  // where column 2 pr takes taps 0..3 and column 2 pr + 1 taps 1..4 (the pair (2, 3) reads tap 1 twice),
  // and writes each output's m / h / l bf16 pairs into the consumer's chain entry (16 tiles x 2 pairs
  // per 32-lane ds_write_b32 group: 2-way, free)
  const int tpr = wave < 6 ? wave >> 1 : 0, th = wave & 1;
  const int ttile = lane >> 1, tq = lane & 1;
  int tcol[5];
  float ka[4], kb[4];
  switch (tpr) {
    case 0:  // 4 d0 - 5 d2 + d4 | -4 (d1 + d2) + d3 + d4
      tcol[0] = 0; tcol[1] = 2; tcol[2] = 4; tcol[3] = 1; tcol[4] = 3;
      ka[0] = 4.f; ka[1] = -5.f; ka[2] = 1.f; ka[3] = 0.f; kb[0] = -4.f; kb[1] = 1.f; kb[2] = -4.f; kb[3] = 1.f;
      break;
    case 1:  // 4 (d1 - d2) + d4 - d3 | 2 (d3 - d1) + d4 - d2
      tcol[0] = 1; tcol[1] = 2; tcol[2] = 3; tcol[3] = 4; tcol[4] = 1;
      ka[0] = 4.f; ka[1] = -4.f; ka[2] = -1.f; ka[3] = 1.f; kb[0] = -1.f; kb[1] = 2.f; kb[2] = 1.f; kb[3] = -2.f;
      break;
    default:  // 2 (d1 - d3) + d4 - d2 | 4 d1 - 5 d3 + d5
      tcol[0] = 2; tcol[1] = 4; tcol[2] = 1; tcol[3] = 3; tcol[4] = 5;
      ka[0] = -1.f; ka[1] = 1.f; ka[2] = 2.f; ka[3] = -2.f; kb[0] = 0.f; kb[1] = 4.f; kb[2] = -5.f; kb[3] = 1.f;
      break;
  }
  const int pbase = (4 * (ttile >> 4)) * kRS + 9 * (ttile & 15) + th;  // patch origin slot
  const char* tb[5];
  char* twm = nullptr;  // this lane's word in the V entry of component 2 pr (plane MH)
  char* twl = nullptr;  // (plane L)
  f32x2 td[5], tea[6], teb[6];
  auto t_begin = [&](int ck) {
    const int p = ck & 1;
    const char* rb = smem + kOffR + p * (kRingF * 4) + 16 * pbase + 8 * tq;
#pragma unroll
    for (int t = 0; t < 5; ++t) tb[t] = rb + 16 * (2 * tcol[t] + (tcol[t] >> 2));
    twm = smem + p * (kVMH * 4) + 2 * tpr * 1024 + 16 * (32 * th + ttile) + 4 * tq;
    twl = smem + kOffL + p * (kVL * 4) + 2 * tpr * 512 + 8 * (32 * th + ttile) + 4 * tq;
#pragma unroll
    for (int t = 0; t < 5; ++t) td[t] = *reinterpret_cast<const f32x2*>(tb[t]);
  };
  auto t_step = [&](int s) {
    if (s < 6) {
#pragma unroll
      for (int e = 0; e < 2; ++e) {
        tea[s][e] = __builtin_fmaf(ka[3], td[3][e], __builtin_fmaf(ka[2], td[2][e], __builtin_fmaf(ka[1], td[1][e], ka[0] * td[0][e])));
        teb[s][e] = __builtin_fmaf(kb[3], td[4][e], __builtin_fmaf(kb[2], td[3][e], __builtin_fmaf(kb[1], td[2][e], kb[0] * td[1][e])));
      }
      if (s < 5) {
#pragma unroll
        for (int t = 0; t < 5; ++t) td[t] = *reinterpret_cast<const f32x2*>(tb[t] + (s + 1) * kRS * 16);
      }
      return;
    }
    const int u = s - 6;
    f32x2 xa, xb;
    switch (u) {
      case 0: xa = bt_row<0>(tea); xb = bt_row<0>(teb); break;
      case 1: xa = bt_row<1>(tea); xb = bt_row<1>(teb); break;
      case 2: xa = bt_row<2>(tea); xb = bt_row<2>(teb); break;
      case 3: xa = bt_row<3>(tea); xb = bt_row<3>(teb); break;
      case 4: xa = bt_row<4>(tea); xb = bt_row<4>(teb); break;
      default: xa = bt_row<5>(tea); xb = bt_row<5>(teb); break;
    }
    const u32x3 ca = split3_pair(xa), cb = split3_pair(xb);
    char* wm = twm + 6 * u * 1024;
    char* wl = twl + 6 * u * 512;
    *reinterpret_cast<unsigned*>(wm) = ca[0];
    *reinterpret_cast<unsigned*>(wm + 8) = ca[1];
    *reinterpret_cast<unsigned*>(wl) = ca[2];
    *reinterpret_cast<unsigned*>(wm + 1024) = cb[0];
    *reinterpret_cast<unsigned*>(wm + 1024 + 8) = cb[1];
    *reinterpret_cast<unsigned*>(wl + 512) = cb[2];
  };
#else
  // T: wave tv = wave < 6 transforms column tv of every (tile, channel half) patch: lane (tile, h)
  // forms e[r] = B_tv(d[r][.]) over the 6 patch rows (the row's taps: up to 4 columns with
  // wave-uniform coefficients), then V[u][tv] = B_u(e) for u = 0..5, split into the operand chain
  // and written to the V buffer at (6u + tv, h, tile) = the M phase's read address.
  // balanced over the SIMDs (waves w and w + 4 share one): waves 0..3 transform columns 0..3 whole,
  // waves 4 / 6 column 4 and waves 5 / 7 column 5, each pair splitting its 6 outputs (u < 3 / u >= 3)
  // and both doing the column's 6 row steps: 326 + 211 VALU per SIMD instead of 326 + 326 / 326
#if KRRN_W4_TSPLIT
  const int tv = wave < 4 ? wave : 4 + (wave & 1);
  const int tulo = wave < 6 ? 0 : 3, tuhi = wave < 4 ? 6 : (wave < 6 ? 3 : 6);
#else
  const int tv = wave < 6 ? wave : 5;  // waves 6, 7 skip the transform
  const int tulo = 0, tuhi = 6;
#endif
  int tcol[4];
  float tk[4];
  switch (tv) {
    case 0: tcol[0] = 0; tcol[1] = 2; tcol[2] = 4; tcol[3] = 4; tk[0] = 4.f; tk[1] = -5.f; tk[2] = 1.f; tk[3] = 0.f; break;
    case 1: tcol[0] = 1; tcol[1] = 2; tcol[2] = 3; tcol[3] = 4; tk[0] = -4.f; tk[1] = -4.f; tk[2] = 1.f; tk[3] = 1.f; break;
    case 2: tcol[0] = 1; tcol[1] = 2; tcol[2] = 3; tcol[3] = 4; tk[0] = 4.f; tk[1] = -4.f; tk[2] = -1.f; tk[3] = 1.f; break;
    case 3: tcol[0] = 1; tcol[1] = 2; tcol[2] = 3; tcol[3] = 4; tk[0] = -2.f; tk[1] = -1.f; tk[2] = 2.f; tk[3] = 1.f; break;
    case 4: tcol[0] = 1; tcol[1] = 2; tcol[2] = 3; tcol[3] = 4; tk[0] = 2.f; tk[1] = -1.f; tk[2] = -2.f; tk[3] = 1.f; break;
    default: tcol[0] = 1; tcol[1] = 3; tcol[2] = 5; tcol[3] = 5; tk[0] = 4.f; tk[1] = -5.f; tk[2] = 1.f; tk[3] = 0.f; break;
  }
  const int ttile = lane & 31, th = lane >> 5;
  const int pbase = (4 * (ttile >> 4)) * kRS + 9 * (ttile & 15) + th;  // patch origin slot
  const char* tb[4];       // this chunk's tap columns in the ring slot the transform reads
  char* twm = nullptr;     // this lane's V entry of component tv (plane MH)
  char* twl = nullptr;     // (plane L)
  f32x4 td[4];             // the taps of the patch row being transformed next
  f32x4 te[6];             // e[r]
  auto t_begin = [&](int ck) {  // transform of chunk ck: addresses, and patch row 0's reads
    const int p = ck & 1;
    const char* rb = smem + kOffR + p * (kRingF * 4) + 16 * pbase;
#pragma unroll
    for (int t = 0; t < 4; ++t) tb[t] = rb + 16 * (2 * tcol[t] + (tcol[t] >> 2));
    twm = smem + p * (kVMH * 4) + tv * 1024 + 16 * lane;
    twl = smem + kOffL + p * (kVL * 4) + tv * 512 + 8 * lane;
#pragma unroll
    for (int t = 0; t < 4; ++t) td[t] = *reinterpret_cast<const f32x4*>(tb[(KRRN_W4_EXP & 64) ? 0 : t]);
  };
  // step s < 6: e[s] from row s's taps, then row s + 1's reads; step 6 + u: output u
  auto t_step = [&](int s) {
    if (s < 6) {
#pragma unroll
      for (int e = 0; e < 4; ++e)
        te[s][e] = __builtin_fmaf(tk[3], td[3][e], __builtin_fmaf(tk[2], td[2][e], __builtin_fmaf(tk[1], td[1][e], tk[0] * td[0][e])));
      if (s < 5) {
#pragma unroll
        for (int t = 0; t < 4; ++t) {
          if ((KRRN_W4_EXP & 64) && t > 0) {  // timing study: one tap read per row, VALU unchanged
            td[t] = td[0];
            asm volatile("" : "+v"(td[t]));
          } else if (KRRN_W4_SKIP3 && t == 3) {
            // columns 0 / 5 have 3 taps (tk[3] = 0): keep row 0's finite 4th tap instead of re-reading
            if (tv >= 1 && tv <= 4) td[3] = *reinterpret_cast<const f32x4*>(tb[3] + (s + 1) * kRS * 16);
          } else {
            td[t] = *reinterpret_cast<const f32x4*>(tb[t] + (s + 1) * kRS * 16);
          }
        }
      }
      return;
    }
    const int u = s - 6;
    if (u < tulo || u >= tuhi) return;
    f32x4 x;
    switch (u) {
      case 0: x = bt_row<0>(te); break;
      case 1: x = bt_row<1>(te); break;
      case 2: x = bt_row<2>(te); break;
      case 3: x = bt_row<3>(te); break;
      case 4: x = bt_row<4>(te); break;
      default: x = bt_row<5>(te); break;
    }
    const u32x6 ch = split3(x);
    *reinterpret_cast<u32x4*>(twm + 6 * u * 1024) = u32x4{ch[0], ch[1], ch[2], ch[3]};
    *reinterpret_cast<u32x2*>(twl + 6 * u * 512) = u32x2{ch[4], ch[5]};
  };
#endif
  // which transform steps run after component k's MFMAs (the VALU work beside the matrix pipe)
  constexpr int kStep0[10] = {0, 1, 2, 3, 4, 5, 7, 9, 11, 12};  // steps kStep0[k] .. kStep0[k + 1] - 1

  auto comp_of = [&](int k) { return 6 * (cu0 + k / 3) + cv0 + k % 3; };
  // one chunk: M(ck) on V[ck & 1], interleaved with T(ck + 1) into V[(ck + 1) & 1]; the raw input
  // of chunk ck + 2 goes into the ring slot T(ck) has read
  auto do_chunk = [&](int ck) {
    const bool tr = !(KRRN_W4_EXP & 4) && ck + 1 < nck && (KRRN_W4_TSPLIT || wave < 6);  // the last chunk: no T
    const int p = ck & 1;
    const char* vm = smem + p * (kVMH * 4) + 16 * lane;
    const char* vlo = smem + kOffL + p * (kVL * 4) + 8 * lane;
    auto chain = [&](int k) {
      const u32x4 mh = *reinterpret_cast<const u32x4*>(vm + comp_of(k) * 1024);
      const u32x2 l = *reinterpret_cast<const u32x2*>(vlo + comp_of(k) * 512);
      return u32x6{mh[0], mh[1], mh[2], mh[3], l[0], l[1]};
    };
    const bool stage = ck + 2 < nck && !(KRRN_W4_EXP & 8);
    __builtin_amdgcn_sched_barrier(0);
    if (tr) t_begin(ck + 1 < nck ? ck + 1 : ck + 1 - 2);  // past the last chunk: a harmless repeat
    u32x6 acn = chain(0);
#pragma unroll
    for (int k = 0; k < 9; ++k) {
      u32x6 ac = acn;
      if (k < 8) acn = chain(k + 1);  // the next component's operands, read under this one's MFMAs
      asm volatile("" : "+v"(ac));  // one register tuple: the MFMA operands are its sub-registers
      u32x6 bc = {wmh[k % 3][0], wmh[k % 3][1], wmh[k % 3][2], wmh[k % 3][3], wl[k % 3][0], wl[k % 3][1]};
      asm volatile("" : "+v"(bc));
#if KRRN_W4_EXP & 1
      acc[k][0] += __uint_as_float(ac[0] ^ ac[4] ^ bc[0] ^ bc[4]);
#else
      acc[k] = __builtin_amdgcn_mfma_f32_32x32x16_bf16(sub4(ac, 0), sub4(bc, 0), acc[k], 0, 0, 0);  // mm + hh
      acc[k] = __builtin_amdgcn_mfma_f32_32x32x16_bf16(sub4(ac, 0), sub4(bc, 2), acc[k], 0, 0, 0);  // mh + hl
      acc[k] = __builtin_amdgcn_mfma_f32_32x32x16_bf16(sub4(ac, 2), sub4(bc, 0), acc[k], 0, 0, 0);  // hm + lh
#endif
#if !(KRRN_W4_EXP & 2)
      if (k < 6) load_w(ck, k + 3); else load_w(ck + 1, k - 6);
#endif
      if (tr) {
#pragma unroll
        for (int st = kStep0[k]; st < kStep0[k + 1]; ++st) t_step(st);
      }
      // the raw input of chunk ck + 2, into the ring slot T(ck) read during chunk ck - 1 (requested at
      // the chunk's start instead, it only moves the wait: profiles/w4_trace.py)
      if (k == 4 && ck < 16) W4_MARK(3 * ck + 1);
      if (k == kRawK && stage) dma_raw(ck + 2, p);
      // issue shape of the slot: the next operands' LDS reads first, then the three MFMAs with the
      // transform VALU in their gaps (one wave's in-order issue would otherwise wait out each
      // dependent MFMA), then the weight reload
      __builtin_amdgcn_sched_group_barrier(0x100, 6, 0);  // DS reads
      __builtin_amdgcn_sched_group_barrier(0x008, 1, 0);  // MFMA
      __builtin_amdgcn_sched_group_barrier(0x002, kGap, 0);  // VALU
      __builtin_amdgcn_sched_group_barrier(0x008, 1, 0);
      __builtin_amdgcn_sched_group_barrier(0x002, kGap, 0);
      __builtin_amdgcn_sched_group_barrier(0x008, 1, 0);
      __builtin_amdgcn_sched_group_barrier(0x002, kGap, 0);
      __builtin_amdgcn_sched_barrier(0);  // keep each component's reload and transform steps in place
    }
  };

  // prologue: raw chunks 0 and 1 to the ring and chunk 0's first weights requested together; T(0)
  // waits only for raw chunk 0 (in-order vmcnt: chunk 1's 3 DMAs and the 6 weight loads may still
  // be in flight), chunk 1 lands under it
  dma_raw(0, 0);
  if (nck > 1) dma_raw(1, 1);
#pragma unroll
  for (int k = 0; k < 3; ++k) load_w(0, k);
  if (nck > 1)
    asm volatile("s_waitcnt vmcnt(9)\n\ts_barrier" ::: "memory");
  else
    asm volatile("s_waitcnt vmcnt(6)\n\ts_barrier" ::: "memory");
  if (!(KRRN_W4_EXP & 4) && (KRRN_W4_TSPLIT || wave < 6)) {
    t_begin(0);
#pragma unroll
    for (int st = 0; st < 12; ++st) t_step(st);
  }
  asm volatile("s_waitcnt vmcnt(6) lgkmcnt(0)\n\ts_barrier" ::: "memory");

  W4_MARK(49);
  for (int ck = 0; ck < nck; ++ck) {
    if (ck < 16) W4_MARK(3 * ck);
    do_chunk(ck);
    if (ck < 16) W4_MARK(3 * ck + 2);
    // hand-offs through LDS: the V buffers (lgkmcnt) and the raw chunk this wave's DMA wrote (issued
    // after component kRawK: the 2 (b128 + b64) weight loads of each later component may stay in flight)
    static_assert(kRawK >= 6 && kRawK <= 8, "vmcnt count below");
    asm volatile("s_waitcnt vmcnt(%0) lgkmcnt(0)\n\ts_barrier" ::"n"(2 * (8 - kRawK)) : "memory");
  }

#if KRRN_W4_EXP & 16
  {
    float sum = 0.f;
#pragma unroll
    for (int k = 0; k < 9; ++k) sum += acc[k][0] + acc[k][15];
    if (sum == 12345.f) a.out[tid] = sum;
    return;
  }
#endif
  // epilogue: 2 passes of 16 tiles (accumulator rows 8 pass .. 8 pass + 7 of each lane: local tile
  // (r & 3) + 8 ((r >> 2) & 1) + 4 h of the pass); a pass's stores free its 72 accumulator registers.
  // Then wave w forms output row i = w & 3 of tile groups (w >> 2) and (w >> 2) + 2: lane (tile of
  // the group, channel quad) -> float4 channel-run stores.
  W4_MARK(50);
  const int enq = lane & 15, etl = lane >> 4, ei = wave & 3;
#pragma unroll
  for (int pass = 0; pass < 2; ++pass) {
    char* ew = smem + (32 * nh + fr) * 4;
#pragma unroll
    for (int k = 0; k < 9; ++k) {
      const int comp = comp_of(k);
#pragma unroll
      for (int q = 0; q < 8; ++q) {
        const int r = 8 * pass + q;
        const int tl = (r & 3) + 8 * ((r >> 2) & 1) + 4 * h;
        *reinterpret_cast<float*>(ew + (comp * 16 + tl) * kET) = acc[k][r];
      }
    }
    __syncthreads();
#pragma unroll
    for (int it = 0; it < 2; ++it) {
      const int tl = 4 * ((wave >> 2) + 2 * it) + etl;
      const int ng = n0 + 4 * enq;
      switch (ei) {
        case 0: epi_row<0, HP>(a, smem, enq, tl, pass, b, ty0, tx0, ng, nb); break;
        case 1: epi_row<1, HP>(a, smem, enq, tl, pass, b, ty0, tx0, ng, nb); break;
        case 2: epi_row<2, HP>(a, smem, enq, tl, pass, b, ty0, tx0, ng, nb); break;
        default: epi_row<3, HP>(a, smem, enq, tl, pass, b, ty0, tx0, ng, nb); break;
      }
    }
    __syncthreads();
  }
#if KRRN_W4_TRACE
  W4_MARK(51);
  __syncthreads();
  if (blockIdx.x < 256)
    for (int i = tid; i < 8 * kTrN; i += 512) g_w4_trace[blockIdx.x * 8 * kTrN + i] = trace_lds[i];
#endif
}

}  // namespace

#if KRRN_W4_TRACE
KRRN_API int krrn_w4_trace_copy(void* dst) {  // 256 blocks x 8 waves x kTrN u32 cycle stamps
  return hipMemcpyFromSymbol(dst, HIP_SYMBOL(g_w4_trace), sizeof(g_w4_trace)) == hipSuccess ? 0 : -1;
}
#endif

KRRN_API int krrn_conv3x3_wino4_x3_f32(const float* in, int in_cs, int in_co, int B, int H, int W, int cin,
                                       const void* U3, int N, int n_store, const float* scale, const float* bias,
                                       const float* res, int res_cs, int res_co, float* out, int out_cs, int out_co,
                                       int relu, void* stream) {
  if (!in || !U3 || !out) return KRRN_EARG;
  if (B < 1 || H < 1 || W < 1 || N < 1 || n_store < 1 || n_store > N) return KRRN_ESHAPE;
  if (cin < kC || (cin % kC) || in_co + cin > in_cs) return KRRN_EALIGN;
  if (!krrn_aligned16(U3) || (((uintptr_t)in) & 15u) || (in_cs & 3) || (in_co & 3)) return KRRN_EALIGN;
  if (out_co + n_store > out_cs) return KRRN_ESHAPE;
  Wino4Args a;
  a.in = in; a.in_cs = in_cs; a.in_co = in_co; a.B = B; a.H = H; a.W = W; a.cin = cin;
  a.img = (long long)H * W * in_cs;
  a.U3 = U3; a.N = N; a.n_store = n_store; a.scale = scale; a.bias = bias;
  a.res = res; a.res_cs = res_cs; a.res_co = res_co;
  a.out = out; a.out_cs = out_cs; a.out_co = out_co; a.relu = relu;
  a.Ht = (H + 3) / 4; a.Wt = (W + 3) / 4;
  const bool ov = !(out_cs & 3) && !(out_co & 3) && krrn_aligned16(out);
  const bool rv = !res || (!(res_cs & 3) && !(res_co & 3) && krrn_aligned16(res));
  const bool sv = (!scale || krrn_aligned16(scale)) && (!bias || krrn_aligned16(bias));
  a.vec = (ov && rv && sv) ? 1 : 0;
  a.w1 = nullptr; a.part = nullptr;
  // 32-bit buffer offsets: one image, and the MH plane (records x 16 B)
  const long long nrec = (long long)(cin / kC) * 36 * N * 2;
  if (a.img * 4 >= 0x7FFF0000LL || nrec * 16 >= 0x7FFF0000LL) return KRRN_ESHAPE;
  const long long rb = (long long)B * krrn_cdiv(a.Ht, kGY) * krrn_cdiv(a.Wt, kGX) * krrn_cdiv(N, kN);
  if (rb > 0x7fffffffLL) return KRRN_ESHAPE;
  hipLaunchKernelGGL(wino_f43_x3_kernel<0>, dim3((unsigned)rb), dim3(512), 0, (hipStream_t)stream, a);
  return krrn_launch_status();
}

KRRN_API int krrn_conv3x3_wino4_x3_head_f32(const float* in, int in_cs, int in_co, int B, int H, int W, int cin,
                                            const void* U3, int N, const float* scale, const float* bias,
                                            const float* res, int res_cs, int res_co, int relu, const float* w1,
                                            const float* b1, int p1, float* part, float* out, int out_c,
                                            void* stream) {
  if (!in || !U3 || !w1 || !part || !out) return KRRN_EARG;
  if (B < 1 || H < 1 || W < 1 || N < 4 || (N & 3) || p1 < 1 || p1 > 4 || out_c < p1) return KRRN_ESHAPE;
  if (cin < kC || (cin % kC) || in_co + cin > in_cs) return KRRN_EALIGN;
  if (!krrn_aligned16(U3) || (((uintptr_t)in) & 15u) || (in_cs & 3) || (in_co & 3)) return KRRN_EALIGN;
  if (!krrn_aligned16(w1) || !krrn_aligned16(part)) return KRRN_EALIGN;
  if ((scale && !krrn_aligned16(scale)) || (bias && !krrn_aligned16(bias))) return KRRN_EALIGN;
  if (res && ((res_cs & 3) || (res_co & 3) || !krrn_aligned16(res))) return KRRN_EALIGN;
  Wino4Args a;
  a.in = in; a.in_cs = in_cs; a.in_co = in_co; a.B = B; a.H = H; a.W = W; a.cin = cin;
  a.img = (long long)H * W * in_cs;
  a.U3 = U3; a.N = N; a.n_store = N; a.scale = scale; a.bias = bias;
  a.res = res; a.res_cs = res_cs; a.res_co = res_co;
  a.out = nullptr; a.out_cs = 0; a.out_co = 0; a.relu = relu; a.vec = 1;
  a.Ht = (H + 3) / 4; a.Wt = (W + 3) / 4;
  a.w1 = w1; a.part = part;
  const long long nrec = (long long)(cin / kC) * 36 * N * 2;
  if (a.img * 4 >= 0x7FFF0000LL || nrec * 16 >= 0x7FFF0000LL) return KRRN_ESHAPE;
  const int nbn = krrn_cdiv(N, kN);
  const long long rb = (long long)B * krrn_cdiv(a.Ht, kGY) * krrn_cdiv(a.Wt, kGX) * nbn;
  const long long M = (long long)B * H * W;
  const long long fb = (M + 255) / 256;
  if (rb > 0x7fffffffLL || fb > 0x7fffffffLL) return KRRN_ESHAPE;
  hipStream_t s = (hipStream_t)stream;
  // p1 <= 3 (nml_final of one class) forms 3 dot products per pixel, p1 = 4 all four
  if (p1 <= 3) hipLaunchKernelGGL(wino_f43_x3_kernel<3>, dim3((unsigned)rb), dim3(512), 0, s, a);
  else hipLaunchKernelGGL(wino_f43_x3_kernel<4>, dim3((unsigned)rb), dim3(512), 0, s, a);
  const int st = krrn_launch_status();
  if (st != KRRN_OK) return st;
  hipLaunchKernelGGL(wino4_head_finish_kernel, dim3((unsigned)fb), dim3(256), 0, s, part, nbn, M, H * W, b1, p1, out,
                     out_c);
  return krrn_launch_status();
}
