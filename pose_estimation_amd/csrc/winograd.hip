// Winograd F(2x2, 3x3) convolution on the gfx950 f32 matrix cores, fully fused.
//
// Serves the stride-1, pad-1 3x3 convs of the KRRN heads (XYZNet / NMLNet at S/2 and S,
// lib/network/krrn.py:46-84), the HRNet last_layer (myhrnet.py:328-346) and the deconv
// BasicBlock (myhrnet.py:324). cuDNN / MIOpen pick Winograd for exactly these f32 convs on the
// reference's own GPU path; here it is one kernel:
//
//   per 2x2 output tile t and input channel c: V = B^T d B  (d = the 4x4 input patch, pad 0)
//   per output channel n:                      U = G g G^T  (host, f64, once per plan)
//   M[xi][t][n] = sum_c V[xi][t][c] U[xi][n][c]   (16 GEMMs, xi = 4u + v)
//   Y = A^T M A (2x2), then out = act(scale[n] * Y + bias[n] (+ res))
//
// with B^T = [1 0 -1 0; 0 1 1 0; 0 -1 1 0; 0 1 0 -1], A^T = [1 1 1 0; 0 1 -1 -1]
// (Lavin & Gray 2016). The 16 products per tile replace 36 multiply-adds of the direct
// conv: 2.25x fewer MFMA flops. Neither V nor M ever leaves the CU.
//
// Default kernel (wino_f23_ring_kernel): block = 16 x 2 output tiles of one image x 64 output
// channels, 256 threads = 4 waves; wave w owns the components xi = 4w .. 4w+3 (row u = w of the
// 4x4 grid) over the whole 32 x 64 block (2 x v_mfma_f32_32x32x2_f32 n-blocks each, 128
// accumulator registers). Input channels stream in chunks of 8. Per chunk the block stages the
// RAW input region of its 32 tiles (6 x 34 pixels x 8 channels, one b128 load per 16-B piece, 2
// per thread, zero outside the image) into a 3-slot LDS ring; each lane reads the 2 patch rows its
// component row needs (8 ds_read_b128) and forms its MFMA A operands V = B^T d B in registers,
// for chunk ck+1 while chunk ck's MFMAs issue. A wave's weights are disjoint from the other
// waves', so they skip LDS: 8 b128 loads per lane per chunk (1 KB contiguous per instruction),
// one chunk ahead. One barrier per chunk. The output transform: wave w holds row u = w of every
// (tile, channel)'s 4x4 M, so the column combination is lane-local and only 2 of 4 values per
// row go through LDS; stores are float4 channel runs. The step runs the split-bf16 forms below
// (wino_f23_x3_kernel); this f32 kernel is its accuracy reference.
// Round 1's register-staged kernel (every thread transforming one (tile, channel) patch into an
// LDS image of V, weights staged through LDS, two barriers per chunk: bit-identical, 1.55 ms) and
// the ring without the transform overlap were removed in round 4.
// Measured (MI355X, 64 x 128 -> 128 x 120 x 120, profiles/bench_wino.py): staged 1.55 ms, ring
// 1.41 ms (84 TF in the matrix pipe; 68 % MFMA-busy by SQ_VALU_MFMA_BUSY_CYCLES at 2.05 GHz,
// waves 73 % issue-stalled, 10 % in s_waitcnt / barriers), ring without the transform overlap
// 1.44 ms; the epilogue costs 6-8 % (1.35 ms with it skipped). Rejected: an LDS-free variant
// (every lane loading its own 8 patch vectors: 1.46 ms, TA busy 2.3x), s-outer MFMA order (no
// gain), and from round 1: double-buffered LDS at one wave per SIMD (2.24 ms), persistent blocks
// prefetching the next tile during the epilogue (1.57 ms, spills), s_setprio around the MFMA
// cluster (+2 %), a 32-wide N tile at 3 blocks/CU (1.54-1.56 ms), a ping-pong kernel with two
// wave groups (1.95 ms), LDS-DMA weights (1.49 ms).
#include "krrn_common.h"

namespace {

constexpr int kWT = 32;       // tiles per block
#ifndef KRRN_WINO_EXP
#define KRRN_WINO_EXP 0
#endif
#ifndef KRRN_WINO_WN
#define KRRN_WINO_WN 64
#endif
constexpr int kWN = KRRN_WINO_WN;  // output channels per block
constexpr int kNJ = kWN / 32;      // 32-wide n-blocks per wave
constexpr int kN4 = kWN / 4;       // 4-channel groups per tile
constexpr int kWC = 8;        // input channels per chunk
constexpr unsigned kWOOB = 0xFFFF0000u;  // > any valid offset, and + channel offsets stays > it

struct WinoArgs {
  const float* in;
  int in_cs, in_co;
  int B, H, W, cin;
  long long img;  // elements per input image
  const float* U;  // [16][N][cin] row-major
  int N, n_store;
  const float* scale;
  const float* bias;
  const float* res;
  int res_cs, res_co;
  float* out;
  int out_cs, out_co;
  int relu;
  int vec;        // float4 epilogue (16-B aligned channel runs, n_store % 4 == 0)
  int Ht, Wt, T;  // tiles per column / row, total tiles
  // head form (krrn_conv3x3_wino_x3_head_f32): the conv's activated output is not stored; its dot
  // with the 4 rows of w1 ([4][N], the following 1x1 conv's weights) over this block's channels goes
  // to part[nb][pixel][4], summed over the n-blocks by wino_head_finish_kernel
  const float* w1;
  float* part;
};

// Output transform Y = A^T M A + epilogue. Wave w holds row u = w of the 4x4 component grid
// (acc[x] = component v = x) for every (tile, channel) of the block, so the column combination
// c0 = M[u][0]+M[u][1]+M[u][2], c1 = M[u][1]-M[u][2]-M[u][3] is lane-local; only (c0, c1)
// go through LDS ([u][c][tile][n], pitch kSP), and each thread then finishes the row
// combination for 2 (tile, 4-channel) pairs and stores 2x2 pixels x float4.
constexpr int kSP = kWN + 4;

__device__ __forceinline__ void wino_epi_put(float* smem, f32x16 (&acc)[4][kNJ]) {
  const int lane = threadIdx.x & 63, wave = (threadIdx.x >> 6) & 3;
  const int fr = lane & 31;
#pragma unroll
  for (int j = 0; j < kNJ; ++j)
#pragma unroll
    for (int r = 0; r < 16; ++r) {
      const int row = (r & 3) + 8 * (r >> 2) + 4 * (lane >> 5);
      const float m0 = acc[0][j][r], m1 = acc[1][j][r], m2 = acc[2][j][r], m3 = acc[3][j][r];
      float* p0 = smem + ((wave * 2 + 0) * kWT + row) * kSP + j * 32 + fr;
      float* p1 = smem + ((wave * 2 + 1) * kWT + row) * kSP + j * 32 + fr;
      *p0 = m0 + m1 + m2;
      *p1 = m1 - m2 - m3;
    }
}

// ---- The f32 ring kernel (krrn_conv3x3_wino_f32): raw input patches through a 3-slot LDS ring,
// the transform done by the consuming waves, weights straight to registers ---------------------
// Block = 16 x 2 output tiles (32 x 4 output pixels of one image) x 64 output channels; wave w
// owns component row u = w (xi = 4w .. 4w+3) as above. Per 8-channel chunk the block stages the
// RAW input region its 32 tiles read (6 rows x 34 cols x 8 channels = 408 16-B pieces, 2 per
// thread, one b128 load each) into a ring slot; each lane then reads the 2 patch rows its
// component row needs (8 ds_read_b128 = 4 columns x 2 rows x its 4 channels), forms
// t = B^T-row (d_a +- d_b) and V[v] = t-combinations in registers (the same f32 operations as the
// staged kernel: bit-identical operands), and feeds them as MFMA A operands. The weights of a
// wave's own 4 components are disjoint from the other waves', so they skip LDS: 8 b128 loads per
// lane per chunk (1 KB contiguous per wave-instruction), one chunk ahead. One barrier per chunk.
constexpr int kGX = 16, kGY = 2;                 // tiles per block (x, y): kGX * kGY == kWT
constexpr int kRR = 2 * kGY + 2, kRC = 2 * kGX + 2;  // raw rows / cols of a block
constexpr int kRPieces = kRR * kRC * 2;          // 16-B pieces per chunk
static_assert(kGX * kGY == kWT && kRPieces <= 512, "ring geometry");
// Ring slot layout: piece (raw row r, column c, channel half h) at 16-B slot r * kRowSlots + 2c + h +
// c / 2 (one slot of padding per column pair). A wave's ds_read_b128 of patch column j reads, per
// lane (tile tx, ty; half h), slot (2 ty + row) * kRowSlots + 5 tx + h + {0, 2, 5, 7}[j]: the 16 lanes
// of each b128 lane group land on 16 distinct 16-B bank slots (kRowSlots = 88 >= the 85 slots of a padded
// row, and = 0 mod 8, which keeps the two tile rows apart). Unpadded (2c + h) they shared 4 bank slots: 4-way conflicts, 62 % of the kernel's
// LDS-array cycles (profiles/r4_wino_pmc.sh, SQ_LDS_BANK_CONFLICT / SQ_LDS_IDX_ACTIVE).
constexpr int kRowSlots = 88;
constexpr int kColOff[4] = {0, 2, 5, 7};
constexpr int kRSlot = kRR * kRowSlots * 4;      // floats per ring slot
constexpr int kRDummy = kRR * kRowSlots - 1;     // the slot threads without a piece write to
__device__ __forceinline__ int ring_slot(int r, int c, int h) { return r * kRowSlots + 2 * c + h + (c >> 1); }
static_assert(2 * (kRC - 1) + 1 + (kRC - 1) / 2 < kRowSlots && (kRowSlots % 8) == 0, "padded ring row");
static_assert((kRR - 1) * kRowSlots + 2 * (kRC - 1) + 1 + (kRC - 1) / 2 < kRDummy, "padded ring slot fits");
static_assert(4 * 2 * kWT * kSP >= 3 * kRSlot, "ring fits in the epilogue's LDS");

// epilogue finish for a 2-D tile block of WT tiles, GX per row: tile tl -> (ty, tx) = (tl / GX, tl % GX);
// smem holds (c0, c1) as [u][q][tile][n] with pitch kSP
template <int WT = kWT, int GX = kGX>
__device__ __forceinline__ void wino_epi_finish2d(const WinoArgs& a, const float* smem, int b, int ty0, int tx0,
                                                  int n0) {
  constexpr int kNP = WT * kN4 / 256;
  const int tid = threadIdx.x;
#pragma unroll
  for (int i = 0; i < kNP; ++i) {
    const int pr = tid + 256 * i;
    const int n4 = pr % kN4, tl = pr / kN4;
    const int n = n0 + 4 * n4;
    const int ty = ty0 + tl / GX, tx = tx0 + tl % GX;
    if (ty >= a.Ht || tx >= a.Wt || n >= a.n_store) continue;
    f32x4 c[4][2];
#pragma unroll
    for (int u = 0; u < 4; ++u)
#pragma unroll
      for (int q = 0; q < 2; ++q) c[u][q] = *reinterpret_cast<const f32x4*>(smem + ((u * 2 + q) * WT + tl) * kSP + 4 * n4);
    f32x4 y[4];
    y[0] = c[0][0] + c[1][0] + c[2][0];
    y[1] = c[0][1] + c[1][1] + c[2][1];
    y[2] = c[1][0] - c[2][0] - c[3][0];
    y[3] = c[1][1] - c[2][1] - c[3][1];
    f32x4 scl = {1.f, 1.f, 1.f, 1.f}, bia = {0.f, 0.f, 0.f, 0.f};
    if (a.vec) {
      if (a.scale) scl = *reinterpret_cast<const f32x4*>(a.scale + n);
      if (a.bias) bia = *reinterpret_cast<const f32x4*>(a.bias + n);
    }
#pragma unroll
    for (int q = 0; q < 4; ++q) {
      const int oy = 2 * ty + (q >> 1), ox = 2 * tx + (q & 1);
      if (oy >= a.H || ox >= a.W) continue;
      const size_t pix = ((size_t)b * a.H + oy) * a.W + ox;
      if (a.vec) {
        f32x4 v = y[q] * scl + bia;
        if (a.res) v += *reinterpret_cast<const f32x4*>(a.res + pix * a.res_cs + a.res_co + n);
        if (a.relu) {
#pragma unroll
          for (int e = 0; e < 4; ++e) v[e] = fmaxf(v[e], 0.f);
        }
        *reinterpret_cast<f32x4*>(a.out + pix * a.out_cs + a.out_co + n) = v;
      } else {
#pragma unroll
        for (int e = 0; e < 4; ++e) {
          if (n + e >= a.n_store) break;
          float v = y[q][e] * (a.scale ? a.scale[n + e] : 1.f) + (a.bias ? a.bias[n + e] : 0.f);
          if (a.res) v += a.res[pix * a.res_cs + a.res_co + n + e];
          if (a.relu) v = fmaxf(v, 0.f);
          a.out[pix * a.out_cs + a.out_co + n + e] = v;
        }
      }
    }
  }
}

// sum over the 16 lanes of a DPP row (every lane gets the sum): quad swaps, then half-row and row
// mirrors
__device__ __forceinline__ float row16_sum(float x) {
  x += __int_as_float(__builtin_amdgcn_update_dpp(0, __float_as_int(x), 0xB1, 0xF, 0xF, false));  // quad [1 0 3 2]
  x += __int_as_float(__builtin_amdgcn_update_dpp(0, __float_as_int(x), 0x4E, 0xF, 0xF, false));  // quad [2 3 0 1]
  x += __int_as_float(__builtin_amdgcn_update_dpp(0, __float_as_int(x), 0x141, 0xF, 0xF, false));  // row_half_mirror
  x += __int_as_float(__builtin_amdgcn_update_dpp(0, __float_as_int(x), 0x140, 0xF, 0xF, false));  // row_mirror
  return x;
}

// Head epilogue: the conv's activated 2x2 pixels x 4 channels per (tile, n4) pair dotted with the
// following 1x1 conv's 4 weight rows, summed over the 16 lanes (n4 = lane % 16) that hold the
// tile's 64 channels, one float4 per pixel to part[nb] (the n-blocks' partials are added in order
// by wino_head_finish_kernel: deterministic). The 128-channel map itself is never written.
template <int WT = kWT, int GX = kGX>
__device__ __forceinline__ void wino_epi_head2d(const WinoArgs& a, const float* smem, int b, int ty0, int tx0,
                                                int n0, int nb) {
  constexpr int kNP = WT * kN4 / 256;
  static_assert(kN4 == 16, "one tile's channels = one DPP row");
  const int tid = threadIdx.x;
  const long long M = (long long)a.B * a.H * a.W;
#pragma unroll
  for (int i = 0; i < kNP; ++i) {
    const int pr = tid + 256 * i;
    const int n4 = pr % kN4, tl = pr / kN4;
    const int n = n0 + 4 * n4;
    const int ty = ty0 + tl / GX, tx = tx0 + tl % GX;
    const bool tok = ty < a.Ht && tx < a.Wt;  // uniform over the row
    const bool nok = n < a.n_store;
    f32x4 c[4][2];
#pragma unroll
    for (int u = 0; u < 4; ++u)
#pragma unroll
      for (int q = 0; q < 2; ++q) c[u][q] = *reinterpret_cast<const f32x4*>(smem + ((u * 2 + q) * WT + tl) * kSP + 4 * n4);
    f32x4 y[4];
    y[0] = c[0][0] + c[1][0] + c[2][0];
    y[1] = c[0][1] + c[1][1] + c[2][1];
    y[2] = c[1][0] - c[2][0] - c[3][0];
    y[3] = c[1][1] - c[2][1] - c[3][1];
    const f32x4 zero = {0.f, 0.f, 0.f, 0.f};
    const f32x4 scl = (nok && a.scale) ? *reinterpret_cast<const f32x4*>(a.scale + n) : f32x4{1.f, 1.f, 1.f, 1.f};
    const f32x4 bia = (nok && a.bias) ? *reinterpret_cast<const f32x4*>(a.bias + n) : zero;
    f32x4 w[4];
#pragma unroll
    for (int o = 0; o < 4; ++o) w[o] = nok ? *reinterpret_cast<const f32x4*>(a.w1 + (size_t)o * a.N + n) : zero;
    float s[4][4];
#pragma unroll
    for (int q = 0; q < 4; ++q) {
      const int oy = 2 * ty + (q >> 1), ox = 2 * tx + (q & 1);
      const bool ok = tok && nok && oy < a.H && ox < a.W;
      f32x4 v = y[q] * scl + bia;
      if (a.res && ok) v += *reinterpret_cast<const f32x4*>(a.res + (((size_t)b * a.H + oy) * a.W + ox) * a.res_cs + a.res_co + n);
      if (a.relu) {
#pragma unroll
        for (int e = 0; e < 4; ++e) v[e] = fmaxf(v[e], 0.f);
      }
      if (!ok) v = zero;
#pragma unroll
      for (int o = 0; o < 4; ++o) s[q][o] = row16_sum(v[0] * w[o][0] + v[1] * w[o][1] + v[2] * w[o][2] + v[3] * w[o][3]);
    }
    if (n4 != 0 || !tok) continue;
#pragma unroll
    for (int q = 0; q < 4; ++q) {
      const int oy = 2 * ty + (q >> 1), ox = 2 * tx + (q & 1);
      if (oy >= a.H || ox >= a.W) continue;
      const size_t pix = ((size_t)b * a.H + oy) * a.W + ox;
      *reinterpret_cast<f32x4*>(a.part + ((size_t)nb * M + pix) * 4) = f32x4{s[q][0], s[q][1], s[q][2], s[q][3]};
    }
  }
}

// out[b][o][p] = sum over n-blocks (in order) of part[nb][b * HW + p][o] + b1[o], o < p1
__global__ __launch_bounds__(256) void wino_head_finish_kernel(const float* __restrict__ part, int nbn, long long M,
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

__global__ __launch_bounds__(256, 2) void wino_f23_ring_kernel(const WinoArgs a) {
  __shared__ __attribute__((aligned(16))) float smem[4 * 2 * kWT * kSP];
  const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
  const int gxn = krrn_cdiv(a.Wt, kGX), gyn = krrn_cdiv(a.Ht, kGY), nbn = krrn_cdiv(a.N, kWN);
  const int per_img = gxn * gyn;
  const int bid = krrn_xcd_remap(blockIdx.x, a.B * per_img * nbn);
  const int sp = bid / nbn, nb = bid - (bid / nbn) * nbn;
  const int b = sp / per_img, r2 = sp - (sp / per_img) * per_img;
  const int by = r2 / gxn, bx = r2 - (r2 / gxn) * gxn;
  const int n0 = nb * kWN;
  const int ty0 = by * kGY, tx0 = bx * kGX;
  const int nck = krrn_cdiv(a.cin, kWC);

  // raw staging: this thread's 2 pieces (pixel q/2 of the block's raw region, channel half q&1)
  const __amdgpu_buffer_rsrc_t rsA = __builtin_amdgcn_make_buffer_rsrc(
      (void*)(a.in + (size_t)b * a.img + a.in_co), (short)0, (int)min(a.img * 4 - (long long)a.in_co * 4, 0x7FFFFFFFLL),
      0x00020000);
  unsigned roff[2];
#pragma unroll
  for (int i = 0; i < 2; ++i) {
    const int q = tid + 256 * i;
    const int pix = q >> 1, hh = q & 1;
    const int rr = pix / kRC, rc = pix - (pix / kRC) * kRC;
    const int iy = 2 * ty0 - 1 + rr, ix = 2 * tx0 - 1 + rc;
    const bool ok = q < kRPieces && iy >= 0 && iy < a.H && ix >= 0 && ix < a.W;
    roff[i] = ok ? (unsigned)((((long long)iy * a.W + ix) * a.in_cs + 4 * hh) * 4) : kWOOB;
  }
  const int hq0 = tid & 1;  // channel half of piece 0 (piece 1 = tid + 256: the same half)
  auto load_raw = [&](int ck, f32x4 (&r)[2]) {
    const unsigned cb = (unsigned)(ck * kWC) * 4u;
    const unsigned cm = (ck < nck && ck * kWC + 4 * hq0 < a.cin) ? 0u : kWOOB;
#pragma unroll
    for (int i = 0; i < 2; ++i)
      r[i] = __builtin_bit_cast(f32x4, __builtin_amdgcn_raw_buffer_load_b128(rsA, (roff[i] + cb) | cm, 0, 0));
  };
  int wslot[2];  // this thread's 2 pieces in the padded slot layout (pieces past the region: a dummy slot)
#pragma unroll
  for (int i = 0; i < 2; ++i) {
    const int q = tid + 256 * i;
    const int pix = q >> 1, rr = pix / kRC;
    wslot[i] = q < kRPieces ? ring_slot(rr, pix - rr * kRC, q & 1) : kRDummy;
  }
  auto store_raw = [&](int slot, const f32x4 (&r)[2]) {
    float* dst = smem + slot * kRSlot;
#pragma unroll
    for (int i = 0; i < 2; ++i) *reinterpret_cast<f32x4*>(dst + 4 * wslot[i]) = r[i];
  };

  // weights of this wave's components: lane (n = j*32 + fr, channels 4h..4h+3) of U[ck][xi][n]
  const int fr = lane & 31, h = lane >> 5;
  const __amdgpu_buffer_rsrc_t rsU = __builtin_amdgcn_make_buffer_rsrc(
      (void*)a.U, (short)0, (int)min((long long)nck * 16 * a.N * kWC * 4, 0x7FFFFFFFLL), 0x00020000);
  unsigned uoff[4][kNJ];
#pragma unroll
  for (int v = 0; v < 4; ++v)
#pragma unroll
    for (int j = 0; j < kNJ; ++j) {
      const int n = n0 + j * 32 + fr;
      uoff[v][j] = n < a.N ? (unsigned)((((long long)(4 * wave + v) * a.N + n) * kWC + 4 * h) * 4) : kWOOB;
    }
  const unsigned ustride = (unsigned)(16 * a.N * kWC * 4);
  auto load_w = [&](int ck, f32x4 (&w)[4][kNJ]) {
    const unsigned wb = (unsigned)ck * ustride;
    const unsigned wm = ck < nck ? 0u : kWOOB;
#pragma unroll
    for (int v = 0; v < 4; ++v)
#pragma unroll
      for (int j = 0; j < kNJ; ++j)
        w[v][j] = __builtin_bit_cast(f32x4, __builtin_amdgcn_raw_buffer_load_b128(rsU, (uoff[v][j] + wb) | wm, 0, 0));
  };

  // this lane's patch rows: t_u = d[ra] + sgn * d[rb] (B^T row u)
  const int ra = wave == 0 ? 0 : (wave == 2 ? 2 : 1);
  const int rb = wave == 0 ? 2 : (wave == 3 ? 3 : (wave == 1 ? 2 : 1));
  const float sgn = wave == 1 ? 1.f : -1.f;
  const int tx = fr % kGX, ty = fr / kGX;
  const int pa = ring_slot(2 * ty + ra, 2 * tx, h);  // slot of (row ra, patch column 0)
  const int pb = ring_slot(2 * ty + rb, 2 * tx, h);

  f32x16 acc[4][kNJ];
#pragma unroll
  for (int x = 0; x < 4; ++x)
#pragma unroll
    for (int j = 0; j < kNJ; ++j)
#pragma unroll
      for (int r = 0; r < 16; ++r) acc[x][j][r] = 0.f;

  auto make_v = [&](const float* sl, f32x4 (&V)[4]) {
    f32x4 t[4];
#pragma unroll
    for (int c = 0; c < 4; ++c) {
      const f32x4 da = *reinterpret_cast<const f32x4*>(sl + 4 * (pa + kColOff[c]));
      const f32x4 db = *reinterpret_cast<const f32x4*>(sl + 4 * (pb + kColOff[c]));
      t[c] = da + sgn * db;
    }
    V[0] = t[0] - t[2];
    V[1] = t[1] + t[2];
    V[2] = t[2] - t[1];
    V[3] = t[1] - t[3];
  };
  auto mma = [&](const f32x4 (&V)[4], const f32x4 (&wc)[4][kNJ]) {
#pragma unroll
    for (int v = 0; v < 4; ++v)
#pragma unroll
      for (int j = 0; j < kNJ; ++j)
#pragma unroll
        for (int s2 = 0; s2 < 4; ++s2)
          acc[v][j] = __builtin_amdgcn_mfma_f32_32x32x2f32(V[v][s2], wc[v][j][s2], acc[v][j], 0, 0, 0);
  };

  f32x4 raw[2];
  f32x4 w[4][kNJ];
    // 3-slot ring: V of chunk ck+1 is formed (LDS reads + transform) beside chunk ck's MFMAs
    load_raw(0, raw);
    load_w(0, w);
    store_raw(0, raw);
    load_raw(1, raw);
    __syncthreads();
    store_raw(1, raw);
    load_raw(2, raw);
    f32x4 V[4];
    make_v(smem, V);
    __syncthreads();
    for (int ck = 0; ck < nck; ++ck) {
      f32x4 wc[4][kNJ];
#pragma unroll
      for (int v = 0; v < 4; ++v)
#pragma unroll
        for (int j = 0; j < kNJ; ++j) wc[v][j] = w[v][j];
      load_w(ck + 1, w);
      f32x4 Vn[4];
      make_v(smem + ((ck + 1) % 3) * kRSlot, Vn);
      mma(V, wc);
      store_raw((ck + 2) % 3, raw);
      load_raw(ck + 3, raw);
#pragma unroll
      for (int v = 0; v < 4; ++v) V[v] = Vn[v];
      __syncthreads();
    }
#if KRRN_WINO_EXP == 4  // timing experiment: one store per lane instead of the epilogue
  float sum = 0.f;
#pragma unroll
  for (int x = 0; x < 4; ++x)
#pragma unroll
    for (int j = 0; j < kNJ; ++j) sum += acc[x][j][0] + acc[x][j][15];
  if (sum == 12345.f) a.out[tid] = sum;
  return;
#endif
  wino_epi_put(smem, acc);
  __syncthreads();
  wino_epi_finish2d(a, smem, b, ty0, tx0, n0);
}

// ---- Split-bf16 ring kernel: the same block, ring and transform as wino_f23_ring_kernel<1>, the
// 16 channel GEMMs on the bf16 matrix cores (v_mfma_f32_32x32x16_bf16, 16x the f32 rate) at f32
// accuracy. Every f32 operand is split round-to-nearest into three bf16 terms,
// x = x_h + x_m + x_l with |x_m| <= 2^-8 |x|, |x_l| <= 2^-16 |x| (exact: 24 significand bits),
// and a product a b is summed over the 6 term pairs h h, h m, m h, h l, l h, m m; the 3 dropped
// (m l, l m, l l) are below 2^-23 |a b|, the size of the f32 MFMA's own product rounding, and
// everything accumulates in f32 (profiles/bench_wino_x3.py: RMS error vs f64 2.8e-7 against the
// f32 kernel's 3.0e-7).
// Register chains, no copies: a lane's 8 bf16 of an MFMA operand are 2 term kinds x its 4 channels
// (k = 8 half + i pairs A and B element i of the same lane), so with the A chain [V_m V_h V_l] and
// the B chain [U_m U_h U_l] (one b128 of plane U_mh + one b64 of plane U_l), 6 registers each, the
// three MFMAs are
//   A[0:3] x B[0:3] = mm + hh,   A[0:3] x B[2:5] = mh + hl,   A[2:5] x B[0:3] = hm + lh.
// An empty asm statement with each chain as a "+v" operand pins it to one 6-register tuple, so the
// operand slices are sub-registers and the weight loads land in the tuple directly. Round 4's A
// chain [V_h V_h V_m V_l] needed h twice, and LLVM rebuilt the overlapping slices with 40 register
// copies per wave and chunk (194 -> 154 VALU instructions in the loop, 250 -> 234 VGPRs).
// V is split in registers (v_cvt_pk_bf16_f32, RNE); U is split on the host (ops.wino_weights_x3).
// Weight addresses: a per-lane voffset per n-block and the chunk / component part in soffset
// (SALU); a wave reloads component v's weights for the next chunk as soon as its MFMAs have
// issued (one weight buffer in registers: acc 128 + weights 48 VGPRs).
// Measured (MI355X, profiles/bench_wino_x3.py, 64 x 128 -> 128): 120x120 1.03-1.06 ms against
// the f32 ring kernel's 1.39-1.47 ms, 60x60 0.27 vs 0.37 ms; in the step 412 vs 483 us per launch
// (12.99 vs 13.68 ms per step on one box). The bf16 MFMAs take ~280 us of the 1.05 ms: timing
// experiments (KRRN_WINO_EXP) put the rest in VALU issue (the split is 5.5 VALU per value, the
// transform ~2.5; a build with no MFMAs and no loads still takes 0.65 ms), then the weight and raw
// loads (-15 % / -11 % without them) and the epilogue (-15 %). Rejected: a 64-tile, 512-thread
// block (2 components x 2 tile-blocks x 2 n-blocks per wave: half the weight loads per MFMA and a
// bank-conflict-free ring layout, but one block per CU: 1.05-1.12 ms), sched_barrier-pinned
// reloads (no change).
typedef __bf16 bf16x8 __attribute__((ext_vector_type(8)));
typedef __bf16 bf16x2 __attribute__((ext_vector_type(2)));
typedef float f32x2 __attribute__((ext_vector_type(2)));
typedef unsigned u32x8 __attribute__((ext_vector_type(8)));
typedef unsigned u32x4 __attribute__((ext_vector_type(4)));
typedef unsigned u32x2 __attribute__((ext_vector_type(2)));

__device__ __forceinline__ unsigned pk_bf16(float a, float b) {
  return __builtin_bit_cast(unsigned, __builtin_convertvector(f32x2{a, b}, bf16x2));  // RNE
}
__device__ __forceinline__ float bf_lo(unsigned p) { return __builtin_bit_cast(float, p << 16); }
__device__ __forceinline__ float bf_hi(unsigned p) { return __builtin_bit_cast(float, p & 0xFFFF0000u); }

typedef unsigned u32x6 __attribute__((ext_vector_type(6)));

// x (4 channels) -> the A chain [x_m x_h x_l] as packed bf16 pairs
__device__ __forceinline__ u32x6 split3_chain(const f32x4 x) {
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

template <bool HEAD>
__global__ __launch_bounds__(256, 2) void wino_f23_x3_kernel(const WinoArgs a) {
  __shared__ __attribute__((aligned(16))) float smem[4 * 2 * kWT * kSP];
  const int tid = threadIdx.x, lane = tid & 63;
  const int wave = __builtin_amdgcn_readfirstlane(tid >> 6);
  const int gxn = krrn_cdiv(a.Wt, kGX), gyn = krrn_cdiv(a.Ht, kGY), nbn = krrn_cdiv(a.N, kWN);
  const int per_img = gxn * gyn;
  const int bid = krrn_xcd_remap(blockIdx.x, a.B * per_img * nbn);
  const int sp = bid / nbn, nb = bid - (bid / nbn) * nbn;
  const int b = sp / per_img, r2 = sp - (sp / per_img) * per_img;
  const int by = r2 / gxn, bx = r2 - (r2 / gxn) * gxn;
  const int n0 = nb * kWN;
  const int ty0 = by * kGY, tx0 = bx * kGX;
  const int nck = krrn_cdiv(a.cin, kWC);

  // raw staging: this thread's 2 pieces (pixel q/2 of the block's raw region, channel half q&1);
  // the chunk's channel offset goes in soffset
  const __amdgpu_buffer_rsrc_t rsA = __builtin_amdgcn_make_buffer_rsrc(
      (void*)(a.in + (size_t)b * a.img + a.in_co), (short)0, (int)min(a.img * 4 - (long long)a.in_co * 4, 0x7FFFFFFFLL),
      0x00020000);
  unsigned roff[2], roffm[2];  // roffm: the upper channel half masked (a last chunk of 4 channels)
#pragma unroll
  for (int i = 0; i < 2; ++i) {
    const int q = tid + 256 * i;
    const int pix = q >> 1, hh = q & 1;
    const int rr = pix / kRC, rc = pix - (pix / kRC) * kRC;
    const int iy = 2 * ty0 - 1 + rr, ix = 2 * tx0 - 1 + rc;
    const bool ok = q < kRPieces && iy >= 0 && iy < a.H && ix >= 0 && ix < a.W;
    roff[i] = ok ? (unsigned)((((long long)iy * a.W + ix) * a.in_cs + 4 * hh) * 4) : kWOOB;
    roffm[i] = hh ? kWOOB : roff[i];
  }
  auto load_raw = [&](int ck, f32x4 (&r)[2]) {  // chunks past the last reload the last (unused)
#if KRRN_WINO_EXP == 6  // timing experiment: the first chunk's raw input only
    if (ck > 0) return;
#endif
    ck = min(ck, nck - 1);
    const bool half = ck * kWC + 4 >= a.cin;
#pragma unroll
    for (int i = 0; i < 2; ++i)
      r[i] = __builtin_bit_cast(f32x4, __builtin_amdgcn_raw_buffer_load_b128(rsA, half ? roffm[i] : roff[i],
                                                                            ck * kWC * 4, 0));
  };
  int wslot[2];  // this thread's 2 pieces in the padded slot layout (pieces past the region: a dummy slot)
#pragma unroll
  for (int i = 0; i < 2; ++i) {
    const int q = tid + 256 * i;
    const int pix = q >> 1, rr = pix / kRC;
    wslot[i] = q < kRPieces ? ring_slot(rr, pix - rr * kRC, q & 1) : kRDummy;
  }
  auto store_raw = [&](int slot, const f32x4 (&r)[2]) {
    float* dst = smem + slot * kRSlot;
#pragma unroll
    for (int i = 0; i < 2; ++i) *reinterpret_cast<f32x4*>(dst + 4 * wslot[i]) = r[i];
  };

  // split weights, record (chunk, xi, n, half): 16 B of plane U_mh, 8 B of plane U_l. Lanes of n
  // past N read channel N-1 (finite; those output columns are never stored).
  const int fr = lane & 31, h = lane >> 5;
  const long long nrec = (long long)nck * 16 * a.N * 2;
  const char* u3 = reinterpret_cast<const char*>(a.U);
  const __amdgpu_buffer_rsrc_t rsMH =
      __builtin_amdgcn_make_buffer_rsrc((void*)u3, (short)0, (int)min(nrec * 16, 0x7FFFFFFFLL), 0x00020000);
  const __amdgpu_buffer_rsrc_t rsL =
      __builtin_amdgcn_make_buffer_rsrc((void*)(u3 + nrec * 16), (short)0, (int)min(nrec * 8, 0x7FFFFFFFLL), 0x00020000);
  unsigned wrec[kNJ];  // per-lane record part: 2 n + half
#pragma unroll
  for (int j = 0; j < kNJ; ++j) wrec[j] = (unsigned)(2 * min(n0 + 32 * j + fr, a.N - 1) + h);
  u32x4 wmh[4][kNJ];
  u32x2 wl[4][kNJ];
  auto load_wv = [&](int ck, int v) {
#if KRRN_WINO_EXP == 5  // timing experiment: the first chunk's weights only
    if (ck > 0) return;
#endif
    ck = min(ck, nck - 1);
    const unsigned srec = (unsigned)(((ck * 16 + 4 * wave + v) * a.N) * 2);  // uniform
#pragma unroll
    for (int j = 0; j < kNJ; ++j) {
      wmh[v][j] = __builtin_bit_cast(u32x4, __builtin_amdgcn_raw_buffer_load_b128(rsMH, wrec[j] * 16u, srec * 16u, 0));
      wl[v][j] = __builtin_bit_cast(u32x2, __builtin_amdgcn_raw_buffer_load_b64(rsL, wrec[j] * 8u, srec * 8u, 0));
    }
  };

  // this lane's patch rows: t_u = d[ra] +- d[rb] (B^T row u = wave)
  const int ra = wave == 0 ? 0 : (wave == 2 ? 2 : 1);
  const int rb = wave == 0 ? 2 : (wave == 3 ? 3 : (wave == 1 ? 2 : 1));
  const int tx = fr % kGX, ty = fr / kGX;
  const int pa = ring_slot(2 * ty + ra, 2 * tx, h);  // slot of (row ra, patch column 0)
  const int pb = ring_slot(2 * ty + rb, 2 * tx, h);

  f32x16 acc[4][kNJ];
#pragma unroll
  for (int x = 0; x < 4; ++x)
#pragma unroll
    for (int j = 0; j < kNJ; ++j)
#pragma unroll
      for (int r = 0; r < 16; ++r) acc[x][j][r] = 0.f;

  // scalar f32 arithmetic (built without SLP packing: v_pk_*_f32 beside MFMAs costs extra issue)
  const float sgn = wave == 1 ? 1.f : -1.f;
  auto make_v = [&](const float* sl, f32x4 (&V)[4]) {
    f32x4 t[4];
#pragma unroll
    for (int c = 0; c < 4; ++c) {
      const f32x4 da = *reinterpret_cast<const f32x4*>(sl + 4 * (pa + kColOff[c]));
      const f32x4 db = *reinterpret_cast<const f32x4*>(sl + 4 * (pb + kColOff[c]));
#pragma unroll
      for (int e = 0; e < 4; ++e) t[c][e] = __builtin_fmaf(sgn, db[e], da[e]);
    }
#pragma unroll
    for (int e = 0; e < 4; ++e) {
      V[0][e] = t[0][e] - t[2][e];
      V[1][e] = t[1][e] + t[2][e];
      V[2][e] = t[2][e] - t[1][e];
      V[3][e] = t[1][e] - t[3][e];
    }
  };

  f32x4 raw[2];
  load_raw(0, raw);
#pragma unroll
  for (int v = 0; v < 4; ++v) load_wv(0, v);
  store_raw(0, raw);
  load_raw(1, raw);
  __syncthreads();
  store_raw(1, raw);
  load_raw(2, raw);
  __syncthreads();
  for (int ck = 0; ck < nck; ++ck) {
    f32x4 V[4];
    make_v(smem + (ck % 3) * kRSlot, V);
#pragma unroll
    for (int v = 0; v < 4; ++v) {
#if KRRN_WINO_EXP == 8  // timing experiment: no split (V's bits as the operand chain)
      u32x6 ac = {__float_as_uint(V[v][0]), __float_as_uint(V[v][1]), __float_as_uint(V[v][2]),
                  __float_as_uint(V[v][3]), __float_as_uint(V[v][0]), __float_as_uint(V[v][1])};
#else
      u32x6 ac = split3_chain(V[v]);
#endif
      asm volatile("" : "+v"(ac));  // one register tuple: the MFMA operands are its sub-registers
#pragma unroll
      for (int j = 0; j < kNJ; ++j) {
        u32x6 bc = {wmh[v][j][0], wmh[v][j][1], wmh[v][j][2], wmh[v][j][3], wl[v][j][0], wl[v][j][1]};
        asm volatile("" : "+v"(bc));
#if KRRN_WINO_EXP == 7  // timing experiment: no MFMAs (operands still formed and loaded)
        acc[v][j][0] += __uint_as_float(ac[0] ^ ac[4] ^ bc[0] ^ bc[4]);
#else
        acc[v][j] = __builtin_amdgcn_mfma_f32_32x32x16_bf16(sub4(ac, 0), sub4(bc, 0), acc[v][j], 0, 0, 0);  // mm + hh
        acc[v][j] = __builtin_amdgcn_mfma_f32_32x32x16_bf16(sub4(ac, 0), sub4(bc, 2), acc[v][j], 0, 0, 0);  // mh + hl
        acc[v][j] = __builtin_amdgcn_mfma_f32_32x32x16_bf16(sub4(ac, 2), sub4(bc, 0), acc[v][j], 0, 0, 0);  // hm + lh
#endif
      }
      load_wv(ck + 1, v);
      // keep the reload here (hipcc otherwise sinks every weight load below all the MFMAs)
      __builtin_amdgcn_sched_barrier(0);
    }
    store_raw((ck + 2) % 3, raw);
    load_raw(ck + 3, raw);
#if KRRN_WINO_EXP != 10  // timing experiment 10: no barrier per chunk (results wrong)
    __syncthreads();
#endif
  }
#if KRRN_WINO_EXP == 11  // timing experiment: one store per lane instead of the epilogue
  float sum = 0.f;
#pragma unroll
  for (int x = 0; x < 4; ++x)
#pragma unroll
    for (int j = 0; j < kNJ; ++j) sum += acc[x][j][0] + acc[x][j][15];
  if (sum == 12345.f) a.out[tid] = sum;
  return;
#endif
  wino_epi_put(smem, acc);
  __syncthreads();
  if constexpr (HEAD)
    wino_epi_head2d(a, smem, b, ty0, tx0, n0, nb);
  else
    wino_epi_finish2d(a, smem, b, ty0, tx0, n0);
}

}  // namespace

KRRN_API int krrn_conv3x3_wino_f32(const float* in, int in_cs, int in_co, int B, int H, int W, int cin,
                                   const float* U, int N, int n_store, const float* scale, const float* bias,
                                   const float* res, int res_cs, int res_co, float* out, int out_cs, int out_co,
                                   int relu, void* stream) {
  if (!in || !U || !out) return KRRN_EARG;
  if (B < 1 || H < 1 || W < 1 || N < 1 || n_store < 1 || n_store > N) return KRRN_ESHAPE;
  if (cin < 4 || (cin & 3) || in_co + cin > in_cs) return KRRN_EALIGN;
  if (!krrn_aligned16(U) || (((uintptr_t)in) & 3u)) return KRRN_EALIGN;
  if (out_co + n_store > out_cs) return KRRN_ESHAPE;
  WinoArgs a;
  a.in = in; a.in_cs = in_cs; a.in_co = in_co; a.B = B; a.H = H; a.W = W; a.cin = cin;
  a.img = (long long)H * W * in_cs;
  a.U = U; a.N = N; a.n_store = n_store; a.scale = scale; a.bias = bias;
  a.res = res; a.res_cs = res_cs; a.res_co = res_co;
  a.out = out; a.out_cs = out_cs; a.out_co = out_co; a.relu = relu;
  a.w1 = nullptr; a.part = nullptr;
  a.Ht = (H + 1) / 2; a.Wt = (W + 1) / 2;
  const bool ov = !(out_cs & 3) && !(out_co & 3) && krrn_aligned16(out);
  const bool rv = !res || (!(res_cs & 3) && !(res_co & 3) && krrn_aligned16(res));
  const bool sv = (!scale || krrn_aligned16(scale)) && (!bias || krrn_aligned16(bias));
  a.vec = (ov && rv && sv && !(n_store & 3)) ? 1 : 0;
  const long long T = (long long)B * a.Ht * a.Wt;
  if (T > 0x7fffffffLL) return KRRN_ESHAPE;
  a.T = (int)T;
  // 32-bit buffer offsets: the images one block's 32 tiles touch, and the weights
  const long long span = ((kWT + (long long)a.Ht * a.Wt - 1) / ((long long)a.Ht * a.Wt) + 1) * a.img * 4;
  if (span >= 0x7FFF0000LL || (long long)krrn_cdiv(cin, kWC) * 16 * N * kWC * 4 >= 0x7FFF0000LL) return KRRN_ESHAPE;
  const long long blocks = (long long)krrn_cdiv(a.T, kWT) * krrn_cdiv(N, kWN);
  if (blocks > 0x7fffffffLL) return KRRN_ESHAPE;
  const long long rb = (long long)B * krrn_cdiv(a.Ht, kGY) * krrn_cdiv(a.Wt, kGX) * krrn_cdiv(N, kWN);
  if (rb > 0x7fffffffLL || a.img * 4 >= 0x7FFF0000LL) return KRRN_ESHAPE;
  hipLaunchKernelGGL(wino_f23_ring_kernel, dim3((unsigned)rb), dim3(256), 0, (hipStream_t)stream, a);
  return krrn_launch_status();
}

KRRN_API int krrn_conv3x3_wino_x3_f32(const float* in, int in_cs, int in_co, int B, int H, int W, int cin,
                                      const void* U3, int N, int n_store, const float* scale, const float* bias,
                                      const float* res, int res_cs, int res_co, float* out, int out_cs, int out_co,
                                      int relu, void* stream) {
  if (!in || !U3 || !out) return KRRN_EARG;
  if (B < 1 || H < 1 || W < 1 || N < 1 || n_store < 1 || n_store > N) return KRRN_ESHAPE;
  if (cin < 4 || (cin & 3) || in_co + cin > in_cs) return KRRN_EALIGN;
  if (!krrn_aligned16(U3) || (((uintptr_t)in) & 3u)) return KRRN_EALIGN;
  if (out_co + n_store > out_cs) return KRRN_ESHAPE;
  WinoArgs a;
  a.in = in; a.in_cs = in_cs; a.in_co = in_co; a.B = B; a.H = H; a.W = W; a.cin = cin;
  a.img = (long long)H * W * in_cs;
  a.U = reinterpret_cast<const float*>(U3); a.N = N; a.n_store = n_store; a.scale = scale; a.bias = bias;
  a.res = res; a.res_cs = res_cs; a.res_co = res_co;
  a.out = out; a.out_cs = out_cs; a.out_co = out_co; a.relu = relu;
  a.w1 = nullptr; a.part = nullptr;
  a.Ht = (H + 1) / 2; a.Wt = (W + 1) / 2;
  const bool ov = !(out_cs & 3) && !(out_co & 3) && krrn_aligned16(out);
  const bool rv = !res || (!(res_cs & 3) && !(res_co & 3) && krrn_aligned16(res));
  const bool sv = (!scale || krrn_aligned16(scale)) && (!bias || krrn_aligned16(bias));
  a.vec = (ov && rv && sv && !(n_store & 3)) ? 1 : 0;
  const long long T = (long long)B * a.Ht * a.Wt;
  if (T > 0x7fffffffLL) return KRRN_ESHAPE;
  a.T = (int)T;
  // 32-bit buffer offsets: one image, and the U_hm plane (records x 16 B)
  const long long nrec = (long long)krrn_cdiv(cin, kWC) * 16 * N * 2;
  if (a.img * 4 >= 0x7FFF0000LL || nrec * 16 >= 0x7FFF0000LL) return KRRN_ESHAPE;
  const long long rb = (long long)B * krrn_cdiv(a.Ht, kGY) * krrn_cdiv(a.Wt, kGX) * krrn_cdiv(N, kWN);
  if (rb > 0x7fffffffLL) return KRRN_ESHAPE;
  hipLaunchKernelGGL(wino_f23_x3_kernel<false>, dim3((unsigned)rb), dim3(256), 0, (hipStream_t)stream, a);
  return krrn_launch_status();
}

KRRN_API int krrn_conv3x3_wino_x3_head_f32(const float* in, int in_cs, int in_co, int B, int H, int W, int cin,
                                           const void* U3, int N, const float* scale, const float* bias,
                                           const float* res, int res_cs, int res_co, int relu, const float* w1,
                                           const float* b1, int p1, float* part, float* out, int out_c,
                                           void* stream) {
  if (!in || !U3 || !w1 || !part || !out) return KRRN_EARG;
  if (B < 1 || H < 1 || W < 1 || N < 4 || (N & 3) || p1 < 1 || p1 > 4 || out_c < p1) return KRRN_ESHAPE;
  if (cin < 4 || (cin & 3) || in_co + cin > in_cs) return KRRN_EALIGN;
  if (!krrn_aligned16(U3) || (((uintptr_t)in) & 3u) || !krrn_aligned16(w1) || !krrn_aligned16(part)) return KRRN_EALIGN;
  if ((scale && !krrn_aligned16(scale)) || (bias && !krrn_aligned16(bias))) return KRRN_EALIGN;
  if (res && ((res_cs & 3) || (res_co & 3) || !krrn_aligned16(res))) return KRRN_EALIGN;
  WinoArgs a;
  a.in = in; a.in_cs = in_cs; a.in_co = in_co; a.B = B; a.H = H; a.W = W; a.cin = cin;
  a.img = (long long)H * W * in_cs;
  a.U = reinterpret_cast<const float*>(U3); a.N = N; a.n_store = N; a.scale = scale; a.bias = bias;
  a.res = res; a.res_cs = res_cs; a.res_co = res_co;
  a.out = nullptr; a.out_cs = 0; a.out_co = 0; a.relu = relu; a.vec = 1;
  a.w1 = w1; a.part = part;
  a.Ht = (H + 1) / 2; a.Wt = (W + 1) / 2;
  const long long T = (long long)B * a.Ht * a.Wt;
  if (T > 0x7fffffffLL) return KRRN_ESHAPE;
  a.T = (int)T;
  const long long nrec = (long long)krrn_cdiv(cin, kWC) * 16 * N * 2;
  if (a.img * 4 >= 0x7FFF0000LL || nrec * 16 >= 0x7FFF0000LL) return KRRN_ESHAPE;
  const int nbn = krrn_cdiv(N, kWN);
  const long long rb = (long long)B * krrn_cdiv(a.Ht, kGY) * krrn_cdiv(a.Wt, kGX) * nbn;
  const long long M = (long long)B * H * W;
  const long long fb = (M + 255) / 256;
  if (rb > 0x7fffffffLL || fb > 0x7fffffffLL) return KRRN_ESHAPE;
  hipStream_t s = (hipStream_t)stream;
  hipLaunchKernelGGL(wino_f23_x3_kernel<true>, dim3((unsigned)rb), dim3(256), 0, s, a);
  const int st = krrn_launch_status();
  if (st != KRRN_OK) return st;
  hipLaunchKernelGGL(wino_head_finish_kernel, dim3((unsigned)fb), dim3(256), 0, s, part, nbn, M, H * W,
                     b1, p1, out, out_c);
  return krrn_launch_status();
}
