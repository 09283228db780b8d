// Implicit-GEMM convolution / GEMM on the gfx950 f32 matrix cores.
//
// One kernel family serves every dense contraction on the KRRN path (SURVEY §8a rows H1-H8,
// D1-D2, the GCN `feature_map @ weights` of G6/G7 and the TBase Conv1d chain P1):
//
//   out[m, n] = act( scale[n] * sum_k A[m, k] * W[n, k] + bias[n] + bias2[m / b2_div, n]
//                    + res[m, n] )
//
// with A the im2col view of an NHWC activation that is never materialised:
//   m = (b, gy, gx) over a B x Hg x Wg grid, k = (tap, c) over ntaps x cin,
//   A[m, (tap, c)] = in[b, gy*in_s + dy[tap], gx*in_s + dx[tap], c]   (0 outside)
// and the output pixel of grid point (gy, gx) is (gy*osy + ooy, gx*osx + oox).
// A stride-s conv is in_s = s with taps (ky-p, kx-p); a stride-2 transposed conv is four
// launches (one per output parity class) with in_s = 1, osy = osx = 2 and the class's 1..4
// taps (sub-pixel decomposition), so no zero-inserted input exists.
//
// Numerics: operands stay f32 and are multiplied on v_mfma_f32_32x32x2_f32, which is
// bit-for-bit a k-ordered fmaf chain (cdna_hip_programming.md §3 "FP32-input MFMA").
// The reference path evaluates in f32 (tools/trainer.py:466-475 has no autocast at
// eval), so this is the reference precision, not a reduced one. The X3 instantiations
// (krrn_conv2d_x3_f32 / krrn_conv2d_group_x3_f32) keep that accuracy on the bf16 matrix cores:
// both operands split into three exact bf16 terms, six term products per f32 product, f32
// accumulation (see "split-bf16 operands" below); the transposed-conv groups run there.
//
// Tiling (MI355X-first):
//   * block = 256 threads = 4 waves laid out WGM (along M) x 4/WGM (along N); block tile
//     BM x BN, k-tile BK (16 or 32); the tile shapes are a menu the host picks from per layer
//     (128x128 for the wide head convs, 256x32 / 128x32 with 4 waves along M for the
//     18/36-channel HRNet branches so the narrow N is not padded to 64);
//   * both LDS tiles are k-contiguous ([row][k], row pitch BK+4 floats, an odd number of
//     16-B slots) so every 16-lane ds_read_b128 group hits 16 distinct bank slots
//     (conflict-free) and one ds_read_b128 feeds 4 MFMAs (lane half h of MFMA step j reads
//     k = 8*(j/4) + 4h + (j%4) inside each 8-wide k group);
//   * global -> register staging runs two k-tiles ahead (two register sets, loop unrolled
//     by 2 so every index is static), LDS is double buffered, one barrier per k-tile, so a
//     tile's loads have two MFMA phases to land;
//   * blockIdx is remapped XCD-aware so tiles that share an A panel share an L2.
// NCHW=true swaps the MFMA operands (C^T) so the lane index runs over pixels and the
// store into an NCHW tensor is coalesced (used for the heads' final 1x1 convs, whose
// outputs are the NCHW `xyz/mask/region/normal` maps of KRRN.forward, krrn.py:100-108).
#include "krrn_common.h"

namespace {

struct ConvArgs {
  const float* in;
  int in_cs, in_co;
  int B, Hi, Wi;
  int cin;  // physical channels per tap (multiple of 4)
  int Hg, Wg, in_s;
  int ntaps;
  int dy[9];
  int dx[9];
  const float* wt;  // [N][K] row-major, K = ntaps * cin
  int K, N, n_store;
  const float* scale;
  const float* bias;
  const float* bias2;
  int b2_div;
  const float* res;
  int res_cs, res_co;
  float* out;
  int out_cs, out_co;
  int Ho, Wo, osy, osx, ooy, oox;
  int relu;
  int M;
  int tapoff[9];   // element offset of each tap: (dy*Wi + dx)*in_cs
  unsigned cin_magic;  // ceil(2^32 / cin): k / cin == umulhi(k, cin_magic) for k * cin < 2^32
  long long img;   // elements per input image: Hi*Wi*in_cs
  // split-K: blockIdx.y = z owns k-tiles [z*kt_per, (z+1)*kt_per) and writes its raw partial
  // sums to ws[z][M][N]; krrn_splitk_epilogue then adds the partials in z order and applies
  // the epilogue (deterministic: no atomics).
  int kt_per;
  float* ws;
  // channel-chunk-major k (krrn_conv_desc.k_chunk = Q > 0): k = ((c / Q) * ntaps + tap) * Q + c % Q
  int kchunk;
  unsigned kc_magic;  // ceil(2^32 / (Q * ntaps))
  unsigned q_magic;   // ceil(2^32 / Q)
  int vec;  // NHWC epilogue in float4 channel runs (every operand it touches is 16-B aligned)
};

template <int BM, int BN, int BK, int WGM>
struct Cfg {
  static constexpr int WGN = 4 / WGM;
  static constexpr int WTM = BM / WGM, WTN = BN / WGN;
  static constexpr int MI = WTM / 32, NI = WTN / 32;
  static constexpr int KQ = BK / 4;             // float4 per tile row
  static constexpr int RPP = 256 / KQ;          // rows staged per pass
  static constexpr int AL = (BM + RPP - 1) / RPP;
  static constexpr int BL = (BN + RPP - 1) / RPP;
  static constexpr int PITCH = BK + 4;          // odd number of 16-B slots
  static constexpr bool A_FULL = AL * RPP == BM, B_FULL = BL * RPP == BN;  // no partial staging pass
  static constexpr int A_FLOATS = BM * PITCH, B_FLOATS = BN * PITCH;
  // split-bf16 operands (X3): 32 B per 4 k (a bf16 chain) per row, row pitch 2 BK + 4 dwords (an
  // odd number of 16-B slots)
  static constexpr int PX = 2 * BK + 4;
  static constexpr int A_X3 = BM * PX, B_X3 = BN * PX;
  static constexpr int BLOCKS_X3 = 2 * (A_X3 + B_X3) * 4 > 80 * 1024 ? 1 : 2;  // blocks per CU by LDS
  static_assert(MI >= 1 && NI >= 1, "wave tile must be at least 32x32");
  static_assert(BK % 8 == 0, "BK multiple of 8");
};

// ---- split-bf16 operands (X3) ------------------------------------------------------------------
// f32 operands split round-to-nearest into three bf16 terms x = x_h + x_m + x_l (exact, 24
// significand bits); a product is summed over the term pairs hh, hm, mh, hl, lh, mm (the dropped
// ml, lm, ll are below 2^-23 |a b|, the f32 product rounding), accumulated in f32 on
// v_mfma_f32_32x32x16_bf16 (16x the f32 MFMA rate: 2.67x per f32 product). A lane's 8 bf16 of an
// MFMA operand are 2 term kinds x its 4 k (element i of A pairs with element i of B): the
// activations are split once while staged, into the LDS chain [h h m l] per 4 k, the weights on
// the host into [m h l 0] (ops.conv_weights_x3), so the three MFMAs per 8 k read register slices:
//   A[0:3] x B[2:5] = hh + hl,   A[2:5] x B[0:3] = hm + mh,   A[4:7] x B[0:3] = mm + lh.
typedef __bf16 cg_bf16x8 __attribute__((ext_vector_type(8)));
typedef __bf16 cg_bf16x2 __attribute__((ext_vector_type(2)));
typedef float cg_f32x2 __attribute__((ext_vector_type(2)));
typedef unsigned cg_u32x8 __attribute__((ext_vector_type(8)));
typedef unsigned cg_u32x4 __attribute__((ext_vector_type(4)));

__device__ __forceinline__ unsigned cg_pk(float a, float b) {
  return __builtin_bit_cast(unsigned, __builtin_convertvector(cg_f32x2{a, b}, cg_bf16x2));  // RNE
}

__device__ __forceinline__ cg_u32x8 cg_split_chain(const f32x4 x) {
  const unsigned h0 = cg_pk(x[0], x[1]), h1 = cg_pk(x[2], x[3]);
  const float r0 = x[0] - __builtin_bit_cast(float, h0 << 16), r1 = x[1] - __builtin_bit_cast(float, h0 & 0xFFFF0000u);
  const float r2 = x[2] - __builtin_bit_cast(float, h1 << 16), r3 = x[3] - __builtin_bit_cast(float, h1 & 0xFFFF0000u);
  const unsigned m0 = cg_pk(r0, r1), m1 = cg_pk(r2, r3);
  const unsigned l0 = cg_pk(r0 - __builtin_bit_cast(float, m0 << 16), r1 - __builtin_bit_cast(float, m0 & 0xFFFF0000u));
  const unsigned l1 = cg_pk(r2 - __builtin_bit_cast(float, m1 << 16), r3 - __builtin_bit_cast(float, m1 & 0xFFFF0000u));
  return cg_u32x8{h0, h1, h0, h1, m0, m1, l0, l1};
}

__device__ __forceinline__ cg_bf16x8 cg_sub4(const cg_u32x8& c, int o) {
  return __builtin_bit_cast(cg_bf16x8, cg_u32x4{c[o], c[o + 1], c[o + 2], c[o + 3]});
}

template <int AL, int BL, bool X3>
struct Stage {
  f32x4 a[AL];
  f32x4 b[BL][X3 ? 2 : 1];  // X3: the 32-B weight chain of the thread's 4 k
};

// One BM x BN output tile (k-slice z of a split-K problem) of problem `a`; `bid` is the tile's
// linear index (M-major over N tiles). Shared by the single-problem and the grouped kernels.
template <int BM, int BN, int BK, int WGM, bool NCHW, bool X3 = false>
__device__ __forceinline__ void conv_tile(const ConvArgs& a, const int bid, const int z) {
  using C = Cfg<BM, BN, BK, WGM>;
  constexpr int MI = C::MI, NI = C::NI, AL = C::AL, BL = C::BL, PITCH = C::PITCH;
  constexpr int A_FLOATS = X3 ? C::A_X3 : C::A_FLOATS, B_FLOATS = X3 ? C::B_X3 : C::B_FLOATS;
  constexpr int PX = C::PX;
  __shared__ __attribute__((aligned(16))) float smem[2 * (A_FLOATS + B_FLOATS)];

  const int tid = threadIdx.x;
  const int lane = tid & 63, wave = tid >> 6;
  const int wm = wave / C::WGN, wn = wave % C::WGN;

  const int n_tiles = (a.N + BN - 1) / BN;
  const int tm = bid / n_tiles, tn = bid % n_tiles;
  const int m0 = tm * BM, n0 = tn * BN;

  // ---- per-thread staging geometry -------------------------------------------------
  // A and W are read with raw buffer loads: an out-of-range offset returns 0, so the im2col
  // zero padding, the K tail and the M / N edges cost no branch. A's resource starts at the
  // first image the tile touches; row offsets are 32-bit relative to it (host-checked).
  const int srow = tid / C::KQ;
  const int kq = (tid % C::KQ) * 4;  // k offset inside the tile
  const int HWg = a.Hg * a.Wg;
  constexpr unsigned kOOB = 0xFFFFFFF0u;
  const int b0 = min(m0, a.M - 1) / HWg;
  const float* abase = a.in + (size_t)b0 * a.img + a.in_co;
  const long long a_avail = ((long long)(a.B - b0) * a.img - a.in_co) * 4;
  const __amdgpu_buffer_rsrc_t rsA = __builtin_amdgcn_make_buffer_rsrc(
      (void*)abase, (short)0, (int)min(a_avail, (long long)kOOB), 0x00020000);
  constexpr unsigned kWB = X3 ? 8u : 4u;  // weight bytes per k
  const __amdgpu_buffer_rsrc_t rsB = __builtin_amdgcn_make_buffer_rsrc(
      (void*)a.wt, (short)0, (int)min((long long)a.N * a.K * kWB, (long long)kOOB), 0x00020000);
  __shared__ int stap[16];
  if (tid < 16) stap[tid] = tid < a.ntaps ? a.tapoff[tid] : 0;
  unsigned a_row[AL];   // element offset of the row's (gy*s, gx*s) pixel, channel 0
  unsigned a_vm[AL];    // bit t: tap t lands inside the image
#pragma unroll
  for (int i = 0; i < AL; ++i) {
    const int r = srow + C::RPP * i;
    const int m = m0 + r;
    const bool ok = (r < BM) && (m < a.M);
    const int mm = ok ? m : 0;
    const int b = mm / HWg;
    const int rr = mm - b * HWg;
    const int gy = rr / a.Wg, gx = rr - (rr / a.Wg) * a.Wg;
    const int iy0 = gy * a.in_s, ix0 = gx * a.in_s;
    a_row[i] = (unsigned)((long long)(b - b0) * a.img + ((long long)iy0 * a.Wi + ix0) * a.in_cs);
    unsigned vm = 0;
#pragma unroll
    for (int t = 0; t < 9; ++t) {
      const int iy = iy0 + a.dy[t], ix = ix0 + a.dx[t];
      vm |= (t < a.ntaps && iy >= 0 && iy < a.Hi && ix >= 0 && ix < a.Wi) ? (1u << t) : 0u;
    }
    a_vm[i] = ok ? vm : 0u;
  }
  unsigned b_row[BL];  // byte offset of weight row n, or kOOB
#pragma unroll
  for (int i = 0; i < BL; ++i) {
    const int r = srow + C::RPP * i;
    const int n = n0 + r;
    b_row[i] = (r < BN && n < a.N) ? (unsigned)n * (unsigned)a.K * kWB : kOOB;
  }
  const int nkt_all = (a.K + BK - 1) / BK;
  const int kt0 = a.ws ? z * a.kt_per : 0;
  const int nkt = a.ws ? min(a.kt_per, nkt_all - kt0) : nkt_all;
  int kk = kt0 * BK + kq;  // absolute k of this thread's staged float4s
  __syncthreads();  // stap

  auto load_tile = [&](Stage<AL, BL, X3>& st) {
    // (tap, channel) of k without a divide or a data-dependent loop
    int tap, cc;
    if (a.kchunk) {
      const int ch = (int)__umulhi((unsigned)kk, a.kc_magic);
      const int rem = kk - ch * a.kchunk * a.ntaps;
      tap = (int)__umulhi((unsigned)rem, a.q_magic);
      cc = ch * a.kchunk + rem - tap * a.kchunk;
      if (kk >= a.K) tap = 31;  // K tail: no tap, reads 0
    } else {
      tap = (int)__umulhi((unsigned)kk, a.cin_magic);
      cc = kk - tap * a.cin;
    }
    const unsigned toff = (unsigned)(stap[min(tap, 15)] + cc);
#pragma unroll
    for (int i = 0; i < AL; ++i) {
      const bool ok = (a_vm[i] >> min(tap, 31)) & 1u;
      const unsigned off = ok ? (a_row[i] + toff) * 4u : kOOB;
      st.a[i] = __builtin_bit_cast(f32x4, __builtin_amdgcn_raw_buffer_load_b128(rsA, off, 0, 0));
    }
    const bool k_ok = kk < a.K;
#pragma unroll
    for (int i = 0; i < BL; ++i) {
      const unsigned off = k_ok ? b_row[i] + (unsigned)kk * kWB : kOOB;
#pragma unroll
      for (int h = 0; h < (X3 ? 2 : 1); ++h)
        st.b[i][h] = __builtin_bit_cast(f32x4, __builtin_amdgcn_raw_buffer_load_b128(rsB, off + 16u * h, 0, 0));
    }
    kk += BK;
  };
  auto store_tile = [&](const Stage<AL, BL, X3>& st, int buf) {
    float* As = smem + buf * (A_FLOATS + B_FLOATS);
    float* Bs = As + A_FLOATS;
#pragma unroll
    for (int i = 0; i < AL; ++i) {
      const int r = srow + C::RPP * i;
      if (!(C::A_FULL || r < BM)) continue;
      if constexpr (X3) {
        const cg_u32x8 c = cg_split_chain(st.a[i]);
        unsigned* d = reinterpret_cast<unsigned*>(As) + r * PX + 2 * kq;
        *reinterpret_cast<cg_u32x4*>(d) = cg_u32x4{c[0], c[1], c[2], c[3]};
        *reinterpret_cast<cg_u32x4*>(d + 4) = cg_u32x4{c[4], c[5], c[6], c[7]};
      } else {
        *reinterpret_cast<f32x4*>(As + r * PITCH + kq) = st.a[i];
      }
    }
#pragma unroll
    for (int i = 0; i < BL; ++i) {
      const int r = srow + C::RPP * i;
      if (!(C::B_FULL || r < BN)) continue;
      if constexpr (X3) {
        float* d = Bs + r * PX + 2 * kq;
        *reinterpret_cast<f32x4*>(d) = st.b[i][0];
        *reinterpret_cast<f32x4*>(d + 4) = st.b[i][X3 ? 1 : 0];
      } else {
        *reinterpret_cast<f32x4*>(Bs + r * PITCH + kq) = st.b[i][0];
      }
    }
  };

  f32x16 acc[MI][NI];
#pragma unroll
  for (int i = 0; i < MI; ++i)
#pragma unroll
    for (int j = 0; j < NI; ++j)
#pragma unroll
      for (int r = 0; r < 16; ++r) acc[i][j][r] = 0.f;

  const int frow = lane & 31, fh = lane >> 5;
  auto compute_x3 = [&](int buf) {
    const unsigned* As = reinterpret_cast<const unsigned*>(smem + buf * (A_FLOATS + B_FLOATS));
    const unsigned* Bs = As + A_FLOATS;
#pragma unroll
    for (int g = 0; g < BK / 8; ++g) {
      const int q = 2 * g + fh;  // this lane half's 4 k of the 8-wide group
      cg_u32x8 af[MI], bf[NI];
#pragma unroll
      for (int i = 0; i < MI; ++i) {
        const unsigned* p = As + (wm * C::WTM + i * 32 + frow) * PX + 8 * q;
        const cg_u32x4 lo = *reinterpret_cast<const cg_u32x4*>(p), hi = *reinterpret_cast<const cg_u32x4*>(p + 4);
        af[i] = cg_u32x8{lo[0], lo[1], lo[2], lo[3], hi[0], hi[1], hi[2], hi[3]};
        // one 8-register tuple: both LDS reads land in it and the MFMA operands are its
        // sub-registers (LLVM otherwise rebuilt the overlapping slices with register copies)
        asm volatile("" : "+v"(af[i]));
      }
#pragma unroll
      for (int j = 0; j < NI; ++j) {
        const unsigned* p = Bs + (wn * C::WTN + j * 32 + frow) * PX + 8 * q;
        const cg_u32x4 lo = *reinterpret_cast<const cg_u32x4*>(p), hi = *reinterpret_cast<const cg_u32x4*>(p + 4);
        bf[j] = cg_u32x8{lo[0], lo[1], lo[2], lo[3], hi[0], hi[1], hi[2], hi[3]};
        asm volatile("" : "+v"(bf[j]));
      }
#pragma unroll
      for (int i = 0; i < MI; ++i)
#pragma unroll
        for (int j = 0; j < NI; ++j) {
          f32x16& d = acc[i][j];
          if constexpr (NCHW) {
            d = __builtin_amdgcn_mfma_f32_32x32x16_bf16(cg_sub4(bf[j], 2), cg_sub4(af[i], 0), d, 0, 0, 0);
            d = __builtin_amdgcn_mfma_f32_32x32x16_bf16(cg_sub4(bf[j], 0), cg_sub4(af[i], 2), d, 0, 0, 0);
            d = __builtin_amdgcn_mfma_f32_32x32x16_bf16(cg_sub4(bf[j], 0), cg_sub4(af[i], 4), d, 0, 0, 0);
          } else {
            d = __builtin_amdgcn_mfma_f32_32x32x16_bf16(cg_sub4(af[i], 0), cg_sub4(bf[j], 2), d, 0, 0, 0);
            d = __builtin_amdgcn_mfma_f32_32x32x16_bf16(cg_sub4(af[i], 2), cg_sub4(bf[j], 0), d, 0, 0, 0);
            d = __builtin_amdgcn_mfma_f32_32x32x16_bf16(cg_sub4(af[i], 4), cg_sub4(bf[j], 0), d, 0, 0, 0);
          }
        }
    }
  };
  auto compute = [&](int buf) {
    if constexpr (X3) {
      compute_x3(buf);
      return;
    }
    const float* As = smem + buf * (A_FLOATS + B_FLOATS);
    const float* Bs = As + A_FLOATS;
#pragma unroll
    for (int g = 0; g < BK / 8; ++g) {
      f32x4 af[MI], bf[NI];
#pragma unroll
      for (int i = 0; i < MI; ++i)
        af[i] = *reinterpret_cast<const f32x4*>(As + (wm * C::WTM + i * 32 + frow) * PITCH + g * 8 + 4 * fh);
#pragma unroll
      for (int j = 0; j < NI; ++j)
        bf[j] = *reinterpret_cast<const f32x4*>(Bs + (wn * C::WTN + j * 32 + frow) * PITCH + g * 8 + 4 * fh);
#pragma unroll
      for (int s = 0; s < 4; ++s)
#pragma unroll
        for (int i = 0; i < MI; ++i)
#pragma unroll
          for (int j = 0; j < NI; ++j) {
            if constexpr (NCHW)
              acc[i][j] = __builtin_amdgcn_mfma_f32_32x32x2f32(bf[j][s], af[i][s], acc[i][j], 0, 0, 0);
            else
              acc[i][j] = __builtin_amdgcn_mfma_f32_32x32x2f32(af[i][s], bf[j][s], acc[i][j], 0, 0, 0);
          }
    }
  };

  // ---- main loop: loads two tiles ahead, LDS double-buffered, unrolled by 2 ---------------
  Stage<AL, BL, X3> s0, s1;
  load_tile(s0);
  if (nkt > 1) load_tile(s1);
  store_tile(s0, 0);
  __syncthreads();
  for (int kt = 0; kt < nkt; kt += 2) {
    if (kt + 2 < nkt) load_tile(s0);
    compute(0);
    if (kt + 1 < nkt) store_tile(s1, 1);
    __syncthreads();
    if (kt + 1 >= nkt) break;
    if (kt + 3 < nkt) load_tile(s1);
    compute(1);
    if (kt + 2 < nkt) store_tile(s0, 0);
    __syncthreads();
  }

  // ---- epilogue -----------------------------------------------------------------------
  if constexpr (!NCHW) {
    if (a.ws) {  // split-K partial: raw sums, N-contiguous rows
      float* w = a.ws + (size_t)z * a.M * a.N;
#pragma unroll
      for (int i = 0; i < MI; ++i)
#pragma unroll
        for (int j = 0; j < NI; ++j) {
          const int n = n0 + wn * C::WTN + j * 32 + frow;
          if (n >= a.N) continue;
#pragma unroll
          for (int r = 0; r < 16; ++r) {
            const int m = m0 + wm * C::WTM + i * 32 + (r & 3) + 8 * (r >> 2) + 4 * fh;
            if (m < a.M) w[(size_t)m * a.N + n] = acc[i][j][r];
          }
        }
      return;
    }
  }
  // output-row table in LDS (the main loop ended on a barrier): image and output pixel of each
  // of the tile's BM rows, computed once per row instead of once per accumulator element
  const int HWo = a.Ho * a.Wo;
  int* s_b = reinterpret_cast<int*>(smem);
  int* s_sp = s_b + BM;
  int* s_b2 = s_sp + BM;
  for (int r = tid; r < BM; r += 256) {
    const int m = min(m0 + r, a.M - 1);
    const int b = m / HWg;
    const int rr = m - b * HWg;
    const int gy = rr / a.Wg, gx = rr - (rr / a.Wg) * a.Wg;
    s_b[r] = b;
    s_sp[r] = (gy * a.osy + a.ooy) * a.Wo + gx * a.osx + a.oox;
    s_b2[r] = m / a.b2_div;
  }
  __syncthreads();
  if constexpr (!NCHW) {
    if (a.vec) {
      // each 32x32 accumulator tile goes through a per-wave LDS square ([row][n], pitch 32: the
      // ds_write_b32 halves and the ds_read_b128 lane groups are conflict-free) and leaves as float4
      // channel runs: 4 store instructions per lane and tile instead of 16 scalar ones
      static_assert(3 * BM + 4 * 1024 <= 2 * (A_FLOATS + B_FLOATS), "epilogue square does not fit");
      float* sq = smem + 3 * BM + wave * 1024;
      const int rq = lane >> 3, cq = 4 * (lane & 7);
#pragma unroll
      for (int i = 0; i < MI; ++i)
#pragma unroll
        for (int j = 0; j < NI; ++j) {
#pragma unroll
          for (int r = 0; r < 16; ++r) sq[((r & 3) + 8 * (r >> 2) + 4 * fh) * 32 + frow] = acc[i][j][r];
          __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
          __builtin_amdgcn_wave_barrier();
          __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
          f32x4 v[4];
#pragma unroll
          for (int p = 0; p < 4; ++p) v[p] = *reinterpret_cast<const f32x4*>(sq + (rq + 8 * p) * 32 + cq);
          __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
          __builtin_amdgcn_wave_barrier();
          __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
          const int n = n0 + wn * C::WTN + j * 32 + cq;
          if (n >= a.n_store) continue;  // n_store is a multiple of 4
          const f32x4 sc = a.scale ? *reinterpret_cast<const f32x4*>(a.scale + n) : f32x4{1.f, 1.f, 1.f, 1.f};
          const f32x4 bi = a.bias ? *reinterpret_cast<const f32x4*>(a.bias + n) : f32x4{0.f, 0.f, 0.f, 0.f};
#pragma unroll
          for (int p = 0; p < 4; ++p) {
            const int row = wm * C::WTM + i * 32 + rq + 8 * p;
            if (m0 + row >= a.M) continue;
            const size_t pix = (size_t)s_b[row] * HWo + s_sp[row];
            f32x4 o = v[p] * sc + bi;
            if (a.bias2) o += *reinterpret_cast<const f32x4*>(a.bias2 + (size_t)s_b2[row] * a.N + n);
            if (a.res) o += *reinterpret_cast<const f32x4*>(a.res + pix * a.res_cs + a.res_co + n);
            if (a.relu) {
#pragma unroll
              for (int e = 0; e < 4; ++e) o[e] = fmaxf(o[e], 0.f);
            }
            *reinterpret_cast<f32x4*>(a.out + pix * a.out_cs + a.out_co + n) = o;
          }
        }
      return;
    }
  }
#pragma unroll
  for (int i = 0; i < MI; ++i)
#pragma unroll
    for (int j = 0; j < NI; ++j) {
      if constexpr (!NCHW) {
        const int n = n0 + wn * C::WTN + j * 32 + frow;
        if (n >= a.n_store) continue;
        const float sc = a.scale ? a.scale[n] : 1.f;
        const float bi = a.bias ? a.bias[n] : 0.f;
#pragma unroll
        for (int r = 0; r < 16; ++r) {
          const int row = wm * C::WTM + i * 32 + (r & 3) + 8 * (r >> 2) + 4 * fh;
          if (m0 + row >= a.M) continue;
          const size_t pix = (size_t)s_b[row] * HWo + s_sp[row];
          float v = acc[i][j][r] * sc + bi;
          if (a.bias2) v += a.bias2[(size_t)s_b2[row] * a.N + n];
          if (a.res) v += a.res[pix * a.res_cs + a.res_co + n];
          if (a.relu) v = fmaxf(v, 0.f);
          a.out[pix * a.out_cs + a.out_co + n] = v;
        }
      } else {
        const int row = wm * C::WTM + i * 32 + frow;
        if (m0 + row >= a.M) continue;
        const int b = s_b[row], sp = s_sp[row], b2r = s_b2[row];
#pragma unroll
        for (int r = 0; r < 16; ++r) {
          const int n = n0 + wn * C::WTN + j * 32 + (r & 3) + 8 * (r >> 2) + 4 * fh;
          if (n >= a.n_store) continue;
          float v = acc[i][j][r] * (a.scale ? a.scale[n] : 1.f) + (a.bias ? a.bias[n] : 0.f);
          if (a.bias2) v += a.bias2[(size_t)b2r * a.N + n];
          if (a.relu) v = fmaxf(v, 0.f);
          a.out[((size_t)b * a.out_cs + a.out_co + n) * HWo + sp] = v;
        }
      }
    }
}

template <int BM, int BN, int BK, int WGM, bool NCHW, bool X3 = false>
__global__ __launch_bounds__(256, (X3 ? Cfg<BM, BN, BK, WGM>::BLOCKS_X3 : 2)) void conv_gemm_f32_kernel(const ConvArgs a) {
  const int tiles = krrn_cdiv(a.M, BM) * krrn_cdiv(a.N, BN);
  conv_tile<BM, BN, BK, WGM, NCHW, X3>(a, krrn_xcd_remap(blockIdx.x, tiles), blockIdx.y);
}

// Grouped launch: up to kMaxGroup independent problems of one tile shape in one grid (the
// HRNet branches' convs at the same block depth: 20/36/72/144 channels at 30/15/8/4 px, each
// alone far too small to fill 256 CUs). Problem q owns blocks [start[q], start[q+1]), split
// into tiles[q] output tiles x splits[q] k-slices.
constexpr int kMaxGroup = 4;
struct ConvGroup {
  int n;
  int inter;  // every problem has the same tile grid and no split-K: blocks interleaved by problem
  int start[kMaxGroup + 1];
  int tiles[kMaxGroup];
  int estart[kMaxGroup + 1];  // split-K epilogue blocks
  int splits[kMaxGroup];
  ConvArgs p[kMaxGroup];
};

template <int BM, int BN, int BK, int WGM, bool X3 = false>
__global__ __launch_bounds__(256, (X3 ? Cfg<BM, BN, BK, WGM>::BLOCKS_X3 : 2)) void conv_group_kernel(const ConvGroup g) {
  const int lin = krrn_xcd_remap(blockIdx.x, g.start[g.n]);
  if (g.inter) {
    // the n problems' tiles of one output region are consecutive blocks, so they land on one XCD
    // at about the same time: a transposed conv's parity classes read the same input rows (each
    // input pixel feeds all four classes), fetched from HBM once into that XCD's L2 instead of once
    // per class (round 3: 653 MB read per launch for 63 MB of input)
    const int q = lin % g.n;
    conv_tile<BM, BN, BK, WGM, false, X3>(g.p[q], lin / g.n, 0);
    return;
  }
  int q = 0;
#pragma unroll
  for (int i = 1; i < kMaxGroup; ++i) q += (i < g.n && lin >= g.start[i]) ? 1 : 0;
  const int local = lin - g.start[q];
  const int tiles = g.tiles[q];
  conv_tile<BM, BN, BK, WGM, false, X3>(g.p[q], local % tiles, local / tiles);
}

// Sum of the split-K partials in z order + the conv epilogue (NHWC output). One thread per
// (m, 4 channels).
__device__ __forceinline__ void splitk_epilogue(const ConvArgs& a, int splits, long long t) {
  const int nq = a.n_store >> 2;
  if (t >= (long long)a.M * nq) return;
  const int m = (int)(t / nq);
  const int n = (int)(t - (long long)m * nq) * 4;
  const size_t plane = (size_t)a.M * a.N;
  const float* w = a.ws + (size_t)m * a.N + n;
  f32x4 v = *reinterpret_cast<const f32x4*>(w);
  for (int z = 1; z < splits; ++z) v += *reinterpret_cast<const f32x4*>(w + z * plane);
  const int HWg = a.Hg * a.Wg;
  const int b = m / HWg;
  const int rr = m - b * HWg;
  const int gy = rr / a.Wg, gx = rr - (rr / a.Wg) * a.Wg;
  const int oy = gy * a.osy + a.ooy, ox = gx * a.osx + a.oox;
  const size_t pix = ((size_t)b * a.Ho + oy) * a.Wo + ox;
#pragma unroll
  for (int q = 0; q < 4; ++q) {
    float x = v[q] * (a.scale ? a.scale[n + q] : 1.f) + (a.bias ? a.bias[n + q] : 0.f);
    if (a.bias2) x += a.bias2[(size_t)(m / a.b2_div) * a.N + n + q];
    if (a.res) x += a.res[pix * a.res_cs + a.res_co + n + q];
    if (a.relu) x = fmaxf(x, 0.f);
    a.out[pix * a.out_cs + a.out_co + n + q] = x;
  }
}

__global__ __launch_bounds__(256) void splitk_epilogue_kernel(const ConvArgs a, int splits) {
  splitk_epilogue(a, splits, (long long)blockIdx.x * 256 + threadIdx.x);
}

__global__ __launch_bounds__(256) void splitk_epilogue_group_kernel(const ConvGroup g) {
  int q = 0;
#pragma unroll
  for (int i = 1; i < kMaxGroup; ++i) q += (i < g.n && (int)blockIdx.x >= g.estart[i]) ? 1 : 0;
  if (g.splits[q] <= 1) return;
  splitk_epilogue(g.p[q], g.splits[q], (long long)(blockIdx.x - g.estart[q]) * 256 + threadIdx.x);
}

template <int BM, int BN, int BK, int WGM, bool NCHW, bool X3 = false>
int launch(const ConvArgs& a, int splits, hipStream_t s) {
  const int nwg = krrn_cdiv(a.M, BM) * krrn_cdiv(a.N, BN);
  hipLaunchKernelGGL((conv_gemm_f32_kernel<BM, BN, BK, WGM, NCHW, X3>), dim3(nwg, a.ws ? splits : 1), dim3(256), 0, s,
                     a);
  if (a.ws) {
    const long long threads = (long long)a.M * (a.n_store >> 2);
    hipLaunchKernelGGL(splitk_epilogue_kernel, dim3((unsigned)((threads + 255) / 256)), dim3(256), 0, s, a,
                       splits);
  }
  return krrn_launch_status();
}

template <int BM, int BN, int BK, int WGM, bool X3 = false>
int launch_group(ConvGroup& g, hipStream_t s) {
  int blocks = 0, eblocks = 0;
  for (int q = 0; q < g.n; ++q) {
    const ConvArgs& a = g.p[q];
    g.tiles[q] = krrn_cdiv(a.M, BM) * krrn_cdiv(a.N, BN);
    g.start[q] = blocks;
    blocks += g.tiles[q] * (a.ws ? g.splits[q] : 1);
    g.estart[q] = eblocks;
    if (a.ws) eblocks += (int)(((long long)a.M * (a.n_store >> 2) + 255) / 256);
  }
  for (int q = g.n; q <= kMaxGroup; ++q) {
    if (q < kMaxGroup) { g.tiles[q] = 1; g.splits[q] = 1; }
    g.start[q] = blocks;
    g.estart[q] = eblocks;
  }
  g.inter = eblocks == 0 ? 1 : 0;
  for (int q = 1; q < g.n; ++q) g.inter &= g.tiles[q] == g.tiles[0] ? 1 : 0;
  hipLaunchKernelGGL((conv_group_kernel<BM, BN, BK, WGM, X3>), dim3(blocks), dim3(256), 0, s, g);
  if (eblocks) hipLaunchKernelGGL(splitk_epilogue_group_kernel, dim3(eblocks), dim3(256), 0, s, g);
  return krrn_launch_status();
}

int tile_bk(int tile) { return (tile == 1 || tile == 2 || tile == 3 || tile == 5) ? 16 : 32; }

// Validate one problem and pack its kernel arguments; resolves tile 0 and the effective
// split count (every k-slice non-empty).
int prepare(const krrn_conv_desc& d, int& tile, ConvArgs& a, int& splits, bool x3 = false) {
  const int B = d.B, Hi = d.Hi, Wi = d.Wi, Hg = d.Hg, Wg = d.Wg, N = d.N, cin = d.cin, ntaps = d.ntaps;
  if (!d.in || !d.wt || !d.out) return KRRN_EARG;
  if (ntaps < 1 || ntaps > 9 || B < 1 || Hi < 1 || Wi < 1 || Hg < 1 || Wg < 1 || N < 1) return KRRN_ESHAPE;
  if (cin < 4 || (cin & 3) || (d.in_cs & 3) || (d.in_co & 3) || d.in_co + cin > d.in_cs) return KRRN_EALIGN;
  if (!krrn_aligned16(d.in) || !krrn_aligned16(d.wt)) return KRRN_EALIGN;
  if (d.n_store < 1 || d.n_store > N) return KRRN_ESHAPE;
  if (d.bias2 && d.b2_div < 1) return KRRN_EARG;
  if (!d.out_nchw && d.out_co + d.n_store > d.out_cs) return KRRN_ESHAPE;
  if (tile < 0 || tile > 8) return KRRN_EARG;
  const long long M = (long long)B * Hg * Wg;
  if (M > 0x7fffffffLL) return KRRN_ESHAPE;
  splits = d.splits;
  if (splits < 1 || splits > 64) return KRRN_EARG;
  if (splits > 1) {
    if (!d.workspace || d.out_nchw) return KRRN_EARG;
    if ((N & 3) || (d.n_store & 3)) return KRRN_EALIGN;
    if (!krrn_aligned16(d.workspace)) return KRRN_EALIGN;
  }
  a.in = d.in; a.in_cs = d.in_cs; a.in_co = d.in_co; a.B = B; a.Hi = Hi; a.Wi = Wi; a.cin = cin;
  a.Hg = Hg; a.Wg = Wg; a.in_s = d.in_s; a.ntaps = ntaps;
  for (int t = 0; t < 9; ++t) { a.dy[t] = t < ntaps ? d.tap_dy[t] : 0; a.dx[t] = t < ntaps ? d.tap_dx[t] : 0; }
  a.wt = d.wt; a.K = ntaps * cin; a.N = N; a.n_store = d.n_store;
  a.scale = d.scale; a.bias = d.bias; a.bias2 = d.bias2; a.b2_div = d.b2_div > 0 ? d.b2_div : 1;
  a.res = d.res; a.res_cs = d.res_cs; a.res_co = d.res_co;
  a.out = d.out; a.out_cs = d.out_cs; a.out_co = d.out_co; a.Ho = d.Ho; a.Wo = d.Wo;
  a.osy = d.osy; a.osx = d.osx; a.ooy = d.ooy; a.oox = d.oox; a.relu = d.relu; a.M = (int)M;
  for (int t = 0; t < 9; ++t) a.tapoff[t] = (a.dy[t] * Wi + a.dx[t]) * d.in_cs;
  a.img = (long long)Hi * Wi * d.in_cs;
  a.cin_magic = (unsigned)((0x100000000ULL + cin - 1) / cin);
  if ((long long)(a.K + 64) * cin >= 0x100000000LL) return KRRN_ESHAPE;
  a.kchunk = d.k_chunk;
  a.kc_magic = a.q_magic = 0;
  if (d.k_chunk) {
    const int Q = d.k_chunk;
    if (Q < 0 || (Q & 3) || cin % Q) return KRRN_EALIGN;
    a.kc_magic = (unsigned)((0x100000000ULL + Q * ntaps - 1) / (Q * ntaps));
    a.q_magic = (unsigned)((0x100000000ULL + Q - 1) / Q);
    if ((long long)(a.K + 64) * Q * ntaps >= 0x100000000LL) return KRRN_ESHAPE;
  }
  // 32-bit buffer offsets: the images one tile can touch (<= 256 rows) and the weights
  const long long HWg = (long long)Hg * Wg;
  const long long span = ((256 + HWg - 1) / HWg + 1) * a.img * 4;
  if (span >= 0xFFFFFFF0LL || (long long)N * a.K * (x3 ? 8 : 4) >= 0xFFFFFFF0LL) return KRRN_ESHAPE;
  if (tile == 0) tile = d.out_nchw ? 3 : (N <= 32 ? 6 : 8);  // same rule as runtime.conv_tile
  a.ws = nullptr;
  a.kt_per = 0;
  if (splits > 1) {
    const int nkt = krrn_cdiv(a.K, tile_bk(tile));
    a.kt_per = krrn_cdiv(nkt, splits);
    splits = krrn_cdiv(nkt, a.kt_per);
    if (splits > 1) a.ws = d.workspace;
  }
  if (splits < 1) splits = 1;
  a.vec = !d.out_nchw && !(d.n_store & 3) && !(d.out_cs & 3) && !(d.out_co & 3) && krrn_aligned16(d.out) &&
          (!d.scale || krrn_aligned16(d.scale)) && (!d.bias || krrn_aligned16(d.bias)) &&
          (!d.bias2 || (!(N & 3) && krrn_aligned16(d.bias2))) &&
          (!d.res || (!(d.res_cs & 3) && !(d.res_co & 3) && krrn_aligned16(d.res)));
  return KRRN_OK;
}

}  // namespace

namespace {
int conv2d(const float* in, int in_cs, int in_co, int B, int Hi, int Wi, int cin, int Hg, int Wg, int in_s, int ntaps,
           const int* tap_dy, const int* tap_dx, const void* wt, int N, int n_store, const float* scale,
           const float* bias, const float* bias2, int b2_div, const float* res, int res_cs, int res_co, float* out,
           int out_cs, int out_co, int Ho, int Wo, int osy, int osx, int ooy, int oox, int relu, int out_nchw,
           int tile, int splits, float* workspace, bool x3, void* stream) {
  if (!tap_dy || !tap_dx) return KRRN_EARG;
  if (ntaps < 1 || ntaps > 9) return KRRN_ESHAPE;
  krrn_conv_desc d;
  d.in = in; d.in_cs = in_cs; d.in_co = in_co; d.B = B; d.Hi = Hi; d.Wi = Wi; d.cin = cin;
  d.Hg = Hg; d.Wg = Wg; d.in_s = in_s; d.ntaps = ntaps;
  for (int t = 0; t < 9; ++t) { d.tap_dy[t] = t < ntaps ? tap_dy[t] : 0; d.tap_dx[t] = t < ntaps ? tap_dx[t] : 0; }
  d.wt = reinterpret_cast<const float*>(wt); d.N = N; d.n_store = n_store; d.scale = scale; d.bias = bias;
  d.bias2 = bias2; d.b2_div = b2_div;
  d.res = res; d.res_cs = res_cs; d.res_co = res_co; d.out = out; d.out_cs = out_cs; d.out_co = out_co;
  d.Ho = Ho; d.Wo = Wo; d.osy = osy; d.osx = osx; d.ooy = ooy; d.oox = oox; d.relu = relu;
  d.out_nchw = out_nchw; d.splits = splits; d.workspace = workspace; d.k_chunk = 0;
  ConvArgs a;
  int sp = 1;
  const int st = prepare(d, tile, a, sp, x3);
  if (st != KRRN_OK) return st;
  hipStream_t s = (hipStream_t)stream;
  if (x3) {  // NHWC output
    if (out_nchw) return KRRN_EARG;
    switch (tile) {
      case 1: return launch<128, 128, 16, 2, false, true>(a, sp, s);
      case 2: return launch<128, 64, 16, 2, false, true>(a, sp, s);
      case 3: return launch<64, 64, 16, 2, false, true>(a, sp, s);
      case 4: return launch<128, 128, 32, 2, false, true>(a, sp, s);
      case 5: return launch<256, 32, 16, 4, false, true>(a, sp, s);
      case 6: return launch<128, 32, 32, 4, false, true>(a, sp, s);
      case 7: return launch<128, 64, 32, 2, false, true>(a, sp, s);
      default: return launch<64, 64, 32, 2, false, true>(a, sp, s);
    }
  }
  if (out_nchw) {
    // narrow heads (mask/region/xyz logits, 3C normals): 32-wide N tiles waste least MFMA work
    if (tile == 6) return launch<128, 32, 32, 4, true>(a, 1, s);
    if (tile == 1 || tile == 4) return launch<128, 128, 16, 2, true>(a, 1, s);
    if (tile == 2 || tile == 7) return launch<128, 64, 16, 2, true>(a, 1, s);
    return launch<64, 64, 16, 2, true>(a, 1, s);
  }
  switch (tile) {
    case 1: return launch<128, 128, 16, 2, false>(a, sp, s);
    case 2: return launch<128, 64, 16, 2, false>(a, sp, s);
    case 3: return launch<64, 64, 16, 2, false>(a, sp, s);
    case 4: return launch<128, 128, 32, 2, false>(a, sp, s);
    case 5: return launch<256, 32, 16, 4, false>(a, sp, s);
    case 6: return launch<128, 32, 32, 4, false>(a, sp, s);
    case 7: return launch<128, 64, 32, 2, false>(a, sp, s);
    default: return launch<64, 64, 32, 2, false>(a, sp, s);
  }
}
}  // namespace

// Tile menu (include/krrn_hip.h): 1 128x128x16, 2 128x64x16, 3 64x64x16, 4 128x128x32,
// 5 256x32x16 (4 waves along M), 6 128x32x32 (4 waves along M), 7 128x64x32, 8 64x64x32.
KRRN_API int krrn_conv2d_f32(const float* in, int in_cs, int in_co, int B, int Hi, int Wi, int cin,
                             int Hg, int Wg, int in_s, int ntaps, const int* tap_dy, const int* tap_dx,
                             const float* wt, int N, int n_store, const float* scale, const float* bias,
                             const float* bias2, int b2_div, const float* res, int res_cs, int res_co,
                             float* out, int out_cs, int out_co, int Ho, int Wo, int osy, int osx, int ooy,
                             int oox, int relu, int out_nchw, int tile, int splits, float* workspace,
                             void* stream) {
  return conv2d(in, in_cs, in_co, B, Hi, Wi, cin, Hg, Wg, in_s, ntaps, tap_dy, tap_dx, wt, N, n_store, scale, bias,
                bias2, b2_div, res, res_cs, res_co, out, out_cs, out_co, Ho, Wo, osy, osx, ooy, oox, relu, out_nchw,
                tile, splits, workspace, false, stream);
}

KRRN_API int krrn_conv2d_x3_f32(const float* in, int in_cs, int in_co, int B, int Hi, int Wi, int cin, int Hg,
                                int Wg, int in_s, int ntaps, const int* tap_dy, const int* tap_dx, const void* wt3,
                                int N, int n_store, const float* scale, const float* bias, const float* bias2,
                                int b2_div, const float* res, int res_cs, int res_co, float* out, int out_cs,
                                int out_co, int Ho, int Wo, int osy, int osx, int ooy, int oox, int relu, int tile,
                                int splits, float* workspace, void* stream) {
  return conv2d(in, in_cs, in_co, B, Hi, Wi, cin, Hg, Wg, in_s, ntaps, tap_dy, tap_dx, wt3, N, n_store, scale, bias,
                bias2, b2_div, res, res_cs, res_co, out, out_cs, out_co, Ho, Wo, osy, osx, ooy, oox, relu, 0, tile,
                splits, workspace, true, stream);
}

namespace {
int conv_group(const krrn_conv_desc* descs, int n, int tile, bool x3, void* stream) {
  if (!descs) return KRRN_EARG;
  if (n < 1 || n > kMaxGroup) return KRRN_ESHAPE;
  if (tile != 1 && tile != 6 && tile != 8) return KRRN_EARG;
  ConvGroup g;
  g.n = n;
  for (int q = 0; q < n; ++q) {
    if (descs[q].out_nchw) return KRRN_EARG;
    int t = tile;
    const int st = prepare(descs[q], t, g.p[q], g.splits[q], x3);
    if (st != KRRN_OK) return st;
  }
  hipStream_t s = (hipStream_t)stream;
  if (x3) {
    if (tile == 1) return launch_group<128, 128, 16, 2, true>(g, s);
    return tile == 6 ? launch_group<128, 32, 32, 4, true>(g, s) : launch_group<64, 64, 32, 2, true>(g, s);
  }
  if (tile == 1) return launch_group<128, 128, 16, 2>(g, s);
  if (tile == 6) return launch_group<128, 32, 32, 4>(g, s);
  return launch_group<64, 64, 32, 2>(g, s);
}
}  // namespace

KRRN_API int krrn_conv2d_group_f32(const krrn_conv_desc* descs, int n, int tile, void* stream) {
  return conv_group(descs, n, tile, false, stream);
}

KRRN_API int krrn_conv2d_group_x3_f32(const krrn_conv_desc* descs, int n, int tile, void* stream) {
  return conv_group(descs, n, tile, true, stream);
}
