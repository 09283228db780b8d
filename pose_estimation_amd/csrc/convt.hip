// Stride-2 transposed convolution (ConvTranspose2d, stride 2, kernel <= 4, padding 1) on the bf16
// matrix cores at f32 accuracy (split-bf16, as everywhere): the backbone's deconv (4x4, 272 -> 128,
// the folded deconv_layer of myhrnet.py:314-326) and XYZNet's first layer (3x3, output_padding 1,
// 128 -> 128, lib/network/krrn.py:47-49), both 30 -> 60 px.
//
// Sub-pixel form: output pixel (2a + py, 2b + px) of parity class c = (py, px) is
//   out[2a+py][2b+px][n] = act(scale[n] * sum_{t in taps(c)} sum_k in[a+dy_t][b+dx_t][k] W_c,t[k][n] + bias[n])
// with 1-4 taps per class, (dy, dx) in {-1, 0, 1}^2 (ops.make_convT). The grouped implicit GEMM
// (conv_gemm.hip) runs the four classes as four problems: every input element is gathered and split
// into its bf16 terms once per (class, tap) use, 16 times for the 4x4 deconv, and each 128-pixel tile
// carries its own prologue / epilogue (2.7-5.7x the input bytes read, round 5 PMC).
//
// Here ONE block computes all four classes of a 4 x 32 region of the input grid (512 output pixels x
// 128 channels), 512 threads = 8 waves; each (class, 64-channel half) is one wave, as 4 grid rows x 2
// channel tiles of 32x32 accumulators (128 registers). Input channels stream
// in chunks of 8: the chunk's 6 x 34 halo region is loaded once (one b128 per thread, one chunk ahead),
// split in registers into the MFMA operand chain [m0 m1 h0 h1 | l0 l1] (winograd4.hip's layout) and
// written to a 2-slot LDS buffer ([row][channel half][col], 16-B and 8-B slots: conflict-free reads);
// every (class, tap) reads its shifted view of it. Per chunk, wave, tap and row: one b128 + one b64
// LDS read (the next one issued a row ahead), three v_mfma_f32_32x32x16_bf16 per channel tile
// (mm + hh, mh + hl, hm + lh); the weights of a (tap, chunk) step arrive two steps ahead in a rotating
// register set (ops.convT_weights_x3: [cin/8][class * 4 + tap][N][2][16 B | 8 B], zero for a class's
// missing taps, which are never read). One barrier per chunk. Epilogue: BN scale / bias, ReLU, stored
// straight from the accumulators (each store instruction = two 128-B channel runs).
#include "krrn_common.h"

namespace {

typedef __bf16 ct_bf16x8 __attribute__((ext_vector_type(8)));
typedef __bf16 ct_bf16x2 __attribute__((ext_vector_type(2)));
typedef float ct_f32x2 __attribute__((ext_vector_type(2)));
typedef unsigned ct_u32x4 __attribute__((ext_vector_type(4)));
typedef unsigned ct_u32x2 __attribute__((ext_vector_type(2)));
typedef unsigned ct_u32x6 __attribute__((ext_vector_type(6)));

constexpr int kR = 4, kCg = 32;                  // grid rows / cols per block
constexpr int kSR = kR + 2, kSC = kCg + 2;       // staged rows / cols (halo 1 on each side)
constexpr int kItems = kSR * 2 * kSC;            // (row, channel half, col) items per chunk: 408
constexpr int kMH = kItems * 16, kL = kItems * 8;  // bytes per buffer, plane MH / plane L
constexpr int kBuf = kMH + kL;
constexpr int kN = 128;
constexpr unsigned kOOB = 0xFFFF0000u;
static_assert(kItems <= 512, "one staging item per thread");

struct ConvTArgs {
  const float* in;
  int in_cs, in_co;
  int B, Hi, Wi, cin;
  long long img;      // elements per input image
  const void* U3;     // plane MH [cin/8][16][N][2][16 B], then plane L [..][8 B]
  int ntap[4];        // taps per class (class = 2 py + px)
  int tap[4][4];      // (dy + 1) * 3 + (dx + 1)
  const float* scale;
  const float* bias;
  int relu;
  float* out;
  int out_cs, out_co, Ho, Wo;
  int gyn, gxn;       // blocks per image column / row
};

__device__ __forceinline__ unsigned ct_pk(float a, float b) {
  return __builtin_bit_cast(unsigned, __builtin_convertvector(ct_f32x2{a, b}, ct_bf16x2));  // RNE
}
__device__ __forceinline__ float ct_lo(unsigned p) { return __builtin_bit_cast(float, p << 16); }
__device__ __forceinline__ float ct_hi(unsigned p) { return __builtin_bit_cast(float, p & 0xFFFF0000u); }

// x (4 channels) -> [m0 m1 h0 h1 l0 l1] (winograd4.hip split3)
__device__ __forceinline__ ct_u32x6 ct_split3(const f32x4 x) {
  const unsigned h0 = ct_pk(x[0], x[1]), h1 = ct_pk(x[2], x[3]);
  const float r0 = x[0] - ct_lo(h0), r1 = x[1] - ct_hi(h0);
  const float r2 = x[2] - ct_lo(h1), r3 = x[3] - ct_hi(h1);
  const unsigned m0 = ct_pk(r0, r1), m1 = ct_pk(r2, r3);
  const unsigned l0 = ct_pk(r0 - ct_lo(m0), r1 - ct_hi(m0)), l1 = ct_pk(r2 - ct_lo(m1), r3 - ct_hi(m1));
  return ct_u32x6{m0, m1, h0, h1, l0, l1};
}

__device__ __forceinline__ ct_bf16x8 ct_sub4(const ct_u32x6& c, int o) {
  return __builtin_bit_cast(ct_bf16x8, ct_u32x4{c[o], c[o + 1], c[o + 2], c[o + 3]});
}

__global__ __launch_bounds__(512, 1) void convt_s2_x3_kernel(const ConvTArgs a) {
  __shared__ __attribute__((aligned(16))) char smem[2 * kBuf];
  const int tid = threadIdx.x, lane = tid & 63;
  const int wave = __builtin_amdgcn_readfirstlane(tid >> 6);
  const int nblk = a.B * a.gyn * a.gxn;
  const int bid = krrn_xcd_remap(blockIdx.x, nblk);
  const int b = bid / (a.gyn * a.gxn), rem = bid - b * (a.gyn * a.gxn);
  const int a0 = (rem / a.gxn) * kR, b0 = (rem - (rem / a.gxn) * a.gxn) * kCg;
  const int nck = a.cin / 8;

  // ---- staging item of this thread: (row sr, channel half sh, col sc) of the halo region --------
  const int sr = tid / (2 * kSC), sh = (tid / kSC) & 1, sc = tid - (tid / kSC) * kSC;
  const bool sitem = tid < kItems;
  const int iy = a0 - 1 + sr, ix = b0 - 1 + sc;
  const bool sok = sitem && iy >= 0 && iy < a.Hi && ix >= 0 && ix < a.Wi;
  const __amdgpu_buffer_rsrc_t rsA = __builtin_amdgcn_make_buffer_rsrc(
      (void*)(a.in + (size_t)b * a.img + a.in_co), (short)0,
      (int)min(a.img * 4 - (long long)a.in_co * 4, 0x7FFFFFFFLL), 0x00020000);
  const unsigned soff = sok ? (unsigned)((((long long)iy * a.Wi + ix) * a.in_cs + 4 * sh) * 4) : kOOB;
  const int sslot = (sr * 2 + sh) * kSC + sc;  // [row][half][col]
  auto load_raw = [&](int ck) {
    return __builtin_bit_cast(f32x4, __builtin_amdgcn_raw_buffer_load_b128(rsA, soff, ck * 32, 0));
  };
  auto store_raw = [&](int buf, const f32x4 x) {
    if (!sitem) return;
    const ct_u32x6 c = ct_split3(x);
    char* base = smem + buf * kBuf;
    *reinterpret_cast<ct_u32x4*>(base + 16 * sslot) = ct_u32x4{c[0], c[1], c[2], c[3]};
    *reinterpret_cast<ct_u32x2*>(base + kMH + 8 * sslot) = ct_u32x2{c[4], c[5]};
  };

  // ---- this wave: class cls, channels 64 nh .. + 63 ------------------------------------------------
  // waves w and w + 4 share a SIMD: classes (0, 3) and (1, 2) pair up there, so with unequal tap counts
  // (XYZNet's 3x3: 1, 2, 2, 4) the SIMDs carry 5 / 5 / 4 / 4 tap steps per chunk instead of 3 / 3 / 6 / 6
  const int cls = wave < 4 ? wave >> 1 : 3 - ((wave >> 1) & 1), nh = wave & 1;
  const int nt = a.ntap[cls];  // wave-uniform (kernel argument)
  const int fr = lane & 31, h = lane >> 5;
  const long long nrec = (long long)nck * 16 * kN * 2;
  const char* u3 = reinterpret_cast<const char*>(a.U3);
  const __amdgpu_buffer_rsrc_t rsMH =
      __builtin_amdgcn_make_buffer_rsrc((void*)u3, (short)0, (int)min(nrec * 16, 0x7FFFFFFFLL), 0x00020000);
  const __amdgpu_buffer_rsrc_t rsL =
      __builtin_amdgcn_make_buffer_rsrc((void*)(u3 + nrec * 16), (short)0, (int)min(nrec * 8, 0x7FFFFFFFLL), 0x00020000);
  const unsigned wrec = (unsigned)(2 * (64 * nh + fr) + h);  // channel tile j adds 64 records
  // weights of step s = ck * nt + t (chunk ck, tap t): both channel tiles' chains
  struct W2 {
    ct_u32x4 mh[2];
    ct_u32x2 l[2];
  };
  auto load_w = [&](int s) {
    W2 w;
    const int ck = min(s / nt, nck - 1), t = s - (s / nt) * nt;
    const unsigned srec = (unsigned)((ck * 16 + cls * 4 + min(t, 3)) * kN * 2);  // uniform
#pragma unroll
    for (int j = 0; j < 2; ++j) {
      w.mh[j] = __builtin_bit_cast(ct_u32x4, __builtin_amdgcn_raw_buffer_load_b128(
                                                 rsMH, (wrec + 64u * j) * 16u, srec * 16u, 0));
      w.l[j] = __builtin_bit_cast(ct_u32x2, __builtin_amdgcn_raw_buffer_load_b64(
                                                rsL, (wrec + 64u * j) * 8u, srec * 8u, 0));
    }
    return w;
  };
  // the A operand of grid row r under tap code tc, for this lane's column fr and channel half h
  auto a_off = [&](int tc, int r) {
    const int dy = tc / 3 - 1, dx = tc - (tc / 3) * 3 - 1;
    return ((r + 1 + dy) * 2 + h) * kSC + fr + 1 + dx;  // slot index
  };
  auto chain = [&](int buf, int slot) {
    const char* base = smem + buf * kBuf;
    const ct_u32x4 mh = *reinterpret_cast<const ct_u32x4*>(base + 16 * slot);
    const ct_u32x2 l = *reinterpret_cast<const ct_u32x2*>(base + kMH + 8 * slot);
    return ct_u32x6{mh[0], mh[1], mh[2], mh[3], l[0], l[1]};
  };

  f32x16 acc[kR][2];
#pragma unroll
  for (int r = 0; r < kR; ++r)
#pragma unroll
    for (int j = 0; j < 2; ++j)
#pragma unroll
      for (int q = 0; q < 16; ++q) acc[r][j][q] = 0.f;

  // ---- prologue: chunk 0 staged, the first two weight steps requested ------------------------------
  store_raw(0, load_raw(0));
  W2 w0 = load_w(0), w1 = load_w(1);
  f32x4 raw = load_raw(1);  // chunk 1 (past the last chunk: a harmless repeat of it)
  __syncthreads();

  int s = 0;
  for (int ck = 0; ck < nck; ++ck) {
    const int p = ck & 1;
    for (int t = 0; t < nt; ++t, ++s) {
      const int tc = a.tap[cls][t];
      ct_u32x6 bc[2];  // this step's weight chains as single register tuples
#pragma unroll
      for (int j = 0; j < 2; ++j) {
        bc[j] = ct_u32x6{w0.mh[j][0], w0.mh[j][1], w0.mh[j][2], w0.mh[j][3], w0.l[j][0], w0.l[j][1]};
        asm volatile("" : "+v"(bc[j]));
      }
      W2 w2 = load_w(s + 2);  // two steps ahead (past the end: a harmless repeat)
      ct_u32x6 an = chain(p, a_off(tc, 0));
#pragma unroll
      for (int r = 0; r < kR; ++r) {
        ct_u32x6 ac = an;
        if (r + 1 < kR) an = chain(p, a_off(tc, r + 1));
        asm volatile("" : "+v"(ac));  // one register tuple: the MFMA operands are its sub-registers
        // the two channel tiles' term products interleaved: no MFMA waits on the one before it
#pragma unroll
        for (int j = 0; j < 2; ++j)
          acc[r][j] = __builtin_amdgcn_mfma_f32_32x32x16_bf16(ct_sub4(ac, 0), ct_sub4(bc[j], 0), acc[r][j], 0, 0, 0);
#pragma unroll
        for (int j = 0; j < 2; ++j)
          acc[r][j] = __builtin_amdgcn_mfma_f32_32x32x16_bf16(ct_sub4(ac, 0), ct_sub4(bc[j], 2), acc[r][j], 0, 0, 0);
#pragma unroll
        for (int j = 0; j < 2; ++j)
          acc[r][j] = __builtin_amdgcn_mfma_f32_32x32x16_bf16(ct_sub4(ac, 2), ct_sub4(bc[j], 0), acc[r][j], 0, 0, 0);
      }
      w0 = w1;
      w1 = w2;
    }
    // chunk ck + 1 into the other buffer (its readers finished at the previous barrier), then the
    // load of chunk ck + 2 into the staging register
    if (ck + 1 < nck) {
      store_raw(p ^ 1, raw);
      raw = load_raw(min(ck + 2, nck - 1));
    }
    __syncthreads();
  }

  // ---- epilogue: BN scale / bias, ReLU, NHWC stores ------------------------------------------------
  const int py = cls >> 1, px = cls & 1;
#pragma unroll
  for (int j = 0; j < 2; ++j) {
    const int n = 64 * nh + 32 * j + fr;
    const float scl = a.scale ? a.scale[n] : 1.f, bia = a.bias ? a.bias[n] : 0.f;
#pragma unroll
    for (int r = 0; r < kR; ++r) {
      const int ga = a0 + r, oy = 2 * ga + py;
      if (ga >= a.Hi || oy >= a.Ho) continue;
#pragma unroll
      for (int q = 0; q < 16; ++q) {
        const int gb = b0 + 8 * (q >> 2) + 4 * h + (q & 3), ox = 2 * gb + px;
        if (gb >= a.Wi || ox >= a.Wo) continue;
        float v = __builtin_fmaf(acc[r][j][q], scl, bia);
        if (a.relu) v = fmaxf(v, 0.f);
        a.out[(((size_t)b * a.Ho + oy) * a.Wo + ox) * a.out_cs + a.out_co + n] = v;
      }
    }
  }
}

}  // namespace

KRRN_API int krrn_convT_s2_x3_f32(const float* in, int in_cs, int in_co, int B, int Hi, int Wi, int cin,
                                  const int* cls_taps, const void* U3, int N, const float* scale, const float* bias,
                                  int relu, float* out, int out_cs, int out_co, int Ho, int Wo, void* stream) {
  if (!in || !cls_taps || !U3 || !out) return KRRN_EARG;
  if (B < 1 || Hi < 1 || Wi < 1 || N != kN || Ho < 1 || Wo < 1 || Ho > 2 * Hi || Wo > 2 * Wi) return KRRN_ESHAPE;
  if (cin < 8 || (cin % 8) || in_co + cin > in_cs || out_co + N > out_cs) return KRRN_ESHAPE;
  if (!krrn_aligned16(U3) || !krrn_aligned16(in) || (in_cs & 3) || (in_co & 3)) return KRRN_EALIGN;
  ConvTArgs a;
  for (int c = 0; c < 4; ++c) {
    const int n = cls_taps[5 * c];
    if (n < 1 || n > 4) return KRRN_EARG;
    a.ntap[c] = n;
    for (int t = 0; t < 4; ++t) {
      const int tc = t < n ? cls_taps[5 * c + 1 + t] : 4;
      if (tc < 0 || tc > 8) return KRRN_EARG;
      a.tap[c][t] = tc;
    }
  }
  a.in = in; a.in_cs = in_cs; a.in_co = in_co; a.B = B; a.Hi = Hi; a.Wi = Wi; a.cin = cin;
  a.img = (long long)Hi * Wi * in_cs;
  a.U3 = U3; a.scale = scale; a.bias = bias; a.relu = relu;
  a.out = out; a.out_cs = out_cs; a.out_co = out_co; a.Ho = Ho; a.Wo = Wo;
  a.gyn = krrn_cdiv(Hi, kR); a.gxn = krrn_cdiv(Wi, kCg);
  const long long nrec = (long long)(cin / 8) * 16 * N * 2;
  if (a.img * 4 >= 0x7FFF0000LL || nrec * 16 >= 0x7FFF0000LL) return KRRN_ESHAPE;
  const long long blocks = (long long)B * a.gyn * a.gxn;
  if (blocks > 0x7fffffffLL) return KRRN_ESHAPE;
  hipLaunchKernelGGL(convt_s2_x3_kernel, dim3((unsigned)blocks), dim3(512), 0, (hipStream_t)stream, a);
  return krrn_launch_status();
}
