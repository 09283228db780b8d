// Direct convolution for the narrow HRNet convs, fused with eval-BN scale / bias, the residual add
// and ReLU: the branch BasicBlocks' 3x3 / stride-1 convs (18/36/72/144 channels at S/4 .. S/32,
// lib/network/hrnet/myhrnet.py:34-63) and the fuse layers' 3x3 / stride-2
// downsamples and 1x1 projections (myhrnet.py:177-225, H4).
//
// These convs are tiny (0.05-0.7 GFLOP at B = 64) and were bound by per-k-tile load latency in the
// implicit-GEMM kernel (a wave's 2-40 k-tiles each wait for an im2col gather; 13-21 us per launch
// for ~3 us of matrix work). Here a block stages the input rows its output pixels read — all
// input channels, with a zero border for the 3x3 ones — into LDS ONCE, and then runs the whole
// K = taps x cin reduction out of LDS: one global-load phase per block instead of one per k-tile.
//
// Block = 256 threads = 4 waves = 64 consecutive output pixels in (b, y, x) raster order (any
// number of images / rows; e.g. 4 whole 4x4 images, or 2.1 rows of a 30-wide image) x NW
// 16-channel output tiles. Wave w owns pixels [16w, 16w + 16) of the block and accumulates NW
// v_mfma_f32_16x16x4_f32 tiles (16 pixels x 16 channels each): 16x16 tiles give 4x the waves of
// 32x32 tiles for the same output, which is what these small-M / small-N problems need to cover
// the CUs. Per (tap, 16-channel group): lane (pixel m = l % 16, quad g = l / 16) reads the 4
// channels 4g..4g+3 of its input pixel from LDS (one ds_read_b128 feeds 4 MFMAs: MFMA s sums
// k = 4g + s over the 4 lane groups) and the matching weight quad of output channel n = l % 16
// straight from global memory (the weights are read by every block: L2-resident). The weights are
// the MFMA's first operand, so each lane ends with 4 consecutive channels of one pixel: the
// epilogue (BN, residual, ReLU) is one float4 load / store per lane and channel tile.
//
// Numerics: f32 operands, f32 accumulation (v_mfma_f32_16x16x4_f32 is an fma chain); the k order
// differs from the implicit-GEMM kernel's, so results agree with it to f32 rounding.
#include "krrn_common.h"

namespace {

struct SmallArgs {
  const float* in;
  int in_cs, in_co;
  int B, H, W, cin;      // input image; cin = physical channels (multiple of 4)
  int ksz, stride, pad;  // 3 / 1 / 1, 3 / 2 / 1 or 1 / 1 / 0
  int Ho, Wo;            // output image
  const float* wt;       // [N][taps * cin], k = tap * cin + c, tap = ky * ksz + kx
  int N, n_store;
  const float* scale;
  const float* bias;
  const float* res;
  int res_cs, res_co;
  float* out;
  int out_cs, out_co;
  int relu;
  int M;                 // B * Ho * Wo
  int q;                 // channel quads per pixel (cin / 4)
  int pitch;             // LDS float4 per staged pixel: q rounded up to odd (conflict-free reads)
};

constexpr unsigned kOOB = 0xFFFFFFF0u;

// Block = 256 threads = 4 waves over PM = 4 / KS m-tiles (16 output pixels each, consecutive in
// (b, y, x) raster order) x NW 16-channel n-tiles; wave w computes m-tile w / KS over the K-slice
// w % KS of the flattened reduction (k = tap * cin + c in 16-wide steps: lane quad g of step st
// is k-quad 4 st + g, i.e. tap (4 st + g) / q, channels 4 ((4 st + g) % q) .. +3, so a step can
// straddle two taps and no channel padding is computed). With KS > 1 the K-slices' partial tiles
// are summed through LDS in slice order (deterministic).
template <int NW, int KS>
__device__ __forceinline__ void small_body(const SmallArgs& a, int bx, int by, float* slab) {
  constexpr int PM = 4 / KS;
  constexpr int kPixB = 16 * PM;
  const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
  const int mi = wave / KS, ks = wave - (wave / KS) * KS;
  const int p0 = bx * kPixB;
  const int n0 = by * NW * 16;
  const int HWo = a.Ho * a.Wo, W2 = a.W + 2 * a.pad;
  // staged rows: for each image bA..bB the input rows its output rows in [p0, p1] read
  const int p1 = min(p0 + kPixB, a.M) - 1;
  const int bA = p0 / HWo, bB = p1 / HWo;
  const int yA = (p0 - bA * HWo) / a.Wo, yB = (p1 - bB * HWo) / a.Wo;
  auto ystart = [&](int b) { return (b == bA ? a.stride * yA : 0) - a.pad; };
  auto yend = [&](int b) { return (b == bB ? a.stride * yB : a.stride * (a.Ho - 1)) + a.ksz - 1 - a.pad; };  // incl.
  int nrows = 0;
  for (int b = bA; b <= bB; ++b) nrows += yend(b) - ystart(b) + 1;

  // ---- stage: nrows x (W + 2 pad) pixels x cin channels, zero outside the image ---------------
  const __amdgpu_buffer_rsrc_t rsA = __builtin_amdgcn_make_buffer_rsrc(
      (void*)(a.in + a.in_co), (short)0, (int)0x7FFFFFF0, 0x00020000);
  const int Q = a.q;
  const int total = nrows * W2 * Q;
  const unsigned qmagic = Q > 1 ? (unsigned)((0x100000000ULL + Q - 1) / Q) : 0u;  // Q == 1: pix = e
  const unsigned w2magic = (unsigned)((0x100000000ULL + W2 - 1) / W2);
  // kSU independent loads in flight per thread, then their LDS writes (a rolled load -> write
  // loop would serialise one memory latency per element)
  constexpr int kSU = 8;
#if KRRN_SMALL_EXP == 2  // timing experiment: no staging loads (LDS left as is)
  if (total < 0)
#endif
  for (int e0 = 0; e0 < total; e0 += 256 * kSU) {
    f32x4 v[kSU];
    int dst[kSU];
#pragma unroll
    for (int u = 0; u < kSU; ++u) {
      const int e = e0 + tid + 256 * u;
      const int pix = Q == 1 ? e : (int)__umulhi((unsigned)e, qmagic);
      const int c4 = e - pix * Q;
      const int rs = (int)__umulhi((unsigned)pix, w2magic), xs = pix - rs * W2;
      int b = bA, r = rs;
      while (b < bB && r >= yend(b) - ystart(b) + 1) {
        r -= yend(b) - ystart(b) + 1;
        ++b;
      }
      const int yin = ystart(b) + r, xin = xs - a.pad;
      const bool ok = e < total && yin >= 0 && yin < a.H && xin >= 0 && xin < a.W;
      const unsigned off =
          ok ? (unsigned)(((((long long)b * a.H + yin) * a.W + xin) * a.in_cs + 4 * c4) * 4) : kOOB;
      v[u] = __builtin_bit_cast(f32x4, __builtin_amdgcn_raw_buffer_load_b128(rsA, off, 0, 0));
      dst[u] = e < total ? 4 * (pix * a.pitch + c4) : -1;
    }
#pragma unroll
    for (int u = 0; u < kSU; ++u) {
      if (dst[u] < 0) continue;
      *reinterpret_cast<f32x4*>(slab + dst[u]) = v[u];
    }
  }

  // ---- this lane's pixel and weight rows ------------------------------------------------------
  const int fr = lane & 15, g = lane >> 4;
  const int m = p0 + 16 * mi + fr;
  int base = 0;  // staged pixel of (b, y, x), the centre tap
  {
    const int mm = min(m, a.M - 1);
    const int b = mm / HWo, rr = mm - b * HWo;
    const int y = rr / a.Wo, x = rr - (rr / a.Wo) * a.Wo;
    int rowslot = 0;
    for (int bb = bA; bb < b; ++bb) rowslot += yend(bb) - ystart(bb) + 1;
    rowslot += a.stride * y - ystart(b);
    base = rowslot * W2 + a.stride * x + a.pad;
  }
  const int taps = a.ksz * a.ksz;
  const int tb = a.ksz == 1 ? 4 : 0;  // a 1x1 conv's one tap is the 3x3 grid's centre
  const int K = taps * a.cin;
  const int KQ = taps * Q;  // k-quads
  const __amdgpu_buffer_rsrc_t rsW = __builtin_amdgcn_make_buffer_rsrc(
      (void*)a.wt, (short)0, (int)min((long long)a.N * K * 4, (long long)kOOB), 0x00020000);
  unsigned wrow[NW];
#pragma unroll
  for (int j = 0; j < NW; ++j) {
    const int n = n0 + 16 * j + fr;
    wrow[j] = n < a.N ? (unsigned)n * (unsigned)K * 4u : kOOB;
  }
  f32x4 acc[NW];
#pragma unroll
  for (int j = 0; j < NW; ++j) acc[j] = f32x4{0.f, 0.f, 0.f, 0.f};
  __syncthreads();

  // ---- K loop over this wave's slice of the 16-wide steps --------------------------------------
  const int nsteps = (KQ + 3) / 4;
  const int per = (nsteps + KS - 1) / KS;
  const int s0 = ks * per, s1 = min(nsteps, s0 + per);
  auto wload = [&](int st, f32x4 (&w)[NW]) {
    const int kq = 4 * st + g;
    const bool ok = st < s1 && kq < KQ;
#pragma unroll
    for (int j = 0; j < NW; ++j) {
      const unsigned off = (ok && wrow[j] != kOOB) ? wrow[j] + (unsigned)kq * 16u : kOOB;
      w[j] = __builtin_bit_cast(f32x4, __builtin_amdgcn_raw_buffer_load_b128(rsW, off, 0, 0));
    }
  };
  // this lane's (tap, channel quad) at step s0, advanced by 4 quads per step
  int kq0 = 4 * s0 + g;
  int tap = kq0 / Q, c4 = kq0 - (kq0 / Q) * Q;
#ifndef KRRN_SMALL_PF
#define KRRN_SMALL_PF 2
#endif
  // weights KRRN_SMALL_PF steps ahead in a register ring (slot u of every PF-step group)
  constexpr int PF = KRRN_SMALL_PF;
  f32x4 wr[PF][NW];
#pragma unroll
  for (int u = 0; u < PF; ++u) wload(s0 + u, wr[u]);
#if KRRN_SMALL_EXP == 1  // timing experiment: no K loop (staging + epilogue only)
  if (s1 > 0x7fffffff - 1)
#endif
  for (int st0 = s0; st0 < s1; st0 += PF) {
#pragma unroll
    for (int u = 0; u < PF; ++u) {
      const int st = st0 + u;
      if (st >= s1) break;
      f32x4 w[NW];
#pragma unroll
      for (int j = 0; j < NW; ++j) w[j] = wr[u][j];
      wload(st + PF, wr[u]);
      const int t3 = tap + tb;
      const int ty = t3 >= 6 ? 1 : (t3 >= 3 ? 0 : -1);
      const int tx = t3 - 3 * (ty + 1) - 1;
      const bool kok = tap < taps;
      const int px = kok ? base + ty * W2 + tx : base;
      f32x4 av = *reinterpret_cast<const f32x4*>(slab + 4 * (px * a.pitch + c4));
      if (!kok) av = f32x4{0.f, 0.f, 0.f, 0.f};
#pragma unroll
      for (int s2 = 0; s2 < 4; ++s2)
#pragma unroll
        for (int j = 0; j < NW; ++j) {
#if KRRN_SMALL_EXP == 3  // timing experiment: no MFMAs (operands still loaded)
          acc[j][s2] += av[s2] * w[j][s2];
#else
          // weights as the first operand (rows = output channels), pixels as the second: lane l's
          // accumulator is channels 4 (l / 16) .. +3 of pixel l % 16 (one float4 in the epilogue)
          acc[j] = __builtin_amdgcn_mfma_f32_16x16x4f32(w[j][s2], av[s2], acc[j], 0, 0, 0);
#endif
        }
      c4 += 4;
      if (c4 >= Q) {  // Q >= 4: at most one wrap per step... Q in [1, 4) wraps more
        c4 -= Q;
        ++tap;
        while (c4 >= Q) {
          c4 -= Q;
          ++tap;
        }
      }
    }
  }

  // ---- K-slice reduction through LDS (slice order: deterministic) ------------------------------
  if constexpr (KS > 1) {
    __syncthreads();  // every wave is done reading the slab
    float* part = slab;
#pragma unroll
    for (int j = 0; j < NW; ++j)
      *reinterpret_cast<f32x4*>(part + ((wave * NW + j) * 64 + lane) * 4) = acc[j];
    __syncthreads();
    if (ks != 0) return;
#pragma unroll
    for (int j = 0; j < NW; ++j) {
      f32x4 v = *reinterpret_cast<const f32x4*>(part + ((wave * NW + j) * 64 + lane) * 4);
      for (int q2 = 1; q2 < KS; ++q2) v += *reinterpret_cast<const f32x4*>(part + (((wave + q2) * NW + j) * 64 + lane) * 4);
      acc[j] = v;
    }
  }

  // ---- epilogue: acc[j][i] = (channel n0 + 16j + 4g + i, pixel 16 mi + fr): float4 per lane ------
  const int mo = p0 + 16 * mi + fr;
  if (mo >= a.M) return;
#pragma unroll
  for (int j = 0; j < NW; ++j) {
    const int n = n0 + 16 * j + 4 * g;
    if (n >= a.n_store) continue;  // n_store is a multiple of 4
    const f32x4 sc = a.scale ? *reinterpret_cast<const f32x4*>(a.scale + n) : f32x4{1.f, 1.f, 1.f, 1.f};
    const f32x4 bi = a.bias ? *reinterpret_cast<const f32x4*>(a.bias + n) : f32x4{0.f, 0.f, 0.f, 0.f};
    f32x4 v = acc[j] * sc + bi;
    if (a.res) v += *reinterpret_cast<const f32x4*>(a.res + (size_t)mo * a.res_cs + a.res_co + n);
    if (a.relu) {
#pragma unroll
      for (int i = 0; i < 4; ++i) v[i] = fmaxf(v[i], 0.f);
    }
    *reinterpret_cast<f32x4*>(a.out + (size_t)mo * a.out_cs + a.out_co + n) = v;
  }
}

template <int NW, int KS>
__global__ __launch_bounds__(256) void conv_small_kernel(const SmallArgs a) {
  extern __shared__ __attribute__((aligned(16))) float slab[];
  small_body<NW, KS>(a, blockIdx.x, blockIdx.y, slab);
}

// LDS floats of the largest slab any block of this problem stages (host mirror of the kernel's
// row count: the input rows of the output rows a block's pixel range covers)
long long slab_floats(const SmallArgs& a, int pixb) {
  const long long HWo = (long long)a.Ho * a.Wo, M = (long long)a.B * HWo;
  long long worst = 0;
  for (long long p0 = 0; p0 < M; p0 += pixb) {
    const long long p1 = (p0 + pixb < M ? p0 + pixb : M) - 1;
    const long long bA = p0 / HWo, bB = p1 / HWo;
    const long long yA = (p0 - bA * HWo) / a.Wo, yB = (p1 - bB * HWo) / a.Wo;
    long long rows = 0;
    for (long long b = bA; b <= bB; ++b)
      rows += (b == bB ? a.stride * yB : a.stride * (a.Ho - 1)) + a.ksz - 1 - (b == bA ? a.stride * yA : 0) + 1;
    if (rows > worst) worst = rows;
    if (p0 >= (long long)pixb * HWo) break;  // block starts repeat modulo lcm(pixb, HWo)
  }
  return worst * (a.W + 2 * a.pad) * a.pitch * 4;
}

// dynamic LDS bytes of one (NW, KS) launch: the slab, or the K-slice partials if larger
long long small_lds(const SmallArgs& a, int nw, int ks) {
  long long lds = slab_floats(a, 64 / ks) * 4;
  const long long red = 4LL * nw * 64 * 4 * 4;
  if (ks > 1 && lds < red) lds = red;
  return lds;
}

int set_lds(const void* fn, long long lds) {
  if (lds > 160 * 1024) return KRRN_ESHAPE;
  if (lds > 64 * 1024) {
    const hipError_t e = hipFuncSetAttribute(fn, hipFuncAttributeMaxDynamicSharedMemorySize, (int)lds);
    if (e != hipSuccess) return (int)e;
  }
  return KRRN_OK;
}

template <int NW, int KS>
int small_launch(const SmallArgs& a, hipStream_t s) {
  constexpr int pixb = 64 / KS;
  const long long lds = small_lds(a, NW, KS);
  const int st = set_lds((const void*)conv_small_kernel<NW, KS>, lds);
  if (st != KRRN_OK) return st;
  const dim3 grid(krrn_cdiv(a.M, pixb), krrn_cdiv(krrn_cdiv(a.N, 16), NW));
  hipLaunchKernelGGL((conv_small_kernel<NW, KS>), grid, dim3(256), (size_t)lds, s, a);
  return krrn_launch_status();
}

int make_args(const float* in, int in_cs, int in_co, int B, int H, int W, int cin, const float* wt, int N,
              int n_store, const float* scale, const float* bias, const float* res, int res_cs, int res_co,
              float* out, int out_cs, int out_co, int relu, int ksize, int stride, int nw, int ks, SmallArgs& a) {
  if (!in || !wt || !out) return KRRN_EARG;
  if (B < 1 || H < 1 || W < 1 || N < 1 || n_store < 1 || n_store > N) return KRRN_ESHAPE;
  if (cin < 4 || (cin & 3) || (in_cs & 3) || (in_co & 3) || in_co + cin > in_cs) return KRRN_EALIGN;
  if (!krrn_aligned16(in) || !krrn_aligned16(wt)) return KRRN_EALIGN;
  if (out_co + n_store > out_cs || (res && res_co + n_store > res_cs)) return KRRN_ESHAPE;
  // the epilogue stores / loads float4 channel quads
  if ((n_store & 3) || (out_cs & 3) || (out_co & 3) || !krrn_aligned16(out)) return KRRN_EALIGN;
  if (res && ((res_cs & 3) || (res_co & 3) || !krrn_aligned16(res))) return KRRN_EALIGN;
  if ((scale && !krrn_aligned16(scale)) || (bias && !krrn_aligned16(bias))) return KRRN_EALIGN;
  if (nw < 1 || nw > 3 || (ks != 1 && ks != 2 && ks != 4)) return KRRN_EARG;
  if ((ksize != 1 && ksize != 3) || (stride != 1 && stride != 2)) return KRRN_EARG;
  const int pad = (ksize - 1) / 2;
  const int Ho = (H + 2 * pad - ksize) / stride + 1, Wo = (W + 2 * pad - ksize) / stride + 1;
  if (Ho < 1 || Wo < 1) return KRRN_ESHAPE;
  const long long M = (long long)B * Ho * Wo;
  if (M > 0x7fffffffLL || (long long)B * H * W * in_cs * 4 >= 0x7FFFFFF0LL ||
      (long long)N * ksize * ksize * cin * 4 >= (long long)kOOB)
    return KRRN_ESHAPE;
  a.ksz = ksize; a.stride = stride; a.pad = pad; a.Ho = Ho; a.Wo = Wo;
  a.in = in; a.in_cs = in_cs; a.in_co = in_co; a.B = B; a.H = H; a.W = W; a.cin = cin;
  a.wt = wt; a.N = N; a.n_store = n_store; a.scale = scale; a.bias = bias;
  a.res = res; a.res_cs = res_cs; a.res_co = res_co; a.out = out; a.out_cs = out_cs; a.out_co = out_co;
  a.relu = relu; a.M = (int)M;
  a.q = cin / 4;
  a.pitch = a.q | 1;
  return KRRN_OK;
}

}  // namespace

KRRN_API int krrn_conv_small_f32(const float* in, int in_cs, int in_co, int B, int H, int W, int cin, const float* wt,
                                 int N, int n_store, const float* scale, const float* bias, const float* res,
                                 int res_cs, int res_co, float* out, int out_cs, int out_co, int relu, int ksize,
                                 int stride, int nw, int ks, void* stream) {
  SmallArgs a;
  const int st = make_args(in, in_cs, in_co, B, H, W, cin, wt, N, n_store, scale, bias, res, res_cs, res_co, out,
                           out_cs, out_co, relu, ksize, stride, nw, ks, a);
  if (st != KRRN_OK) return st;
  hipStream_t s = (hipStream_t)stream;
#define KRRN_SMALL(NWV, KSV) \
  if (nw == NWV && ks == KSV) return small_launch<NWV, KSV>(a, s);
  KRRN_SMALL(1, 1) KRRN_SMALL(2, 1) KRRN_SMALL(3, 1)
  KRRN_SMALL(1, 2) KRRN_SMALL(2, 2) KRRN_SMALL(3, 2)
  KRRN_SMALL(1, 4) KRRN_SMALL(2, 4) KRRN_SMALL(3, 4)
#undef KRRN_SMALL
  return KRRN_EARG;
}

