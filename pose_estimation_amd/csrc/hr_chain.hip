// HRNet branch chain: ALL the BasicBlocks of one HRNet branch of one module in ONE launch
// (lib/network/hrnet/myhrnet.py:34-63 BasicBlock, :226-231 `x[i] = self.branches[i](x[i])`,
// SURVEY §8a H3). Each BasicBlock is conv3x3+BN+ReLU then conv3x3+BN + residual + ReLU, stride 1,
// channels unchanged; four blocks per branch and module.
//
// The branch convs are tiny (0.3-0.4 GFLOP at B = 64) and run as 8 dependent launches per module and
// branch on conv_small_kernel (conv_small.hip), each 13-25 us in the step, about half of it fixed
// cost: the launch, the staging of the input rows from HBM / L2 and the epilogue's round trip.
// Here one workgroup owns ONE image of the branch for the whole chain: the image's activation map
// and the block's intermediate map both stay in LDS ([pixel][channel], f32) from the branch input
// to the branch output, so a module's 8 convs cost one HBM read of the input, one write of the
// output and 8 LDS-resident convolutions separated by workgroup barriers.
//
// Per conv: K = 9 taps x cp channels, flattened k = tap * cp + c (ops.make_conv's packing) in 16-
// channel steps (4 channel quads; a step may straddle two taps). The matrix math is split-bf16 at
// f32 accuracy (the three-term split of winograd.hip / gemm_panel.hip: six bf16 term products per
// f32 product on v_mfma_f32_16x16x32_bf16, f32 accumulation): weights are the MFMA's first operand
// (rows = 16 output channels, host-split chain [m h l] per lane, chain_weights_x3), the LDS
// activations its second (columns = 16 pixels; lane (r, g) reads channel quad g of its pixel's tap
// and splits it into the [h h m l] register chain), so a lane's accumulator is 4 consecutive output
// channels of one pixel: the epilogue (BN scale / bias, residual, ReLU) is one float4 LDS read / write
// per lane and tile. Out-of-image taps read a zero quad. Work split: waves take m-tiles (16 pixels)
// round robin with every n-tile (MSPLIT), or, for maps of <= 3 m-tiles, every m-tile with n-tiles
// round robin; the weights of a step are loaded once per wave (L2) and used for all its m-tiles.
#include "krrn_common.h"

namespace {

typedef __bf16 hc_bf16x8 __attribute__((ext_vector_type(8)));
typedef __bf16 hc_bf16x2 __attribute__((ext_vector_type(2)));
typedef float hc_f32x2 __attribute__((ext_vector_type(2)));
typedef unsigned hc_u32x2 __attribute__((ext_vector_type(2)));
typedef unsigned hc_u32x4 __attribute__((ext_vector_type(4)));
typedef unsigned hc_u32x8 __attribute__((ext_vector_type(8)));

constexpr int kChainMaxConv = 8;

struct ChainArgs {
  const float* in;
  int in_cs, in_co;
  float* out;
  int out_cs, out_co;
  int H, W, cp;    // map height / width, physical channels (multiple of 4)
  int Q, KQ;       // channel quads per pixel, k-quads per conv (9 Q)
  int pitch;       // LDS floats per pixel: 4 x (Q rounded up to odd), conflict-free 16-pixel reads
  int nconv;       // 2 x BasicBlocks
  int MT, NT, S;   // 16-pixel m-tiles, 16-channel n-tiles, 16-channel k-steps per conv
  const unsigned* wt[kChainMaxConv];  // chain_weights_x3: [NT][S][64][4] u32 then [NT][S][64][2] u32
  const float* scale[kChainMaxConv];  // folded eval BN, cp floats each
  const float* bias[kChainMaxConv];
};

__device__ __forceinline__ unsigned hc_pk(float a, float b) {
  return __builtin_bit_cast(unsigned, __builtin_convertvector(hc_f32x2{a, b}, hc_bf16x2));  // RNE
}

// x (4 channels) -> the [x_h x_h x_m x_l] register chain (winograd.hip split3_chain)
__device__ __forceinline__ hc_u32x8 hc_split(const f32x4 x) {
  const unsigned h0 = hc_pk(x[0], x[1]), h1 = hc_pk(x[2], x[3]);
  const float r0 = x[0] - __builtin_bit_cast(float, h0 << 16), r1 = x[1] - __builtin_bit_cast(float, h0 & 0xFFFF0000u);
  const float r2 = x[2] - __builtin_bit_cast(float, h1 << 16), r3 = x[3] - __builtin_bit_cast(float, h1 & 0xFFFF0000u);
  const unsigned m0 = hc_pk(r0, r1), m1 = hc_pk(r2, r3);
  const unsigned l0 = hc_pk(r0 - __builtin_bit_cast(float, m0 << 16), r1 - __builtin_bit_cast(float, m0 & 0xFFFF0000u));
  const unsigned l1 = hc_pk(r2 - __builtin_bit_cast(float, m1 << 16), r3 - __builtin_bit_cast(float, m1 & 0xFFFF0000u));
  return hc_u32x8{h0, h1, h0, h1, m0, m1, l0, l1};
}

__device__ __forceinline__ hc_bf16x8 hc_sub4(const hc_u32x8& c, int o) {
  return __builtin_bit_cast(hc_bf16x8, hc_u32x4{c[o], c[o + 1], c[o + 2], c[o + 3]});
}

template <int MTW, int NTW, bool MSPLIT>
__global__ __launch_bounds__(256) void hr_chain_kernel(const ChainArgs a) {
  extern __shared__ __attribute__((aligned(16))) float lds[];
  const int HW = a.H * a.W;
  float* const xm = lds;                    // the branch activation [HW][pitch]
  float* const hm = lds + HW * a.pitch;     // a BasicBlock's intermediate [HW][pitch]
  float* const zq = hm + HW * a.pitch;      // one zero quad: every out-of-image tap reads it
  const int tid = threadIdx.x, lane = tid & 63;
  const int wave = __builtin_amdgcn_readfirstlane(tid >> 6);
  const int b = blockIdx.x;

  // ---- the image in: global NHWC (channel slice) -> LDS ----------------------------------------
  {
    const float* src = a.in + (size_t)b * HW * a.in_cs + a.in_co;
    for (int e = tid; e < HW * a.Q; e += 256) {
      const int p = e / a.Q, q = e - (e / a.Q) * a.Q;
      *reinterpret_cast<f32x4*>(xm + p * a.pitch + 4 * q) =
          *reinterpret_cast<const f32x4*>(src + (size_t)p * a.in_cs + 4 * q);
    }
    if (tid < 4) zq[tid] = 0.f;
  }
  __syncthreads();

  // ---- this lane's pixels and tiles ------------------------------------------------------------
  const int r = lane & 15, g = lane >> 4;
  int py[MTW], px[MTW], pb[MTW];  // pixel row / column, LDS offset (pb < 0: past the map)
#pragma unroll
  for (int i = 0; i < MTW; ++i) {
    const int mt = MSPLIT ? wave + 4 * i : i;
    const int p = 16 * mt + r;
    const bool ok = mt < a.MT && p < HW;
    py[i] = ok ? p / a.W : -4;
    px[i] = ok ? p - (p / a.W) * a.W : -4;
    pb[i] = ok ? p * a.pitch : -1;
  }
  int ntl[NTW];
#pragma unroll
  for (int j = 0; j < NTW; ++j) {
    const int nt = MSPLIT ? j : wave + 4 * j;
    ntl[j] = nt < a.NT ? nt : -1;
  }

  for (int c = 0; c < a.nconv; ++c) {
    const float* sm = (c & 1) ? hm : xm;
    float* dm = (c & 1) ? xm : hm;
    const unsigned* wc = a.wt[c];
    const hc_u32x4* wmh = reinterpret_cast<const hc_u32x4*>(wc);
    const hc_u32x2* wl = reinterpret_cast<const hc_u32x2*>(wc + (size_t)a.NT * a.S * 64 * 4);
    f32x4 acc[MTW][NTW];
#pragma unroll
    for (int i = 0; i < MTW; ++i)
#pragma unroll
      for (int j = 0; j < NTW; ++j) acc[i][j] = f32x4{0.f, 0.f, 0.f, 0.f};
    hc_u32x4 cmh[NTW];
    hc_u32x2 cl[NTW];
    auto wload = [&](int s, hc_u32x4 (&mh)[NTW], hc_u32x2 (&l)[NTW]) {
      const int sc = s < a.S ? s : a.S - 1;
#pragma unroll
      for (int j = 0; j < NTW; ++j) {
        const int t = ntl[j] < 0 ? 0 : ntl[j];
        const size_t rec = ((size_t)t * a.S + sc) * 64 + lane;
        mh[j] = wmh[rec];
        l[j] = wl[rec];
      }
    };
    wload(0, cmh, cl);
    for (int s = 0; s < a.S; ++s) {
      hc_u32x4 nmh[NTW];
      hc_u32x2 nl[NTW];
      wload(s + 1, nmh, nl);  // one step ahead (the last one reloads step S - 1, unused)
      // this lane's k-quad of the step: tap (ky, kx) and channel quad
      const int kq = 4 * s + g;
      const bool kok = kq < a.KQ;
      const int tap = kok ? kq / a.Q : 4;
      const int c4 = kok ? kq - tap * a.Q : 0;
      const int ty = tap / 3 - 1, tx = tap - 3 * (tap / 3) - 1;
      const int delta = (ty * a.W + tx) * a.pitch + 4 * c4;
#pragma unroll
      for (int i = 0; i < MTW; ++i) {
        const int yy = py[i] + ty, xx = px[i] + tx;
        const bool ok = kok && pb[i] >= 0 && (unsigned)yy < (unsigned)a.H && (unsigned)xx < (unsigned)a.W;
        const f32x4 v = *reinterpret_cast<const f32x4*>(ok ? sm + pb[i] + delta : zq);
        const hc_u32x8 ac = hc_split(v);
#pragma unroll
        for (int j = 0; j < NTW; ++j) {
          if (ntl[j] < 0) continue;
          const hc_u32x8 w8 = {cmh[j][0], cmh[j][1], cmh[j][2], cmh[j][3], cl[j][0], cl[j][1], 0u, 0u};
          // W[h l] x X[h h] = hh + lh, W[m h] x X[h m] = mh + hm, W[m h] x X[m l] = mm + hl
          acc[i][j] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(hc_sub4(w8, 2), hc_sub4(ac, 0), acc[i][j], 0, 0, 0);
          acc[i][j] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(hc_sub4(w8, 0), hc_sub4(ac, 2), acc[i][j], 0, 0, 0);
          acc[i][j] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(hc_sub4(w8, 0), hc_sub4(ac, 4), acc[i][j], 0, 0, 0);
        }
      }
#pragma unroll
      for (int j = 0; j < NTW; ++j) {
        cmh[j] = nmh[j];
        cl[j] = nl[j];
      }
    }
    // ---- epilogue: lane (r, g) holds channels 16 nt + 4 g .. + 3 of pixel 16 mt + r ------------
    const float* scl = a.scale[c];
    const float* bia = a.bias[c];
#pragma unroll
    for (int i = 0; i < MTW; ++i) {
      if (pb[i] < 0) continue;
#pragma unroll
      for (int j = 0; j < NTW; ++j) {
        if (ntl[j] < 0) continue;
        const int n = 16 * ntl[j] + 4 * g;
        if (n >= a.cp) continue;
        f32x4 v = acc[i][j] * *reinterpret_cast<const f32x4*>(scl + n) + *reinterpret_cast<const f32x4*>(bia + n);
        if (c & 1) v += *reinterpret_cast<const f32x4*>(xm + pb[i] + n);  // BasicBlock residual
#pragma unroll
        for (int e = 0; e < 4; ++e) v[e] = fmaxf(v[e], 0.f);
        *reinterpret_cast<f32x4*>(dm + pb[i] + n) = v;
      }
    }
    __syncthreads();  // conv c's map complete before conv c + 1 reads it / overwrites its source
  }

  // ---- the image out: LDS -> global NHWC (channel slice) ---------------------------------------
  {
    const float* res = (a.nconv & 1) ? hm : xm;
    float* dst = a.out + (size_t)b * HW * a.out_cs + a.out_co;
    for (int e = tid; e < HW * a.Q; e += 256) {
      const int p = e / a.Q, q = e - (e / a.Q) * a.Q;
      *reinterpret_cast<f32x4*>(dst + (size_t)p * a.out_cs + 4 * q) =
          *reinterpret_cast<const f32x4*>(res + p * a.pitch + 4 * q);
    }
  }
}

// (MTW, NTW) menu: MSPLIT forms for maps of >= 4 m-tiles, the !MSPLIT form for smaller ones
struct ChainCfg {
  int mtw, ntw;
  bool msplit;
};
constexpr ChainCfg kChainCfgs[] = {{16, 2, true}, {8, 3, true}, {4, 5, true}, {2, 5, true}, {1, 8, true}, {3, 4, false}};

int chain_pick(int MT, int NT) {
  int best = -1, area = 1 << 30;
  for (int i = 0; i < (int)(sizeof(kChainCfgs) / sizeof(kChainCfgs[0])); ++i) {
    const ChainCfg& k = kChainCfgs[i];
    const bool fits = k.msplit ? (MT >= 4 && krrn_cdiv(MT, 4) <= k.mtw && NT <= k.ntw)
                               : (MT <= k.mtw && krrn_cdiv(NT, 4) <= k.ntw);
    if (fits && k.mtw * k.ntw < area) {
      best = i;
      area = k.mtw * k.ntw;
    }
  }
  return best;
}

long long chain_lds_bytes(int H, int W, int cp) {
  const int pitch = 4 * ((cp / 4) | 1);
  return (2LL * H * W * pitch + 4) * 4;
}

}  // namespace

KRRN_API int krrn_hr_chain_query(int H, int W, int cp) {
  if (H < 1 || W < 1 || cp < 4 || (cp & 3)) return KRRN_ESHAPE;
  if (chain_lds_bytes(H, W, cp) > 160 * 1024) return KRRN_ESHAPE;
  const int MT = krrn_cdiv(H * W, 16), NT = krrn_cdiv(cp, 16);
  return chain_pick(MT, NT) < 0 ? KRRN_EUNSUPPORTED : KRRN_OK;
}

KRRN_API int krrn_hr_chain_f32(const float* in, int in_cs, int in_co, float* out, int out_cs, int out_co, int B, int H,
                               int W, int cp, int nconv, const void* const* wt, const float* const* scale,
                               const float* const* bias, void* stream) {
  if (!in || !out || !wt || !scale || !bias) return KRRN_EARG;
  if (nconv < 2 || nconv > kChainMaxConv || (nconv & 1)) return KRRN_EARG;
  if (B < 1) return KRRN_ESHAPE;
  const int st = krrn_hr_chain_query(H, W, cp);
  if (st != KRRN_OK) return st;
  if ((in_cs & 3) || (in_co & 3) || (out_cs & 3) || (out_co & 3) || in_co + cp > in_cs || out_co + cp > out_cs)
    return KRRN_EALIGN;
  if (!krrn_aligned16(in) || !krrn_aligned16(out)) return KRRN_EALIGN;
  ChainArgs a;
  a.in = in; a.in_cs = in_cs; a.in_co = in_co; a.out = out; a.out_cs = out_cs; a.out_co = out_co;
  a.H = H; a.W = W; a.cp = cp; a.Q = cp / 4; a.KQ = 9 * a.Q; a.pitch = 4 * (a.Q | 1);
  a.nconv = nconv;
  a.MT = krrn_cdiv(H * W, 16); a.NT = krrn_cdiv(cp, 16); a.S = krrn_cdiv(a.KQ, 4);
  for (int c = 0; c < kChainMaxConv; ++c) {
    a.wt[c] = nullptr; a.scale[c] = nullptr; a.bias[c] = nullptr;
  }
  for (int c = 0; c < nconv; ++c) {
    if (!wt[c] || !scale[c] || !bias[c]) return KRRN_EARG;
    if (!krrn_aligned16(wt[c]) || !krrn_aligned16(scale[c]) || !krrn_aligned16(bias[c])) return KRRN_EALIGN;
    a.wt[c] = reinterpret_cast<const unsigned*>(wt[c]);
    a.scale[c] = scale[c];
    a.bias[c] = bias[c];
  }
  const long long lds = chain_lds_bytes(H, W, cp);
  const int cfg = chain_pick(a.MT, a.NT);
  hipStream_t s = (hipStream_t)stream;
#define KRRN_CHAIN(MTW, NTW, MS)                                                                         \
  {                                                                                                      \
    const void* fn = (const void*)hr_chain_kernel<MTW, NTW, MS>;                                         \
    if (lds > 64 * 1024) {                                                                               \
      const hipError_t e = hipFuncSetAttribute(fn, hipFuncAttributeMaxDynamicSharedMemorySize, (int)lds); \
      if (e != hipSuccess) return (int)e;                                                                \
    }                                                                                                    \
    hipLaunchKernelGGL((hr_chain_kernel<MTW, NTW, MS>), dim3(B), dim3(256), (size_t)lds, s, a);          \
    return krrn_launch_status();                                                                         \
  }
  switch (cfg) {
    case 0: KRRN_CHAIN(16, 2, true)
    case 1: KRRN_CHAIN(8, 3, true)
    case 2: KRRN_CHAIN(4, 5, true)
    case 3: KRRN_CHAIN(2, 5, true)
    case 4: KRRN_CHAIN(1, 8, true)
    case 5: KRRN_CHAIN(3, 4, false)
    default: return KRRN_EUNSUPPORTED;
  }
#undef KRRN_CHAIN
}
