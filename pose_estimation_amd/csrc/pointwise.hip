// Memory-bound glue of the KRRN forward: bilinear resampling (HRNet fuse / final concat,
// myhrnet.py:242-245, 511-516; UpsamplingBilinear2d in the heads, krrn.py:56, 78), layout
// changes at the API boundary, class selection + normal normalisation (krrn.py:100-108),
// the `choose` gather (krrn.py:121-122), row gathers (Pool_layer sampling, the final
// concat of fusion.py:234-238, the one-hot column of krrn.py:132-138) and the TBase tail
// (posenet.py:76-80 + krrn.py:153).
#include <math.h>

#include "krrn_common.h"

namespace {

// IT = the flat-index type: 32-bit whenever the launch fits (64-bit division is emulated and
// dominated these memory-bound kernels)
template <typename IT>
__global__ void resize_bilinear_kernel(const float* __restrict__ in, int Hi, int Wi, int in_cs, int in_co, int C4,
                                       float* __restrict__ out, int Ho, int Wo, int out_cs, int out_co,
                                       const float* __restrict__ add, int add_cs, int add_co, float sh, float sw,
                                       int align, int relu, IT total) {
  const IT e = (IT)blockIdx.x * blockDim.x + threadIdx.x;
  if (e >= total) return;
  const int c4 = (int)(e % C4);
  IT p = e / C4;
  const int ox = (int)(p % Wo);
  p /= Wo;
  const int oy = (int)(p % Ho);
  const int b = (int)(p / Ho);
  int y0, y1, x0, x1;
  float ly0, ly1, lx0, lx1;
  krrn_src_index(oy, Hi, sh, align, y0, y1, ly0, ly1);
  krrn_src_index(ox, Wi, sw, align, x0, x1, lx0, lx1);
  const float* ib = in + (long long)b * Hi * Wi * in_cs + in_co + 4 * c4;
  const f32x4 v00 = *reinterpret_cast<const f32x4*>(ib + ((long long)y0 * Wi + x0) * in_cs);
  const f32x4 v01 = *reinterpret_cast<const f32x4*>(ib + ((long long)y0 * Wi + x1) * in_cs);
  const f32x4 v10 = *reinterpret_cast<const f32x4*>(ib + ((long long)y1 * Wi + x0) * in_cs);
  const f32x4 v11 = *reinterpret_cast<const f32x4*>(ib + ((long long)y1 * Wi + x1) * in_cs);
  f32x4 r = krrn_bilerp4(v00, v01, v10, v11, ly0, ly1, lx0, lx1);
  const long long opix = ((long long)b * Ho + oy) * Wo + ox;
  if (add) r = *reinterpret_cast<const f32x4*>(add + opix * add_cs + add_co + 4 * c4) + r;
  if (relu) {
    r.x = fmaxf(r.x, 0.f); r.y = fmaxf(r.y, 0.f); r.z = fmaxf(r.z, 0.f); r.w = fmaxf(r.w, 0.f);
  }
  *reinterpret_cast<f32x4*>(out + opix * out_cs + out_co + 4 * c4) = r;
}

// Upsampling (Ho >= Hi, Wo >= Wi: adjacent outputs' source windows move by at most one pixel) as
// 2x2 output pixels x one channel quad per thread: the four outputs read a 3x3 source patch (9
// float4 loads instead of 16), each output combines its 2x2 of it with the same expression as
// resize_bilinear_kernel (bit-identical results).
__device__ __forceinline__ f32x4 pick3(const f32x4 (&r)[3], int i) { return i == 0 ? r[0] : (i == 1 ? r[1] : r[2]); }

__global__ void resize_up2x2_kernel(const float* __restrict__ in, int Hi, int Wi, int in_cs, int in_co, int C4,
                                    float* __restrict__ out, int Ho, int Wo, int out_cs, int out_co,
                                    const float* __restrict__ add, int add_cs, int add_co, float sh, float sw,
                                    int align, int relu, int Ho2, int Wo2, int total) {
  const int e = blockIdx.x * blockDim.x + threadIdx.x;
  if (e >= total) return;
  const int c4 = e % C4;
  int p = e / C4;
  const int ox2 = p % Wo2;
  p /= Wo2;
  const int oy2 = p % Ho2;
  const int b = p / Ho2;
  int y0[2], y1[2], x0[2], x1[2];
  float ly0[2], ly1[2], lx0[2], lx1[2];
#pragma unroll
  for (int d = 0; d < 2; ++d) {
    krrn_src_index(min(2 * oy2 + d, Ho - 1), Hi, sh, align, y0[d], y1[d], ly0[d], ly1[d]);
    krrn_src_index(min(2 * ox2 + d, Wo - 1), Wi, sw, align, x0[d], x1[d], lx0[d], lx1[d]);
  }
  const float* ib = in + (long long)b * Hi * Wi * in_cs + in_co + 4 * c4;
  f32x4 P[3][3];
#pragma unroll
  for (int r = 0; r < 3; ++r)
#pragma unroll
    for (int c = 0; c < 3; ++c) {
      const int yy = min(y0[0] + r, Hi - 1), xx = min(x0[0] + c, Wi - 1);
      P[r][c] = *reinterpret_cast<const f32x4*>(ib + ((long long)yy * Wi + xx) * in_cs);
    }
#pragma unroll
  for (int dy = 0; dy < 2; ++dy) {
    const int oy = 2 * oy2 + dy;
    if (oy >= Ho) break;
    const int ra = y0[dy] - y0[0], rb = y1[dy] - y0[0];
    f32x4 row0[3], row1[3];
#pragma unroll
    for (int c = 0; c < 3; ++c) {
      row0[c] = ra == 0 ? P[0][c] : P[1][c];
      row1[c] = rb == 0 ? P[0][c] : (rb == 1 ? P[1][c] : P[2][c]);
    }
#pragma unroll
    for (int dx = 0; dx < 2; ++dx) {
      const int ox = 2 * ox2 + dx;
      if (ox >= Wo) break;
      const int ca = x0[dx] - x0[0], cb = x1[dx] - x0[0];
      const f32x4 v00 = pick3(row0, ca), v01 = pick3(row0, cb), v10 = pick3(row1, ca), v11 = pick3(row1, cb);
      f32x4 r = krrn_bilerp4(v00, v01, v10, v11, ly0[dy], ly1[dy], lx0[dx], lx1[dx]);
      const long long opix = ((long long)b * Ho + oy) * Wo + ox;
      if (add) r = *reinterpret_cast<const f32x4*>(add + opix * add_cs + add_co + 4 * c4) + r;
      if (relu) {
        r.x = fmaxf(r.x, 0.f); r.y = fmaxf(r.y, 0.f); r.z = fmaxf(r.z, 0.f); r.w = fmaxf(r.w, 0.f);
      }
      *reinterpret_cast<f32x4*>(out + opix * out_cs + out_co + 4 * c4) = r;
    }
  }
}

template <typename IT>
__global__ void add_relu_kernel(const float* __restrict__ a, int a_cs, int a_co, const float* __restrict__ b,
                                int b_cs, int b_co, float* __restrict__ out, int o_cs, int o_co, int C4, int relu,
                                IT total) {
  const IT e = (IT)blockIdx.x * blockDim.x + threadIdx.x;
  if (e >= total) return;
  const int c4 = (int)(e % C4);
  const long long pix = e / C4;
  f32x4 r = *reinterpret_cast<const f32x4*>(a + pix * a_cs + a_co + 4 * c4);
  if (b) r = r + *reinterpret_cast<const f32x4*>(b + pix * b_cs + b_co + 4 * c4);
  if (relu) {
    r.x = fmaxf(r.x, 0.f); r.y = fmaxf(r.y, 0.f); r.z = fmaxf(r.z, 0.f); r.w = fmaxf(r.w, 0.f);
  }
  *reinterpret_cast<f32x4*>(out + pix * o_cs + o_co + 4 * c4) = r;
}

__global__ void nchw_to_nhwc_kernel(const float* __restrict__ in, int C, int HW, float* __restrict__ out, int o_cs,
                                    int o_co, long long total) {
  const long long e = (long long)blockIdx.x * blockDim.x + threadIdx.x;
  if (e >= total) return;
  const int p = (int)(e % HW);
  const long long bc = e / HW;
  const int c = (int)(bc % C);
  const long long b = bc / C;
  out[(b * HW + p) * o_cs + o_co + c] = in[e];
}

__global__ void heads_select_kernel(const float* __restrict__ fx, int Cx, int xyz_off, const float* __restrict__ fn,
                                    int Cn, const long long* __restrict__ cls, float* __restrict__ xyz,
                                    float* __restrict__ nml, int HW, long long total) {
  const long long e = (long long)blockIdx.x * blockDim.x + threadIdx.x;
  if (e >= total) return;
  const int p = (int)(e % HW);
  const long long b = e / HW;
  const int c = (int)cls[b];
  const float* sx = fx + (b * Cx + xyz_off + 3 * c) * HW + p;
  const float* sn = fn + (b * Cn + 3 * c) * HW + p;
  float* dx = xyz + b * 3 * HW + p;
  float* dn = nml + b * 3 * HW + p;
  dx[0] = sx[0];
  dx[HW] = sx[HW];
  dx[2 * HW] = sx[2 * HW];
  const float n0 = sn[0], n1 = sn[HW], n2 = sn[2 * HW];
  // F.normalize(p=2, dim=1, eps=1e-12): x / max(||x||_2, eps)
  const float nr = fmaxf(sqrtf(n0 * n0 + n1 * n1 + n2 * n2), 1e-12f);
  dn[0] = n0 / nr;
  dn[HW] = n1 / nr;
  dn[2 * HW] = n2 / nr;
}

__global__ void points_gather_kernel(const float* __restrict__ cloud, const float* __restrict__ xyz,
                                     const float* __restrict__ nml, const long long* __restrict__ choose, int N,
                                     int HW, float* __restrict__ p9, long long total) {
  const long long e = (long long)blockIdx.x * blockDim.x + threadIdx.x;
  if (e >= total) return;
  const long long b = e / N;
  const long long pix = choose[e];
  float* o = p9 + e * 9;
  const float* cl = cloud + e * 3;
  o[0] = cl[0];
  o[1] = cl[1];
  o[2] = cl[2];
  const float* x = xyz + b * 3 * HW + pix;
  const float* n = nml + b * 3 * HW + pix;
  o[3] = x[0];
  o[4] = x[HW];
  o[5] = x[2 * HW];
  o[6] = n[0];
  o[7] = n[HW];
  o[8] = n[2 * HW];
}

template <bool IDX64, bool VEC>
__global__ void gather_rows_kernel(const void* __restrict__ idx, long long idx_bs, int nrows,
                                   const float* __restrict__ src, long long src_bs, int src_st,
                                   float* __restrict__ dst, long long dst_bs, int dst_st, int width,
                                   long long total) {
  const long long e = (long long)blockIdx.x * blockDim.x + threadIdx.x;
  if (e >= total) return;
  const int wq = VEC ? width / 4 : width;
  const int w = (int)(e % wq);
  const long long br = e / wq;
  const int r = (int)(br % nrows);
  const long long b = br / nrows;
  const long long ii = b * idx_bs + r;
  const long long row = IDX64 ? ((const long long*)idx)[ii] : (long long)((const int*)idx)[ii];
  const float* s = src + b * src_bs + row * src_st;
  float* d = dst + b * dst_bs + (long long)r * dst_st;
  if constexpr (VEC) {
    *reinterpret_cast<f32x4*>(d + 4 * w) = *reinterpret_cast<const f32x4*>(s + 4 * w);
  } else {
    d[w] = s[w];
  }
}

// pred_t[b] = mean_i( cloud[b, i] + W4[0:3] . h[b, i] + b4[0:3] )   (one block per crop)
// TBase conv4 (C -> 3, +bias) and pred_t = mean_N(cloud + t_res) (posenet.py:80, krrn.py:150-153).
// One block of 16 waves per crop (the B = 64 blocks cannot fill the chip, so each brings 256 points
// into flight per pass: 77 -> 36 us per launch measured in the step); 4 lanes per point, each lane a float4 stripe of the
// C-channel row (a wave reads 16 rows x 64 contiguous bytes per load), 2 shuffles finish the dot
// product. The mean is a fixed-order reduction (per-lane partials, then a fixed tree), so runs are
// bit-reproducible.
constexpr int kTailWaves = 16;
__global__ __launch_bounds__(64 * kTailWaves) void tbase_tail_kernel(const float* __restrict__ h, int n, int C,
                                                         const float* __restrict__ w4,
                                                         const float* __restrict__ b4,
                                                         const float* __restrict__ cloud,
                                                         float* __restrict__ pred_t, float* __restrict__ t_res) {
  __shared__ float red[kTailWaves][3];
  const int b = blockIdx.x;
  const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
  const int q = lane & 3, pl = lane >> 2;
  const int C4 = C >> 2;
  const float bx = b4[0], by = b4[1], bz = b4[2];
  float sx = 0.f, sy = 0.f, sz = 0.f;
  for (int i0 = 0; i0 < n; i0 += 16 * kTailWaves) {
    const int i = i0 + wave * 16 + pl;
    if (i < n) {
      const f32x4* hr = reinterpret_cast<const f32x4*>(h + ((long long)b * n + i) * C);
      float a0 = 0.f, a1 = 0.f, a2 = 0.f;
      for (int c4 = q; c4 < C4; c4 += 4) {
        const f32x4 x = hr[c4];
        const f32x4 w0 = reinterpret_cast<const f32x4*>(w4)[c4];
        const f32x4 w1 = reinterpret_cast<const f32x4*>(w4 + C)[c4];
        const f32x4 w2 = reinterpret_cast<const f32x4*>(w4 + 2 * C)[c4];
        a0 += w0[0] * x[0] + w0[1] * x[1] + w0[2] * x[2] + w0[3] * x[3];
        a1 += w1[0] * x[0] + w1[1] * x[1] + w1[2] * x[2] + w1[3] * x[3];
        a2 += w2[0] * x[0] + w2[1] * x[1] + w2[2] * x[2] + w2[3] * x[3];
      }
      a0 += __shfl_xor(a0, 1);
      a1 += __shfl_xor(a1, 1);
      a2 += __shfl_xor(a2, 1);
      a0 += __shfl_xor(a0, 2);
      a1 += __shfl_xor(a1, 2);
      a2 += __shfl_xor(a2, 2);
      if (q == 0) {
        const float t0 = a0 + bx, t1 = a1 + by, t2 = a2 + bz;
        if (t_res) {
          float* tr = t_res + ((long long)b * n + i) * 3;
          tr[0] = t0; tr[1] = t1; tr[2] = t2;
        }
        const float* cp = cloud + ((long long)b * n + i) * 3;
        sx += cp[0] + t0;
        sy += cp[1] + t1;
        sz += cp[2] + t2;
      }
    }
  }
#pragma unroll
  for (int off = 4; off < 64; off <<= 1) {
    sx += __shfl_xor(sx, off);
    sy += __shfl_xor(sy, off);
    sz += __shfl_xor(sz, off);
  }
  if (lane == 0) {
    red[wave][0] = sx; red[wave][1] = sy; red[wave][2] = sz;
  }
  __syncthreads();
  if (threadIdx.x < 3) {
    const int j = threadIdx.x;
    float acc = 0.f;
#pragma unroll
    for (int w = 0; w < kTailWaves; ++w) acc += red[w][j];
    pred_t[b * 3 + j] = acc / (float)n;
  }
}

// TBase conv1 on the gathered concat, split by linearity (krrn.py:132-141, fusion.py:234-238):
// feat[i] = [fm_5[nn2[i]] | feat_1[nn1[i]] | feat_2[nn1[i]]], so W1 . feat[i] =
// P2[nn2[i]] + P1[nn1[i]] with P2 = fm_5 W_a^T on the N/16 level-2 rows and P1 = [feat_1 | feat_2]
// W_bc^T on the N/4 level-1 rows (5.7x fewer MFMA flops than the GEMM over all N points). This
// kernel gathers and adds the two row sets and applies the folded BN, the one-hot column
// (bias2, per crop) and the ReLU: out = act(scale * (A[ia] + B[ib]) + bias + bias2[b]).
template <typename IT>
__global__ void gather2_add_kernel(const int* __restrict__ ia, const float* __restrict__ A, long long a_bs, int a_st,
                                   const int* __restrict__ ib, const float* __restrict__ Bm, long long b_bs,
                                   int b_st, int n, int C4, const float* __restrict__ scale,
                                   const float* __restrict__ bias, const float* __restrict__ bias2, int relu,
                                   float* __restrict__ out, long long o_bs, int o_st, IT total) {
  const IT e = (IT)blockIdx.x * blockDim.x + threadIdx.x;
  if (e >= total) return;
  const int c4 = (int)(e % C4);
  const IT bi = e / C4;
  const int i = (int)(bi % n);
  const int b = (int)(bi / n);
  const int ra = ia[(long long)b * n + i], rb = ib[(long long)b * n + i];
  const f32x4 x = *reinterpret_cast<const f32x4*>(A + b * a_bs + (long long)ra * a_st + 4 * c4) +
                  *reinterpret_cast<const f32x4*>(Bm + b * b_bs + (long long)rb * b_st + 4 * c4);
  f32x4 v = x * *reinterpret_cast<const f32x4*>(scale + 4 * c4) + *reinterpret_cast<const f32x4*>(bias + 4 * c4);
  if (bias2) v += *reinterpret_cast<const f32x4*>(bias2 + (long long)b * 4 * C4 + 4 * c4);
  if (relu) {
    v.x = fmaxf(v.x, 0.f); v.y = fmaxf(v.y, 0.f); v.z = fmaxf(v.z, 0.f); v.w = fmaxf(v.w, 0.f);
  }
  *reinterpret_cast<f32x4*>(out + b * o_bs + (long long)i * o_st + 4 * c4) = v;
}

inline dim3 grid1(long long total) { return dim3((unsigned)((total + 255) / 256)); }

}  // namespace

KRRN_API int krrn_resize_bilinear_f32(const float* in, int B, int Hi, int Wi, int in_cs, int in_co, int C,
                                      float* out, int Ho, int Wo, int out_cs, int out_co, const float* add,
                                      int add_cs, int add_co, int align_corners, int relu, void* stream) {
  if (!in || !out) return KRRN_EARG;
  if (B < 1 || Hi < 1 || Wi < 1 || Ho < 1 || Wo < 1 || C < 1) return KRRN_ESHAPE;
  if ((C & 3) || (in_cs & 3) || (in_co & 3) || (out_cs & 3) || (out_co & 3) || !krrn_aligned16(in) ||
      !krrn_aligned16(out))
    return KRRN_EALIGN;
  if (add && ((add_cs & 3) || (add_co & 3) || !krrn_aligned16(add))) return KRRN_EALIGN;
  float sh, sw;
  if (align_corners) {
    sh = Ho > 1 ? (float)(Hi - 1) / (float)(Ho - 1) : 0.f;
    sw = Wo > 1 ? (float)(Wi - 1) / (float)(Wo - 1) : 0.f;
  } else {
    sh = (float)Hi / (float)Ho;
    sw = (float)Wi / (float)Wo;
  }
  const int Ho2 = (Ho + 1) / 2, Wo2 = (Wo + 1) / 2;
  const long long total2 = (long long)B * Ho2 * Wo2 * (C / 4);
  // the 2x2 form for large upsamples only (the heads' 472 MB ones: 161 -> 118 us); the HRNet
  // fuse layers' small ones want the 4x more threads of the plain kernel (7.6 vs 9.0 us)
  constexpr long long up_min = 1LL << 21;
  if (Ho >= Hi && Wo >= Wi && total2 >= up_min && total2 < 0x7fffffffLL) {
    hipLaunchKernelGGL(resize_up2x2_kernel, grid1(total2), dim3(256), 0, (hipStream_t)stream, in, Hi, Wi, in_cs, in_co,
                       C / 4, out, Ho, Wo, out_cs, out_co, add, add_cs, add_co, sh, sw, align_corners, relu, Ho2, Wo2,
                       (int)total2);
    return krrn_launch_status();
  }
  const long long total = (long long)B * Ho * Wo * (C / 4);
  if (total < 0x7fffffffLL)
    hipLaunchKernelGGL(resize_bilinear_kernel<int>, grid1(total), dim3(256), 0, (hipStream_t)stream, in, Hi, Wi,
                       in_cs, in_co, C / 4, out, Ho, Wo, out_cs, out_co, add, add_cs, add_co, sh, sw, align_corners,
                       relu, (int)total);
  else
    hipLaunchKernelGGL(resize_bilinear_kernel<long long>, grid1(total), dim3(256), 0, (hipStream_t)stream, in, Hi,
                       Wi, in_cs, in_co, C / 4, out, Ho, Wo, out_cs, out_co, add, add_cs, add_co, sh, sw,
                       align_corners, relu, total);
  return krrn_launch_status();
}

KRRN_API int krrn_add_relu_f32(const float* a, int a_cs, int a_co, const float* b, int b_cs, int b_co, float* out,
                               int o_cs, int o_co, long long npix, int C, int relu, void* stream) {
  if (!a || !out) return KRRN_EARG;
  if (npix < 1 || C < 1) return KRRN_ESHAPE;
  if ((C & 3) || (a_cs & 3) || (a_co & 3) || (o_cs & 3) || (o_co & 3) || (b && ((b_cs & 3) || (b_co & 3))))
    return KRRN_EALIGN;
  const long long total = npix * (C / 4);
  if (total < 0x7fffffffLL)
    hipLaunchKernelGGL(add_relu_kernel<int>, grid1(total), dim3(256), 0, (hipStream_t)stream, a, a_cs, a_co, b, b_cs,
                       b_co, out, o_cs, o_co, C / 4, relu, (int)total);
  else
    hipLaunchKernelGGL(add_relu_kernel<long long>, grid1(total), dim3(256), 0, (hipStream_t)stream, a, a_cs, a_co, b,
                       b_cs, b_co, out, o_cs, o_co, C / 4, relu, total);
  return krrn_launch_status();
}

KRRN_API int krrn_nchw_to_nhwc_f32(const float* in, int B, int C, int H, int W, float* out, int o_cs, int o_co,
                                   void* stream) {
  if (!in || !out) return KRRN_EARG;
  if (B < 1 || C < 1 || H < 1 || W < 1 || o_co + C > o_cs) return KRRN_ESHAPE;
  const long long total = (long long)B * C * H * W;
  hipLaunchKernelGGL(nchw_to_nhwc_kernel, grid1(total), dim3(256), 0, (hipStream_t)stream, in, C, H * W, out, o_cs,
                     o_co, total);
  return krrn_launch_status();
}

KRRN_API int krrn_heads_select_f32(const float* fx, int Cx, int xyz_off, const float* fn, int Cn,
                                   const long long* cls, float* xyz_out, float* nml_out, int B, int H, int W,
                                   void* stream) {
  if (!fx || !fn || !cls || !xyz_out || !nml_out) return KRRN_EARG;
  if (B < 1 || H < 1 || W < 1 || Cx < xyz_off + 3 || Cn < 3) return KRRN_ESHAPE;
  const long long total = (long long)B * H * W;
  hipLaunchKernelGGL(heads_select_kernel, grid1(total), dim3(256), 0, (hipStream_t)stream, fx, Cx, xyz_off, fn, Cn,
                     cls, xyz_out, nml_out, H * W, total);
  return krrn_launch_status();
}

KRRN_API int krrn_points_gather_f32(const float* cloud, const float* xyz, const float* nml, const long long* choose,
                                    int B, int N, int H, int W, float* p9, void* stream) {
  if (!cloud || !xyz || !nml || !choose || !p9) return KRRN_EARG;
  if (B < 1 || N < 1 || H < 1 || W < 1) return KRRN_ESHAPE;
  const long long total = (long long)B * N;
  hipLaunchKernelGGL(points_gather_kernel, grid1(total), dim3(256), 0, (hipStream_t)stream, cloud, xyz, nml, choose,
                     N, H * W, p9, total);
  return krrn_launch_status();
}

KRRN_API int krrn_gather_rows_f32(const void* idx, int idx64, long long idx_bs, int nrows, const float* src,
                                  long long src_bs, int src_st, float* dst, long long dst_bs, int dst_st, int width,
                                  int B, void* stream) {
  if (!idx || !src || !dst) return KRRN_EARG;
  if (B < 1 || nrows < 1 || width < 1) return KRRN_ESHAPE;
  const bool vec = !(width & 3) && !(src_st & 3) && !(dst_st & 3) && !(src_bs & 3) && !(dst_bs & 3) &&
                   krrn_aligned16(src) && krrn_aligned16(dst);
  const long long total = (long long)B * nrows * (vec ? width / 4 : width);
  hipStream_t s = (hipStream_t)stream;
#define KRRN_GR(I64, V)                                                                                    \
  hipLaunchKernelGGL((gather_rows_kernel<I64, V>), grid1(total), dim3(256), 0, s, idx, idx_bs, nrows, src, \
                     src_bs, src_st, dst, dst_bs, dst_st, width, total)
  if (idx64) {
    if (vec) KRRN_GR(true, true); else KRRN_GR(true, false);
  } else {
    if (vec) KRRN_GR(false, true); else KRRN_GR(false, false);
  }
#undef KRRN_GR
  return krrn_launch_status();
}

KRRN_API int krrn_tbase_tail_f32(const float* h, int B, int n, int C, const float* w4, const float* b4,
                                 const float* cloud, float* pred_t, float* t_res, void* stream) {
  if (!h || !w4 || !b4 || !cloud || !pred_t) return KRRN_EARG;
  if (B < 1 || n < 1 || C < 1) return KRRN_ESHAPE;
  if ((C & 3) || !krrn_aligned16(h) || !krrn_aligned16(w4)) return KRRN_EALIGN;
  hipLaunchKernelGGL(tbase_tail_kernel, dim3(B), dim3(64 * kTailWaves), 0, (hipStream_t)stream, h, n, C, w4, b4, cloud, pred_t,
                     t_res);
  return krrn_launch_status();
}

KRRN_API int krrn_gather2_add_f32(const int* ia, const float* A, long long a_bs, int a_st, const int* ib, const float* B_,
                                  long long b_bs, int b_st, int n, int C, const float* scale, const float* bias,
                                  const float* bias2, int relu, float* out, long long o_bs, int o_st, int B,
                                  void* stream) {
  if (!ia || !A || !ib || !B_ || !scale || !bias || !out) return KRRN_EARG;
  if (n < 1 || C < 1 || B < 1) return KRRN_ESHAPE;
  if ((C & 3) || (a_st & 3) || (b_st & 3) || (o_st & 3) || (a_bs & 3) || (b_bs & 3) || (o_bs & 3) ||
      !krrn_aligned16(A) || !krrn_aligned16(B_) || !krrn_aligned16(out) || !krrn_aligned16(scale) ||
      !krrn_aligned16(bias) || (bias2 && !krrn_aligned16(bias2)))
    return KRRN_EALIGN;
  const long long total = (long long)B * n * (C / 4);
  if (total < 0x7fffffffLL)
    hipLaunchKernelGGL(gather2_add_kernel<int>, grid1(total), dim3(256), 0, (hipStream_t)stream, ia, A, a_bs, a_st, ib,
                       B_, b_bs, b_st, n, C / 4, scale, bias, bias2, relu, out, o_bs, o_st, (int)total);
  else
    hipLaunchKernelGGL(gather2_add_kernel<long long>, grid1(total), dim3(256), 0, (hipStream_t)stream, ia, A, a_bs,
                       a_st, ib, B_, b_bs, b_st, n, C / 4, scale, bias, bias2, relu, out, o_bs, o_st, total);
  return krrn_launch_status();
}
