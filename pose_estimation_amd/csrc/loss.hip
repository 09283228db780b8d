// Eval-time losses of the KRRN path: KRRNLoss (lib/network/loss.py:44-85)
// is still evaluated at test time (tools/trainer.py:476), so its four dense map losses and the
// ADD(-S) pose loss run here instead of as a chain of torch ops over [B, C, H, W] maps.
//
//   MapLoss(fn) (lib/network/loss_utils.py:49-70): per pixel fn(x, t), pixels whose target is
//     all-zero over dim 1 (for the label maps: label == 0) excluded, sum / count of valid pixels;
//     fn = l1 (xyz, loss_utils.py:12-13), 1 - cosine (normals, :8-10, torch's CosineSimilarity:
//     each vector divided by max(|v|, 1e-6), then the dot product), cross_entropy (region, mask:
//     -log(softmax(x)[label] + 1e-6), :15-17).
//   PoseLoss (loss.py:19-42): model_points @ R^T + t, for symmetric classes each predicted point
//     matched to its nearest target point (the KeOps argkmin of train.py:126: squared distance,
//     ties -> lower index), mean |pred - target| per crop, mean over the batch.
//
// Memory-bound: one pass over the maps (each pixel's R + M logits read once, the softmax done in
// registers), f64 per-block partial sums reduced in a fixed order by a second one-block kernel,
// so results are bit-reproducible run to run (no atomics).
#include <math.h>

#include "krrn_common.h"

namespace {

constexpr int kLossThreads = 256;
constexpr int kLossPixPerBlock = 4096;  // pixels of one crop per block

__device__ __forceinline__ double block_sum(double v, double* red) {
#pragma unroll
  for (int off = 32; off > 0; off >>= 1) v += __shfl_xor(v, off);
  const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
  __syncthreads();
  if (lane == 0) red[wave] = v;
  __syncthreads();
  double s = 0.0;
  for (int w = 0; w < kLossThreads / 64; ++w) s += red[w];
  return s;
}

// -log(softmax(x)[label] + 1e-6) over the C channels of one pixel (stride HW), torch's
// max-subtracted softmax in f32
__device__ __forceinline__ float ce_pixel(const float* x, int C, int HW, int label) {
  float mx = x[0];
  for (int c = 1; c < C; ++c) mx = fmaxf(mx, x[(size_t)c * HW]);
  float s = 0.f, el = 0.f;
  for (int c = 0; c < C; ++c) {
    const float e = expf(x[(size_t)c * HW] - mx);
    s += e;
    if (c == label) el = e;
  }
  return -logf(el / s + 1e-6f);
}

__global__ __launch_bounds__(kLossThreads) void map_losses_kernel(
    const float* __restrict__ xyz, const float* __restrict__ xyz_gt, const float* __restrict__ nml,
    const float* __restrict__ nml_gt, const float* __restrict__ region, int R, const long long* __restrict__ region_gt,
    const float* __restrict__ mask, int M, const long long* __restrict__ mask_gt, int HW, double* __restrict__ part) {
  __shared__ double red[kLossThreads / 64];
  const int b = blockIdx.y;
  const int p0 = blockIdx.x * kLossPixPerBlock;
  const int p1 = min(HW, p0 + kLossPixPerBlock);
  double s[4] = {0.0, 0.0, 0.0, 0.0}, n[4] = {0.0, 0.0, 0.0, 0.0};
  for (int p = p0 + threadIdx.x; p < p1; p += kLossThreads) {
    const size_t o3 = (size_t)b * 3 * HW + p;
    if (xyz) {
      const float t0 = xyz_gt[o3], t1 = xyz_gt[o3 + HW], t2 = xyz_gt[o3 + 2 * HW];
      if (t0 != 0.f || t1 != 0.f || t2 != 0.f) {
        const float l = fabsf(xyz[o3] - t0) + fabsf(xyz[o3 + HW] - t1) + fabsf(xyz[o3 + 2 * HW] - t2);
        s[0] += l;
        n[0] += 1.0;
      }
    }
    if (nml) {
      const float t0 = nml_gt[o3], t1 = nml_gt[o3 + HW], t2 = nml_gt[o3 + 2 * HW];
      if (t0 != 0.f || t1 != 0.f || t2 != 0.f) {
        const float x0 = nml[o3], x1 = nml[o3 + HW], x2 = nml[o3 + 2 * HW];
        const float nx = fmaxf(sqrtf(x0 * x0 + x1 * x1 + x2 * x2), 1e-6f);
        const float nt = fmaxf(sqrtf(t0 * t0 + t1 * t1 + t2 * t2), 1e-6f);
        const float cs = (x0 / nx) * (t0 / nt) + (x1 / nx) * (t1 / nt) + (x2 / nx) * (t2 / nt);
        s[1] += 1.f - cs;
        n[1] += 1.0;
      }
    }
    if (region) {
      const long long lab = region_gt[(size_t)b * HW + p];
      if (lab != 0 && lab >= 0 && lab < R) {
        s[2] += ce_pixel(region + (size_t)b * R * HW + p, R, HW, (int)lab);
        n[2] += 1.0;
      }
    }
    if (mask) {
      const long long lab = mask_gt[(size_t)b * HW + p];
      if (lab != 0 && lab >= 0 && lab < M) {
        s[3] += ce_pixel(mask + (size_t)b * M * HW + p, M, HW, (int)lab);
        n[3] += 1.0;
      }
    }
  }
  double* out = part + ((size_t)blockIdx.y * gridDim.x + blockIdx.x) * 8;
#pragma unroll
  for (int k = 0; k < 4; ++k) {
    const double ss = block_sum(s[k], red);
    const double nn = block_sum(n[k], red);
    if (threadIdx.x == 0) {
      out[k] = ss;
      out[4 + k] = nn;
    }
  }
}

// sums of nparts partial records [nparts][8] in index order -> out[0..3] = sum/count
// (0 when a map has no valid pixel), out[4..7] = the valid-pixel counts
__global__ __launch_bounds__(kLossThreads) void map_losses_final_kernel(const double* __restrict__ part, int nparts,
                                                                      double* __restrict__ out) {
  __shared__ double red[kLossThreads / 64];
  __shared__ double tot[8];
  for (int k = 0; k < 8; ++k) {
    double v = 0.0;
    // fixed assignment of partials to lanes and a fixed tree: reproducible
    for (int i = threadIdx.x; i < nparts; i += kLossThreads) v += part[(size_t)i * 8 + k];
    const double t = block_sum(v, red);
    if (threadIdx.x == 0) tot[k] = t;
  }
  __syncthreads();
  if (threadIdx.x < 4) {
    const double c = tot[4 + threadIdx.x];
    out[threadIdx.x] = c > 0.0 ? tot[threadIdx.x] / c : 0.0;
    out[4 + threadIdx.x] = c;
  }
}

// per-crop means: block b sums crop b's partial records [nbx][8] in index order -> out[b][0..3]
// = sum / count (0 without a valid pixel), out[b][4..7] = counts. trainer.py:180-182 adds each
// crop's own loss (batch size 1) to its object's running sums.
__global__ __launch_bounds__(kLossThreads) void map_losses_crop_kernel(const double* __restrict__ part, int nbx,
                                                                     double* __restrict__ out) {
  __shared__ double red[kLossThreads / 64];
  __shared__ double tot[8];
  const double* pb = part + (size_t)blockIdx.x * nbx * 8;
  for (int k = 0; k < 8; ++k) {
    double v = 0.0;
    for (int i = threadIdx.x; i < nbx; i += kLossThreads) v += pb[(size_t)i * 8 + k];
    const double t = block_sum(v, red);
    if (threadIdx.x == 0) tot[k] = t;
  }
  __syncthreads();
  if (threadIdx.x < 4) {
    const double c = tot[4 + threadIdx.x];
    out[(size_t)blockIdx.x * 8 + threadIdx.x] = c > 0.0 ? tot[threadIdx.x] / c : 0.0;
    out[(size_t)blockIdx.x * 8 + 4 + threadIdx.x] = c;
  }
}

// PoseLoss: grid (ceil(P / 256), B); targets of crop b staged through LDS in tiles for the
// nearest-point search of symmetric classes
constexpr int kPoseTile = 2048;

__global__ __launch_bounds__(kLossThreads) void pose_loss_kernel(const float* __restrict__ R, const float* __restrict__ t,
                                                                 const float* __restrict__ target,
                                                                 const float* __restrict__ mp,
                                                                 const long long* __restrict__ cls,
                                                                 const int* __restrict__ sym, int nsym, int P,
                                                                 double* __restrict__ part) {
  __shared__ float tl[kPoseTile * 3];
  __shared__ double red[kLossThreads / 64];
  const int b = blockIdx.y;
  const int i = blockIdx.x * kLossThreads + threadIdx.x;
  const float* Rb = R + (size_t)b * 9;
  const float* tb = t + (size_t)b * 3;
  const float* tg = target + (size_t)b * P * 3;
  bool is_sym = false;
  const long long c = cls[b];
  for (int k = 0; k < nsym; ++k) is_sym |= (long long)sym[k] == c;
  float px = 0.f, py = 0.f, pz = 0.f;
  if (i < P) {
    const float* m = mp + ((size_t)b * P + i) * 3;
    // torch matmul [P,3] @ [3,3]^T then + t: k-ordered sums
    px = m[0] * Rb[0] + m[1] * Rb[1] + m[2] * Rb[2] + tb[0];
    py = m[0] * Rb[3] + m[1] * Rb[4] + m[2] * Rb[5] + tb[1];
    pz = m[0] * Rb[6] + m[1] * Rb[7] + m[2] * Rb[8] + tb[2];
  }
  int sel = i;
  if (is_sym) {  // block-uniform
    float best = INFINITY;
    int bi = 0;
    for (int j0 = 0; j0 < P; j0 += kPoseTile) {
      const int nj = min(kPoseTile, P - j0);
      __syncthreads();
      for (int e = threadIdx.x; e < nj * 3; e += kLossThreads) tl[e] = tg[(size_t)j0 * 3 + e];
      __syncthreads();
      if (i < P) {
        for (int j = 0; j < nj; ++j) {
          const float dx = px - tl[3 * j], dy = py - tl[3 * j + 1], dz = pz - tl[3 * j + 2];
          const float d = dx * dx + dy * dy + dz * dz;
          if (d < best) {
            best = d;
            bi = j0 + j;
          }
        }
      }
    }
    sel = bi;
  }
  double v = 0.0;
  if (i < P) {
    const float* q = tg + (size_t)sel * 3;
    const float dx = px - q[0], dy = py - q[1], dz = pz - q[2];
    v = sqrtf(dx * dx + dy * dy + dz * dz);
  }
  const double s = block_sum(v, red);
  if (threadIdx.x == 0) part[(size_t)b * gridDim.x + blockIdx.x] = s;
}

__global__ __launch_bounds__(kLossThreads) void pose_loss_final_kernel(const double* __restrict__ part, int nblk,
                                                                      int B, int P, double* __restrict__ out) {
  __shared__ double red[kLossThreads / 64];
  double v = 0.0;
  for (int b = threadIdx.x; b < B; b += kLossThreads) {
    double s = 0.0;
    for (int k = 0; k < nblk; ++k) s += part[(size_t)b * nblk + k];
    v += s / (double)P;
  }
  const double t = block_sum(v, red);
  if (threadIdx.x == 0) out[0] = t / (double)B;
}

// ADD / ADD-S per crop (Metric.cal_adds_cuda, lib/utils/metric.py:17-35, as Trainer.cal_dis calls
// it, tools/trainer.py:370-381): pred = model_points @ R^T + t; ADD = mean_i |pred_i - target_i|;
// for a symmetric class ADD-S = mean over targets i of min over preds j |pred_j - target_i| (the
// reference's [N, N, 3] broadcast, norm over dim 2, min over dim 1). grid (ceil(P / 256), B):
// one target per thread, the crop's predicted points rebuilt into LDS tile by tile; the min is
// taken over exact direct-difference squared norms (no expanded-distance shortcut), then sqrt.
__global__ __launch_bounds__(kLossThreads) void add_metric_kernel(const float* __restrict__ R, const float* __restrict__ t,
                                                                  const float* __restrict__ mp,
                                                                  const float* __restrict__ target,
                                                                  const long long* __restrict__ cls,
                                                                  const int* __restrict__ sym, int nsym, int P,
                                                                  double* __restrict__ part) {
  __shared__ float pl[kPoseTile * 3];
  __shared__ double red[kLossThreads / 64];
  const int b = blockIdx.y;
  const int i = blockIdx.x * kLossThreads + threadIdx.x;
  const float* Rb = R + (size_t)b * 9;
  const float* tb = t + (size_t)b * 3;
  const float* mb = mp + (size_t)b * P * 3;
  const float* tg = target + (size_t)b * P * 3;
  bool is_sym = false;
  const long long c = cls[b];
  for (int k = 0; k < nsym; ++k) is_sym |= (long long)sym[k] == c;
  float qx = 0.f, qy = 0.f, qz = 0.f;
  if (i < P) {
    qx = tg[(size_t)i * 3];
    qy = tg[(size_t)i * 3 + 1];
    qz = tg[(size_t)i * 3 + 2];
  }
  double v = 0.0;
  if (!is_sym) {  // block-uniform
    if (i < P) {
      const float* m = mb + (size_t)i * 3;
      const float px = m[0] * Rb[0] + m[1] * Rb[1] + m[2] * Rb[2] + tb[0];
      const float py = m[0] * Rb[3] + m[1] * Rb[4] + m[2] * Rb[5] + tb[1];
      const float pz = m[0] * Rb[6] + m[1] * Rb[7] + m[2] * Rb[8] + tb[2];
      const float dx = px - qx, dy = py - qy, dz = pz - qz;
      v = sqrtf(dx * dx + dy * dy + dz * dz);
    }
  } else {
    float best = INFINITY;
    for (int j0 = 0; j0 < P; j0 += kPoseTile) {
      const int nj = min(kPoseTile, P - j0);
      __syncthreads();
      for (int e = threadIdx.x; e < nj; e += kLossThreads) {
        const float* m = mb + (size_t)(j0 + e) * 3;
        pl[3 * e] = m[0] * Rb[0] + m[1] * Rb[1] + m[2] * Rb[2] + tb[0];
        pl[3 * e + 1] = m[0] * Rb[3] + m[1] * Rb[4] + m[2] * Rb[5] + tb[1];
        pl[3 * e + 2] = m[0] * Rb[6] + m[1] * Rb[7] + m[2] * Rb[8] + tb[2];
      }
      __syncthreads();
      if (i < P) {
        for (int j = 0; j < nj; ++j) {
          const float dx = pl[3 * j] - qx, dy = pl[3 * j + 1] - qy, dz = pl[3 * j + 2] - qz;
          best = fminf(best, dx * dx + dy * dy + dz * dz);
        }
      }
    }
    if (i < P) v = sqrtf(best);
  }
  const double s = block_sum(v, red);
  if (threadIdx.x == 0) part[(size_t)b * gridDim.x + blockIdx.x] = s;
}

// per crop: fixed-order sum of its nblk partials / P
__global__ __launch_bounds__(kLossThreads) void add_metric_final_kernel(const double* __restrict__ part, int nblk,
                                                                       int B, int P, double* __restrict__ out) {
  const int b = blockIdx.x * kLossThreads + threadIdx.x;
  if (b >= B) return;
  double s = 0.0;
  for (int k = 0; k < nblk; ++k) s += part[(size_t)b * nblk + k];
  out[b] = s / (double)P;
}

}  // namespace

KRRN_API int krrn_map_losses_ws(int B, int HW, long long* n_doubles) {
  if (!n_doubles) return KRRN_EARG;
  if (B < 1 || HW < 1) return KRRN_ESHAPE;
  *n_doubles = (long long)B * krrn_cdiv(HW, kLossPixPerBlock) * 8;
  return KRRN_OK;
}

KRRN_API int krrn_map_losses_f32(const float* xyz, const float* xyz_gt, const float* nml, const float* nml_gt,
                                 const float* region, int R, const long long* region_gt, const float* mask, int M,
                                 const long long* mask_gt, int B, int HW, double* ws, double* out, void* stream) {
  if (!ws || !out) return KRRN_EARG;
  if ((xyz && !xyz_gt) || (nml && !nml_gt) || (region && !region_gt) || (mask && !mask_gt)) return KRRN_EARG;
  if (B < 1 || HW < 1 || (region && R < 1) || (mask && M < 1)) return KRRN_ESHAPE;
  const int nbx = krrn_cdiv(HW, kLossPixPerBlock);
  if (B > 65535) return KRRN_ESHAPE;
  hipStream_t s = (hipStream_t)stream;
  hipLaunchKernelGGL(map_losses_kernel, dim3(nbx, B), dim3(kLossThreads), 0, s, xyz, xyz_gt, nml, nml_gt, region, R,
                     region_gt, mask, M, mask_gt, HW, ws);
  hipLaunchKernelGGL(map_losses_final_kernel, dim3(1), dim3(kLossThreads), 0, s, ws, nbx * B, out);
  return krrn_launch_status();
}

KRRN_API int krrn_map_losses_crop_f32(const double* ws, int B, int HW, double* out_crop, void* stream) {
  if (!ws || !out_crop) return KRRN_EARG;
  if (B < 1 || HW < 1) return KRRN_ESHAPE;
  hipLaunchKernelGGL(map_losses_crop_kernel, dim3(B), dim3(kLossThreads), 0, (hipStream_t)stream, ws,
                     krrn_cdiv(HW, kLossPixPerBlock), out_crop);
  return krrn_launch_status();
}

KRRN_API int krrn_pose_loss_ws(int B, int P, long long* n_doubles) {
  if (!n_doubles) return KRRN_EARG;
  if (B < 1 || P < 1) return KRRN_ESHAPE;
  *n_doubles = (long long)B * krrn_cdiv(P, kLossThreads);
  return KRRN_OK;
}

KRRN_API int krrn_pose_loss_f32(const float* target_r, const float* pred_t, const float* target,
                                const float* model_points, const long long* cls_id, const int* sym, int nsym, int B,
                                int P, double* ws, double* out, void* stream) {
  if (!target_r || !pred_t || !target || !model_points || !cls_id || !ws || !out || (nsym > 0 && !sym))
    return KRRN_EARG;
  if (B < 1 || P < 1 || B > 65535 || nsym < 0) return KRRN_ESHAPE;
  const int nbx = krrn_cdiv(P, kLossThreads);
  hipStream_t s = (hipStream_t)stream;
  hipLaunchKernelGGL(pose_loss_kernel, dim3(nbx, B), dim3(kLossThreads), 0, s, target_r, pred_t, target, model_points,
                     cls_id, sym, nsym, P, ws);
  hipLaunchKernelGGL(pose_loss_final_kernel, dim3(1), dim3(kLossThreads), 0, s, ws, nbx, B, P, out);
  return krrn_launch_status();
}

KRRN_API int krrn_add_metric_f32(const float* pred_r, const float* pred_t, const float* model_points,
                                 const float* target, const long long* cls_id, const int* sym, int nsym, int B, int P,
                                 double* ws, double* out, void* stream) {
  if (!pred_r || !pred_t || !model_points || !target || !cls_id || !ws || !out || (nsym > 0 && !sym))
    return KRRN_EARG;
  if (B < 1 || P < 1 || B > 65535 || nsym < 0) return KRRN_ESHAPE;
  const int nbx = krrn_cdiv(P, kLossThreads);
  hipStream_t s = (hipStream_t)stream;
  hipLaunchKernelGGL(add_metric_kernel, dim3(nbx, B), dim3(kLossThreads), 0, s, pred_r, pred_t, model_points, target,
                     cls_id, sym, nsym, P, ws);
  hipLaunchKernelGGL(add_metric_final_kernel, dim3(krrn_cdiv(B, kLossThreads)), dim3(kLossThreads), 0, s, ws, nbx, B,
                     P, out);
  return krrn_launch_status();
}
