// Farthest point sampling (tools/script/sample_model.py:35-48, the offline
// sampler of the 64 FPS region centres KRRN's region head is trained against,
// batchdataset.py:723-728): start at point 0; repeatedly take the point whose distance to the
// selected set is largest (np.argmax: the lowest index among ties), with the distance evaluated
// exactly as numpy does (f32 diff, squares summed left to right, sqrt; no FMA contraction).
//
// One workgroup per point set: the running distance-to-set lives in registers (up to kFpsPer
// points per thread), each step is a register update plus one block-wide (max, lowest index)
// reduction through wave shuffles and LDS.
#include <math.h>

#include "krrn_common.h"

namespace {

constexpr int kFpsThreads = 1024;
constexpr int kFpsPer = 16;  // points per thread -> n <= 16384

__device__ __forceinline__ void argmax_merge(float& v, int& i, float v2, int i2) {
  if (v2 > v || (v2 == v && i2 < i)) {
    v = v2;
    i = i2;
  }
}

__global__ __launch_bounds__(kFpsThreads) void fps_kernel(const float* __restrict__ pts, int n, int ns,
                                                           int* __restrict__ out) {
#pragma clang fp contract(off)
  __shared__ float wv[kFpsThreads / 64];
  __shared__ int wi[kFpsThreads / 64];
  __shared__ int cur;
  const int b = blockIdx.x;
  const float* P = pts + (size_t)b * n * 3;
  const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
  float px[kFpsPer], py[kFpsPer], pz[kFpsPer], d[kFpsPer];
#pragma unroll
  for (int k = 0; k < kFpsPer; ++k) {
    const int j = tid + k * kFpsThreads;
    const bool ok = j < n;
    px[k] = ok ? P[3 * j] : 0.f;
    py[k] = ok ? P[3 * j + 1] : 0.f;
    pz[k] = ok ? P[3 * j + 2] : 0.f;
    d[k] = ok ? INFINITY : -INFINITY;  // dist_to_set starts as dist to point 0, min'd below
  }
  int sel = 0;
  for (int s = 0; s < ns; ++s) {
    if (tid == 0) out[(size_t)b * ns + s] = sel;
    const float sx = P[3 * sel], sy = P[3 * sel + 1], sz = P[3 * sel + 2];
    float bv = -INFINITY;
    int bi = 0x7fffffff;
#pragma unroll
    for (int k = 0; k < kFpsPer; ++k) {
      const int j = tid + k * kFpsThreads;
      if (j < n) {
        const float dx = px[k] - sx, dy = py[k] - sy, dz = pz[k] - sz;
        const float dd = sqrtf(dx * dx + dy * dy + dz * dz);
        d[k] = fminf(d[k], dd);
        argmax_merge(bv, bi, d[k], j);
      }
    }
#pragma unroll
    for (int off = 32; off > 0; off >>= 1) {
      const float v2 = __shfl_xor(bv, off);
      const int i2 = __shfl_xor(bi, off);
      argmax_merge(bv, bi, v2, i2);
    }
    if (lane == 0) {
      wv[wave] = bv;
      wi[wave] = bi;
    }
    __syncthreads();
    if (tid == 0) {
      float v = wv[0];
      int i = wi[0];
      for (int w = 1; w < kFpsThreads / 64; ++w) argmax_merge(v, i, wv[w], wi[w]);
      cur = i;
    }
    __syncthreads();
    sel = cur;
  }
}

}  // namespace

KRRN_API int krrn_fps_f32(const float* pts, int B, int n, int n_samples, int* out_idx, void* stream) {
  if (!pts || !out_idx) return KRRN_EARG;
  if (B < 1 || n < 1 || n > kFpsThreads * kFpsPer || n_samples < 1) return KRRN_ESHAPE;
  hipLaunchKernelGGL(fps_kernel, dim3(B), dim3(kFpsThreads), 0, (hipStream_t)stream, pts, n, n_samples, out_idx);
  return krrn_launch_status();
}
