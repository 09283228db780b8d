// Counter-based randomness for the sampling steps of the KRRN eval path, on the device so a
// whole forward can be replayed from a hipGraph:
//   krrn_randperm_i32     torch.randperm(n)[:k] (Pool_layer, gcn3d.py:239; get_pose's
//                         choose subset, trainer.py:406-408): random 32-bit keys sorted
//                         (key, index) in LDS by a bitonic network, first k indices kept.
//   krrn_ransac_subsets   5 distinct correspondence indices per RANSAC hypothesis
//                         (cv::RANSACPointSetRegistrator::getSubset semantics: uniform,
//                         duplicates rejected).
//   krrn_rng_advance      seed += 1 (last node of a replayed step).
// The 64-bit seed lives in device memory; `stream` separates independent draws.
#include "krrn_common.h"

namespace {

__device__ __forceinline__ unsigned long long mix64(unsigned long long z) {
  z += 0x9E3779B97F4A7C15ull;
  z = (z ^ (z >> 30)) * 0xBF58476D1CE4E5B9ull;
  z = (z ^ (z >> 27)) * 0x94D049BB133111EBull;
  return z ^ (z >> 31);
}

__device__ __forceinline__ unsigned int rand32(unsigned long long seed, unsigned int stream, unsigned int row,
                                               unsigned int i) {
  const unsigned long long a = mix64(seed ^ (0xD1B54A32D192ED03ull * (stream + 1)));
  const unsigned long long b = mix64(a + 0x632BE59BD9B4E019ull * (row + 1));
  return (unsigned int)(mix64(b + i) >> 32);
}

constexpr int kPermMax = 4096;

__device__ __forceinline__ void randperm_row(unsigned long long* keys, unsigned long long seed, unsigned int stream,
                                             int row, int n, int k, int* __restrict__ out) {
  int np2 = 1;
  while (np2 < n) np2 <<= 1;
  for (int i = threadIdx.x; i < np2; i += blockDim.x) {
    keys[i] = i < n ? (((unsigned long long)rand32(seed, stream, row, i) << 32) | (unsigned)i) : ~0ull;
  }
  __syncthreads();
  for (int size = 2; size <= np2; size <<= 1) {
    for (int stride = size >> 1; stride > 0; stride >>= 1) {
      for (int i = threadIdx.x; i < np2; i += blockDim.x) {
        const int j = i ^ stride;
        if (j > i) {
          const bool up = (i & size) == 0;
          const unsigned long long a = keys[i], bb = keys[j];
          if ((a > bb) == up) { keys[i] = bb; keys[j] = a; }
        }
      }
      __syncthreads();
    }
  }
  for (int i = threadIdx.x; i < k; i += blockDim.x) out[(long long)row * k + i] = (int)(keys[i] & 0xffffffffu);
}

__global__ __launch_bounds__(1024) void randperm_kernel(const unsigned long long* __restrict__ seed_ptr,
                                                        unsigned int stream, int n, int k, int* __restrict__ out) {
  __shared__ unsigned long long keys[kPermMax];
  randperm_row(keys, *seed_ptr, stream, blockIdx.x, n, k, out);
}

constexpr int kMultiMax = 8;
struct PermDraws {
  unsigned int stream[kMultiMax];
  int n[kMultiMax], k[kMultiMax];
  int* out[kMultiMax];
};

__global__ __launch_bounds__(1024) void randperm_multi_kernel(const unsigned long long* __restrict__ seed_ptr,
                                                              const PermDraws d) {
  __shared__ unsigned long long keys[kPermMax];
  const int q = blockIdx.x;
  randperm_row(keys, *seed_ptr, d.stream[q], 0, d.n[q], d.k[q], d.out[q]);
}

__global__ void subsets_kernel(const unsigned long long* __restrict__ seed_ptr, unsigned int stream, int H, int P,
                               int total, int* __restrict__ out) {
  const int e = blockIdx.x * blockDim.x + threadIdx.x;
  if (e >= total) return;
  const unsigned long long seed = *seed_ptr;
  int ids[5];
  unsigned int ctr = 0;
  for (int s = 0; s < 5; ++s) {
    for (;;) {
      const int x = (int)(((unsigned long long)rand32(seed, stream, (unsigned)e, ctr++) * (unsigned)P) >> 32);
      bool dup = false;
      for (int q = 0; q < s; ++q) dup |= ids[q] == x;
      if (!dup || ctr > 4096) { ids[s] = x; break; }
    }
  }
  for (int s = 0; s < 5; ++s) out[(long long)e * 5 + s] = ids[s];
}

__global__ void advance_kernel(unsigned long long* seed_ptr) { *seed_ptr += 1ull; }

}  // namespace

KRRN_API int krrn_randperm_i32(const unsigned long long* seed_ptr, unsigned int stream, int n, int k, int rows,
                               int* out, void* hstream) {
  if (!seed_ptr || !out) return KRRN_EARG;
  if (n < 1 || n > kPermMax || k < 1 || k > n || rows < 1) return KRRN_ESHAPE;
  hipLaunchKernelGGL(randperm_kernel, dim3(rows), dim3(1024), 0, (hipStream_t)hstream, seed_ptr, stream, n, k, out);
  return krrn_launch_status();
}

KRRN_API int krrn_randperm_multi_i32(const unsigned long long* seed_ptr, int count, const unsigned int* stream_id,
                                     const int* n, const int* k, int* const* out, void* hstream) {
  if (!seed_ptr || !stream_id || !n || !k || !out) return KRRN_EARG;
  if (count < 1 || count > kMultiMax) return KRRN_ESHAPE;
  PermDraws d;
  for (int q = 0; q < count; ++q) {
    if (!out[q]) return KRRN_EARG;
    if (n[q] < 1 || n[q] > kPermMax || k[q] < 1 || k[q] > n[q]) return KRRN_ESHAPE;
    d.stream[q] = stream_id[q]; d.n[q] = n[q]; d.k[q] = k[q]; d.out[q] = out[q];
  }
  hipLaunchKernelGGL(randperm_multi_kernel, dim3(count), dim3(1024), 0, (hipStream_t)hstream, seed_ptr, d);
  return krrn_launch_status();
}

KRRN_API int krrn_ransac_subsets(const unsigned long long* seed_ptr, unsigned int stream, int B, int H, int P,
                                 int* out, void* hstream) {
  if (!seed_ptr || !out) return KRRN_EARG;
  if (B < 1 || H < 1 || P < 5) return KRRN_ESHAPE;
  const int total = B * H;
  hipLaunchKernelGGL(subsets_kernel, dim3((total + 255) / 256), dim3(256), 0, (hipStream_t)hstream, seed_ptr, stream,
                     H, P, total, out);
  return krrn_launch_status();
}

KRRN_API int krrn_rng_advance(unsigned long long* seed_ptr, void* hstream) {
  if (!seed_ptr) return KRRN_EARG;
  hipLaunchKernelGGL(advance_kernel, dim3(1), dim3(1), 0, (hipStream_t)hstream, seed_ptr);
  return krrn_launch_status();
}
