// Shared device helpers for the KRRN gfx950 kernels.
//
// Every entry point in this library follows one contract (include/krrn_hip.h):
//   * the caller owns every buffer (device pointers), the library never allocates;
//   * work is enqueued on the caller's hipStream_t, no host synchronisation;
//   * return 0 on success, a negative KRRN_E* code for a shape/argument violation
//     (detected on the host before launch), or the hipError_t of the launch.
#pragma once
#include <hip/hip_runtime.h>
#include <stdint.h>

// the public declarations: every definition below must match them (checked by the compiler)
#include "../../include/krrn_hip.h"

#define KRRN_API extern "C" __attribute__((visibility("default")))

typedef float f32x4 __attribute__((ext_vector_type(4)));
typedef float f32x16 __attribute__((ext_vector_type(16)));

static inline int krrn_launch_status() {
  hipError_t e = hipGetLastError();
  return e == hipSuccess ? KRRN_OK : (int)e;
}

static inline bool krrn_aligned16(const void* p) { return (((uintptr_t)p) & 15u) == 0; }

__host__ __device__ static inline int krrn_cdiv(int a, int b) { return (a + b - 1) / b; }

// Bijective XCD-aware block remap (cdna_hip_programming.md §5 "XCD swizzle must be
// bijective"): consecutive logical tiles land on the same XCD so that tiles that share
// an operand panel hit the same L2.
__device__ __forceinline__ int krrn_xcd_remap(int orig, int nwg) {
  const int nx = 8;
  if (nwg < nx) return orig;
  const int q = nwg / nx, r = nwg % nx;
  const int xcd = orig % nx, slot = orig / nx;
  const int base = (xcd < r) ? xcd * (q + 1) : r * (q + 1) + (xcd - r) * q;
  return base + slot;
}

// PyTorch's upsample_bilinear2d source index (aten/src/ATen/native/UpSample.h,
// area_pixel_compute_source_index) evaluated in f32: the resize kernels (pointwise.hip) and the
// Winograd kernel that upsamples its input while staging it (winograd.hip) share it.
__device__ __forceinline__ void krrn_src_index(int dst, int in_size, float scale, int align, int& i0, int& i1,
                                               float& l0, float& l1) {
  float s;
  if (align) {
    s = scale * (float)dst;
  } else {
    s = scale * ((float)dst + 0.5f) - 0.5f;
    s = s < 0.f ? 0.f : s;
  }
  int i = (int)s;
  i = i > in_size - 1 ? in_size - 1 : i;
  i0 = i;
  i1 = i + ((i < in_size - 1) ? 1 : 0);
  float lam = s - (float)i;
  lam = fminf(fmaxf(lam, 0.f), 1.f);
  l1 = lam;
  l0 = 1.f - lam;
}

// The bilinear blend l_y0 (l_x0 v00 + l_x1 v01) + l_y1 (l_x0 v10 + l_x1 v11) of UpSample.h, every
// operation rounded (no FMA contraction), so every kernel that blends gives bit-identical values.
__device__ __forceinline__ f32x4 krrn_bilerp4(f32x4 v00, f32x4 v01, f32x4 v10, f32x4 v11, float ly0, float ly1,
                                              float lx0, float lx1) {
#pragma clang fp contract(off)
  return ly0 * (lx0 * v00 + lx1 * v01) + ly1 * (lx0 * v10 + lx1 * v11);
}
