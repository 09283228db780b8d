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
