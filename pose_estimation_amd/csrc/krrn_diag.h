// Diagnostics-only entry points, compiled into the separate diagnostics build of the library
// (`make -C pose_estimation_amd/csrc diag` -> build/diag/libkrrn_hip_diag.so, -DKRRN_DIAG=1) and
// never into libkrrn_hip.so: the product library keeps no global state.
// Used by profiles/f0_shadow.py through KRRN_HIP_LIB.
#pragma once
#include "../../include/krrn_hip.h"

#ifdef __cplusplus
extern "C" {
#endif

/* Diagnostics: from now on every surface conv (krrn_gcn_conv_f32 with Y == NULL, 3-D, C = 128)
 * writes, per (crop, point, neighbour j), 8 words: the neighbour index, the point's and the
 * neighbour's coordinates as read (f32 bits), the crop; then per block (linear index after the
 * XCD remap) 20 words: digests of the staged directions and of the point directions as the block's
 * LDS holds them before the support loop (4), the XCC id and HW_ID register it ran on (2), the
 * arguments out (2 words), o_bs, o_st, S, relu, dn, v (low words) as the block read them (8), two
 * unused, the same digests after the support loop (4); then per (block, thread, support s < 8)
 * 8 floats: the support's max and the first direction-weight quad as held in registers. Launch i
 * goes into slot i % nslots of `buf` (slot_words u32 each, >= B * n * k * 8 + 20 * nb + 16384 * nb
 * with nb = B * ceil(n / 8) blocks). buf = NULL turns it off; every call resets the launch
 * count. One host mutex per surface-conv launch. */
int krrn_gcn_debug(void* buf, int nslots, long long slot_words);


#ifdef __cplusplus
}
#endif
