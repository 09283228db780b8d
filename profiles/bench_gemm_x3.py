"""Micro-bench: krrn_gemm_x3_f32 alone on one GEMM shape (for rocprofv3 --pmc passes).
usage: python3 profiles/bench_gemm_x3.py [M K N] (default: TBase conv2, 64000 x 1024 -> 256)"""
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from pose_estimation_amd import _lib, ops  # noqa: E402
from pose_estimation_amd.runtime import P, ptr  # noqa: E402

M, K, N = (int(v) for v in sys.argv[1:4]) if len(sys.argv) > 3 else (64000, 1024, 256)
dev = torch.device("cuda", 0)
g = torch.Generator().manual_seed(0)
A = torch.randn(M, K, generator=g).to(dev)
W = (torch.randn(N, K, generator=g) / K ** 0.5).to(dev)
w3 = ops.gemm_weights_x3(W)
out = torch.empty(M, N, device=dev)
st = P(torch.cuda.current_stream().cuda_stream)
fn = lambda: _lib.check(_lib.lib().krrn_gemm_x3_f32(ptr(A), K, M, K, N, ptr(w3), P(0), P(0), 0, ptr(out), N, 0, 1,  # noqa: E731
                                                    0, 0, 0, st), "gemm_x3")
fn()
torch.cuda.synchronize()
a, b = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
a.record()
for _ in range(20):
    fn()
b.record()
torch.cuda.synchronize()
ms = a.elapsed_time(b) / 20
print(f"gemm_x3 M{M} K{K} N{N}: {ms * 1e3:.1f} us, {2.0 * M * N * K / ms / 1e9:.0f} TFLOP/s f32-equivalent")
