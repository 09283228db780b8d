"""Diagnostic: do the fusion's level-0 kernels give the same bits when the three branches run side by
side on three streams (as the plan's graph runs them) as when they run one after another?
Each case: a serial reference, then 20 concurrent repetitions compared bit for bit.

usage (GPU box): python3 profiles/concurrency_kernels.py"""
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from pose_estimation_amd import _lib, ops  # noqa: E402
from pose_estimation_amd.runtime import P, ptr  # noqa: E402
from pose_estimation_amd.synthetic import make_batch  # noqa: E402

dev = torch.device("cuda", 0)
B, N, S, C, K = 4, 1000, 7, 128, 10
L = _lib.lib()
g = torch.Generator().manual_seed(0)
cloud = make_batch(B, 120, N, seed=1)["cloud"]
v = torch.zeros(B, N, 9)
v[..., :3] = cloud
v[..., 3:] = torch.randn(B, N, 6, generator=g)
vd = v.to(dev)
idx = torch.empty(B, N, K, dtype=torch.int32, device=dev)
st0 = P(torch.cuda.current_stream().cuda_stream)
_lib.check(L.krrn_knn_f32(ptr(vd), N * 9, 9, N, P(0), ptr(vd), N * 9, 9, N, 3, K, 1, 0, B, ptr(idx), st0), "knn")
dns = [(lambda d: (d / d.norm(dim=0, keepdim=True)).to(dev))(torch.randn(3, S * C, generator=g)) for _ in range(3)]
Ys = [torch.randn(B * N, (S + 1) * C, generator=g).to(dev) for _ in range(3)]
F0 = torch.zeros(B, N, 384, device=dev)
F1 = torch.zeros(B, N, 384, device=dev)
Ws = [(torch.randn(1024, 128, generator=g) / 128 ** 0.5).to(dev) for _ in range(3)]
wps = [ops.gemm_weights_panel(w) for w in Ws]
bias = [(0.1 * torch.randn(1024, generator=g)).to(dev) for _ in range(3)]
Yout = [torch.zeros(B * N, 1024, device=dev) for _ in range(3)]
A = torch.randn(B * N, 384, generator=g).to(dev)
streams = [torch.cuda.Stream() for _ in range(3)]
torch.cuda.synchronize()


def surface(bi, st):
    _lib.check(L.krrn_gcn_conv_f32(ptr(idx), N, K, P(vd.data_ptr() + 12 * bi), N * 9, 9, 3, ptr(dns[bi]), S, C, P(0),
                                   P(0), P(0), 1, P(F0.data_ptr() + 512 * bi), N * 384, 384, B, st), "surface")


def conv(bi, st):
    _lib.check(L.krrn_gcn_conv_f32(ptr(idx), N, K, P(vd.data_ptr() + 12 * bi), N * 9, 9, 3, ptr(dns[bi]), S, C,
                                   ptr(Ys[bi]), P(0), P(0), 1, P(F1.data_ptr() + 512 * bi), N * 384, 384, B, st), "conv")


def gemm(bi, st):
    _lib.check(L.krrn_gemm_panel_x3_f32(P(A.data_ptr() + 512 * bi), 384, B * N, 128, 1024, ptr(wps[bi]), ptr(bias[bi]),
                                        P(0), 0, ptr(Yout[bi]), 1024, 0, 4, st), "panel")


for name, fn, outs in (("surface", surface, [F0]), ("conv", conv, [F1]), ("panel", gemm, Yout)):
    for o in outs:
        o.zero_()
    for bi in range(3):
        fn(bi, st0)
    torch.cuda.synchronize()
    ref = [o.clone() for o in outs]
    bad = 0
    for rep in range(20):
        for o in outs:
            o.zero_()
        torch.cuda.synchronize()
        for bi, s in enumerate(streams):
            fn(bi, P(s.cuda_stream))
        torch.cuda.synchronize()
        if not all(torch.equal(a, b) for a, b in zip(ref, outs)):
            bad += 1
            d = max(float((a - b).abs().max()) for a, b in zip(ref, outs))
            print(f"  {name} rep {rep}: maxdiff {d:.3e}", flush=True)
    # serial again
    for o in outs:
        o.zero_()
    for bi in range(3):
        fn(bi, st0)
    torch.cuda.synchronize()
    ser_ok = all(torch.equal(a, b) for a, b in zip(ref, outs))
    print(f"{name}: {bad}/20 concurrent repetitions differ; serial repeat equal: {ser_ok}", flush=True)
