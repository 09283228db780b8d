"""Micro-bench of the fusion's level-0 / level-1 kernels at config 2 (B crops x N = 1000 points):
the K = 128 GCN GEMMs (krrn_gemm_panel_x3_f32 per column split, krrn_gemm_x3_f32, hipBLASLt via
torch.mm) and the gather-convs (krrn_gcn_conv_f32: Conv_surface and Conv_layer, level 0 and 1).
Prints one JSON line per measurement (us per launch, GB/s of the launch's compulsory bytes).

usage (GPU box): python3 profiles/bench_fusion_kernels.py
"""
import json
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from pose_estimation_amd import _lib, ops  # noqa: E402
from pose_estimation_amd.runtime import P, ptr  # noqa: E402
from pose_estimation_amd.synthetic import make_batch  # noqa: E402

dev = torch.device("cuda", 0)
B, N = int(os.environ.get("B", 64)), 1000
S, C, K = 7, 128, 10
L = _lib.lib()
st = P(torch.cuda.current_stream().cuda_stream)


def ev_time(fn, reps=30):
    fn()
    torch.cuda.synchronize()
    a, b = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    a.record()
    for _ in range(reps):
        fn()
    b.record()
    torch.cuda.synchronize()
    return a.elapsed_time(b) / reps * 1e3


def emit(**kw):
    print(json.dumps(kw), flush=True)


# ---- K = 128 GEMMs: A = a 128-column slice of [M, 384] rows, out [M, 1024] -------------------
for level, M in ((0, B * N), (1, B * N // 4)):
    g = torch.Generator().manual_seed(level)
    A = torch.randn(M, 384, generator=g).to(dev)
    W = (torch.randn(1024, 128, generator=g) / 128 ** 0.5).to(dev)
    bias = (0.1 * torch.randn(1024, generator=g)).to(dev)
    out = torch.empty(M, 1024, device=dev)
    byts = 4.0 * (M * 128 + M * 1024)
    wp = ops.gemm_weights_panel(W)
    ref = A[:, 128:256].double() @ W.double().t() + bias.double()
    for cs in (1, 2, 4, 8):
        def run(cs=cs):
            _lib.check(L.krrn_gemm_panel_x3_f32(P(A.data_ptr() + 512), 384, M, 128, 1024, ptr(wp), ptr(bias), P(0), 0,
                                                ptr(out), 1024, 0, cs, st), "panel")
        us = ev_time(run)
        err = float((out.double() - ref).abs().max())
        emit(kernel="gemm_panel_x3", level=level, M=M, csplit=cs, us=round(us, 2),
             GBs=round(byts / us / 1e3, 1), TFs=round(2.0 * M * 128 * 1024 / us / 1e6, 1), max_err=err)
    w3 = ops.gemm_weights_x3(W)

    def run_x3():
        _lib.check(L.krrn_gemm_x3_f32(P(A.data_ptr() + 512), 384, M, 128, 1024, ptr(w3), ptr(bias), P(0), 0, ptr(out),
                                      1024, 0, 1, 0, 0, 0, st), "x3")
    us = ev_time(run_x3)
    emit(kernel="gemm_x3", level=level, M=M, us=round(us, 2), GBs=round(byts / us / 1e3, 1))
    Aw = A[:, 128:256]
    us = ev_time(lambda: torch.addmm(bias, Aw, W.t(), out=out))
    emit(kernel="hipblaslt(torch.addmm)", level=level, M=M, us=round(us, 2), GBs=round(byts / us / 1e3, 1))

# ---- gather-convs -----------------------------------------------------------------------------
cloud = make_batch(B, 120, N, seed=1)["cloud"]
for level, n in ((0, N), (1, N // 4)):
    g = torch.Generator().manual_seed(level)
    pts = cloud if level == 0 else torch.stack([c[torch.randperm(N, generator=g)[:n]] for c in cloud])
    v = torch.zeros(B, n, 9)
    v[..., :3] = pts
    v[..., 3:] = torch.randn(B, n, 6, generator=g)
    vd = v.to(dev)
    idx = torch.empty(B, n, K, dtype=torch.int32, device=dev)
    _lib.check(L.krrn_knn_f32(ptr(vd), n * 9, 9, n, P(0), ptr(vd), n * 9, 9, n, 3, K, 1, 0, B, ptr(idx), st), "knn")
    dn = torch.randn(3, S * C, generator=g)
    dn = (dn / dn.norm(dim=0, keepdim=True)).to(dev)
    Y = torch.randn(B, n, (S + 1) * C, generator=g).to(dev)
    bs, bb = torch.ones(C, device=dev), torch.zeros(C, device=dev)
    out = torch.empty(B, n, C, device=dev)
    for has_y in (False, True):
        def run(has_y=has_y):
            _lib.check(L.krrn_gcn_conv_f32(ptr(idx), n, K, ptr(vd), n * 9, 9, 3, ptr(dn), S, C,
                                           ptr(Y) if has_y else P(0), ptr(bs) if has_y else P(0),
                                           ptr(bb) if has_y else P(0), 1, ptr(out), n * C, C, B, st), "gcn")
        us = ev_time(run)
        byts = 4.0 * B * n * (C + ((S + 1) * C if has_y else 0))
        emit(kernel="gcn_conv", level=level, has_y=has_y,
             us=round(us, 2), GBs=round(byts / us / 1e3, 1))
